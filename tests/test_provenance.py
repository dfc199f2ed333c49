"""Binary provenance: the engine library carries the digest of the sources it was compiled from
(sr_build_digest), and the loader refuses a library built from other sources.
CPU only: loading the library and reading the digest need no device."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from stateright_amd import _native, build  # noqa: E402


def test_library_digest_matches_sources():
    assert _native.build_digest() == build.source_digest()


def _copy_tree(dst):
    shutil.copytree(os.path.join(ROOT, "stateright_amd"), os.path.join(dst, "stateright_amd"),
                    ignore=shutil.ignore_patterns("build", "__pycache__", "*.o"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))


def _load_in(root, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    env.pop("SR_LIB_PATH", None)
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from stateright_amd import _native\n"
            "try:\n    _native.load(); print('loaded')\n"
            "except _native.StaleLibraryError as e:\n    print('refused:', e)\n") % root
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120).stdout


def test_copied_tree_loads(tmp_path):
    _copy_tree(str(tmp_path))
    assert _load_in(str(tmp_path)).startswith("loaded")


@pytest.mark.parametrize("edited", ["stateright_amd/csrc/kernels.hpp", "include/stateright_gpu.h"])
def test_edited_source_is_refused(tmp_path, edited):
    _copy_tree(str(tmp_path))
    with open(os.path.join(str(tmp_path), edited), "a") as f:
        f.write("\n// an edit the library was not built from\n")
    out = _load_in(str(tmp_path))
    assert out.startswith("refused:"), out
    assert build.source_digest() in out  # the digest the library carries is named
