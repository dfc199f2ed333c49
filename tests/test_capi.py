"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/stateright_gpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "stateright_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(sr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("sr_gpu_bfs_spawn", "sr_gpu_bfs_join", "sr_gpu_bfs_is_done", "sr_gpu_bfs_state_count",
                 "sr_gpu_bfs_unique_state_count", "sr_gpu_bfs_max_depth", "sr_gpu_bfs_discovery",
                 "sr_gpu_bfs_free"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from stateright_amd import _native
    lib = _native.load()
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} declared in the header but not exported"


def test_python_signatures_match_header():
    from stateright_amd import _native
    bound = {n for n, _, _ in _native.SIGNATURES}
    assert bound == set(declared_functions())


def test_struct_layouts():
    from stateright_amd import _native
    lib = _native.load()
    o = _native.sr_opts()
    lib.sr_opts_init(ctypes.byref(o))
    assert o.struct_size == ctypes.sizeof(_native.sr_opts)


def test_spawn_without_device_fails_loudly():
    from stateright_amd import TwoPhaseSys, CheckerError
    from stateright_amd import _native
    if _native.load().sr_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(CheckerError):
        TwoPhaseSys(3).checker().spawn_bfs()


def test_unsupported_parameters_rejected():
    from stateright_amd import _native
    lib = _native.load()
    if lib.sr_device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    arr = (ctypes.c_int64 * 1)(99)
    assert not lib.sr_gpu_bfs_spawn(_native.SR_MODEL_2PC, arr, 1, None)


def test_paxos_action_codes_match_golden_encoding():
    # The product's Deliver encoder and the test-side restatement agree on the reference path.
    from stateright_amd import Paxos
    from paxos_golden import PAXOS_VALUE_CHOSEN_PATH
    ours = [
        Paxos.deliver(4, 1, "Put", 4, "B"),
        Paxos.deliver(1, 0, "Prepare", (1, 1)),
        Paxos.deliver(0, 1, "Prepared", (1, 1), None),
        Paxos.deliver(1, 2, "Accept", (1, 1), (4, 4, "B")),
        Paxos.deliver(2, 1, "Accepted", (1, 1)),
        Paxos.deliver(1, 4, "PutOk", 4),
        Paxos.deliver(1, 2, "Decided", (1, 1), (4, 4, "B")),
        Paxos.deliver(4, 2, "Get", 8),
    ]
    assert ours == PAXOS_VALUE_CHOSEN_PATH
    with pytest.raises(ValueError):
        Paxos(2, server_count=5)


def test_quotient_table_encoding_selftest():
    # The exact visited set for multi-word states (quotient mode): the key permutation is a
    # bijection (exhaustive up to 18 bits) and slot values decode to their keys (host-side check).
    from stateright_amd import _native
    lib = _native.load()
    assert lib.sr_selftest_tables() == 0, _native.last_error()


def test_selftest_models_self_loops():
    # every self-loop slot the FAST expansion skips really returns the state (host BFS, 2pc N<=7)
    from stateright_amd import _native
    lib = _native.load()
    assert lib.sr_selftest_models() == 0, _native.last_error()


def test_opts_init_sized_writes_only_the_callers_bytes():
    # a binding built against an older, shorter sr_opts: the library must not write past it
    import ctypes as C
    from stateright_amd import _native
    lib = _native.load()
    buf = (C.c_uint8 * 128)(*([0xAB] * 128))
    lib.sr_opts_init_sized(C.cast(buf, C.POINTER(_native.sr_opts)), 24)
    assert int.from_bytes(bytes(buf[0:4]), "little") == 24  # struct_size = what it wrote
    assert bytes(buf[4:24]) == bytes(20)
    assert bytes(buf[24:128]) == bytes([0xAB] * 104)
    full = _native.sr_opts()
    lib.sr_opts_init_sized(C.byref(full), 4096)  # a larger mirror: the library's own size
    assert full.struct_size == C.sizeof(_native.sr_opts)
