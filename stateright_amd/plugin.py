"""GpuModels compiled into their own plugin libraries (include/stateright_gpu_model.hpp).

    from stateright_amd.plugin import Plugin
    puzzle = Plugin("examples/plugins/libsliding_puzzle.so", "sliding_puzzle")
    checker = puzzle.model(1, 4, 2, 3, 5, 8, 6, 7, 0).checker().spawn_bfs().join()

The plugin library exports `sr_plugin_<name>()`; the engine library runs its engine instances
(sr_gpu_bfs_spawn_plugin) behind the same `Checker` surface as the registered models.
"""
import ctypes

from . import _native as N
from .checker import CheckerBuilder


class Plugin:
    def __init__(self, path, name):
        N.load()  # the engine library first: the plugin's runtime symbols bind to the same HIP / RCCL
        self.path, self.name = path, name
        self._lib = ctypes.CDLL(path)
        fn = getattr(self._lib, f"sr_plugin_{name}")
        fn.restype = ctypes.c_void_p
        fn.argtypes = []
        self.handle = fn()
        if not self.handle:
            raise ImportError(f"{path}: sr_plugin_{name}() returned NULL")

    def model(self, *params):
        return PluginModel(self, params)

    def fingerprint(self, params, described):
        """The engine's fingerprint of a state given by its description (plugin's `undescribe`)."""

        class _Raw(ctypes.Structure):
            _fields_ = [("abi", ctypes.c_uint32), ("opts_size", ctypes.c_uint32), ("name", ctypes.c_char_p),
                        ("create", ctypes.c_void_p),
                        ("fingerprint", ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32,
                                                         ctypes.POINTER(ctypes.c_int64), ctypes.c_int32,
                                                         ctypes.POINTER(ctypes.c_uint64)))]
        raw = ctypes.cast(self.handle, ctypes.POINTER(_Raw)).contents
        p = (ctypes.c_int64 * max(1, len(params)))(*params)
        d = (ctypes.c_int64 * max(1, len(described)))(*described)
        out = ctypes.c_uint64()
        st = raw.fingerprint(p, len(params), d, len(described), ctypes.byref(out))
        if st != 0:
            raise ValueError(f"plugin fingerprint failed (status {st})")
        return out.value


class PluginModel:
    MODEL_ID = -1

    def __init__(self, plugin, params):
        self.plugin = plugin
        self._params = [int(x) for x in params]

    def params(self):
        return list(self._params)

    def checker(self):
        return CheckerBuilder(self)


def model_fingerprint(model, described):
    """The engine's fingerprint (sr_model_fingerprint) of a registered model's state, given by its
    canonical description; compare with GpuBfsChecker.discovery_fingerprints."""
    params = list(model.params())
    p = (ctypes.c_int64 * max(1, len(params)))(*params)
    d = (ctypes.c_int64 * max(1, len(described)))(*described)
    out = ctypes.c_uint64()
    st = N.load().sr_model_fingerprint(model.MODEL_ID, p, len(params), d, len(described), ctypes.byref(out))
    if st != 0:
        raise ValueError(f"sr_model_fingerprint: {N.last_error()} (status {st})")
    return out.value
