"""Multi-GPU partitioned search: one process per GPU, RCCL over xGMI.

    # under torchrun / torch.distributed.run (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_PORT set)
    from stateright_amd import TwoPhaseSys
    from stateright_amd.distributed import Communicator
    comm = Communicator.from_env()                       # no torch import, no torch HIP runtime
    checker = TwoPhaseSys(11).checker().comm(comm).spawn_bfs().join()   # global counts on every rank

The RCCL communicator is created natively (sr_dist_init). Its 128-byte unique id travels from
rank 0 to the others either through a file next to the launcher (`from_env`, one node) or through
an initialised torch.distributed group (`from_torch`). `local_group(world)` builds `world` ranks
that are threads of this process (the in-process transport of include/stateright_gpu.h), which
runs the engine's multi-rank code on one GPU. `shm(rank, world, name)` makes the ranks separate
processes of one host with a shared-memory host transport (tests and rehearsals on one GPU).
"""
import ctypes
import os
import tempfile
import time

from . import _native as N
from .checker import CheckerError


class Communicator:
    def __init__(self, rank, world, unique_id, device):
        lib = N.load()
        self._lib = lib
        self.rank, self.world, self.device = rank, world, device
        self.handle = lib.sr_dist_init(rank, world, bytes(unique_id), device)
        if not self.handle:
            raise CheckerError("sr_dist_init")

    @classmethod
    def _wrap(cls, handle, device):
        c = cls.__new__(cls)
        c._lib = N.load()
        c.handle = handle
        c.rank = c._lib.sr_dist_rank(handle)
        c.world = c._lib.sr_dist_world(handle)
        c.device = device
        return c

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(N.SR_DIST_ID_BYTES)
        if N.load().sr_dist_unique_id(buf) != 0:
            raise CheckerError("sr_dist_unique_id")
        return buf.raw

    @classmethod
    def from_torch(cls, device=None):
        """Bootstraps from an initialised torch.distributed process group."""
        import torch.distributed as dist
        rank, world = dist.get_rank(), dist.get_world_size()
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(rank, world, obj[0], rank if device is None else device)

    @classmethod
    def from_env(cls, device=None, timeout=120.0):
        """Bootstraps from the torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_PORT) on
        ONE node without importing torch: rank 0 writes the unique id to a file keyed by the
        launcher (parent pid) and MASTER_PORT; the other ranks poll for it."""
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        key = f"sr_uid_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
        path = os.path.join(tempfile.gettempdir(), key)
        if rank == 0:
            uid = cls.unique_id()
            tmp = path + f".{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(uid)
            os.replace(tmp, path)
        else:
            t0 = time.monotonic()
            while not os.path.exists(path):
                if time.monotonic() - t0 > timeout:
                    raise TimeoutError(f"rank {rank}: no RCCL unique id at {path} after {timeout} s")
                time.sleep(0.01)
            with open(path, "rb") as f:
                uid = f.read()
        c = cls(rank, world, uid, local if device is None else device)
        if rank == 0:
            c._uid_path = path
        return c

    @classmethod
    def local_group(cls, world, devices=None):
        """`world` communicators whose ranks are threads of this process (in-process transport)."""
        lib = N.load()
        handles = (ctypes.c_void_p * world)()
        devs = (ctypes.c_int32 * world)(*(devices or [0] * world))
        if lib.sr_dist_local_group(world, devs, handles) != 0:
            raise CheckerError("sr_dist_local_group")
        return [cls._wrap(handles[r], devs[r]) for r in range(world)]

    @classmethod
    def shm(cls, rank, world, name, device=0, slot_bytes=64 << 20, devices_distinct=False):
        """One rank of `world` PROCESSES of this host whose host-side transport is the POSIX
        shared-memory segment `name` (every rank passes the same name). Its collectives are staged
        host copies; the partitioned levels use the direct exchange through IPC, as under RCCL. It
        runs the one-process-per-GPU code path with all ranks on ONE GPU, where RCCL refuses two
        ranks on one device."""
        lib = N.load()
        h = lib.sr_dist_shm_init(rank, world, name.encode(), device, slot_bytes, 1 if devices_distinct else 0)
        if not h:
            raise CheckerError("sr_dist_shm_init")
        return cls._wrap(h, device)

    def kind(self):
        buf = ctypes.create_string_buffer(16)
        self._lib.sr_dist_kind(self.handle, buf, 16)
        return buf.value.decode()

    def nranks(self):
        """Ranks the transport reports (RCCL: ncclCommCount)."""
        return self._lib.sr_dist_nranks(self.handle)

    def barrier(self):
        """This rank's device work finished, then every rank meets (collective)."""
        if self._lib.sr_dist_barrier(self.handle) != 0:
            raise CheckerError("sr_dist_barrier")

    def allreduce(self, values, op="max"):
        """Element-wise max or min of a list of floats over the ranks (collective)."""
        arr = (ctypes.c_double * len(values))(*values)
        if self._lib.sr_dist_allreduce_f64(self.handle, arr, len(values), {"min": 0, "max": 1}[op]) != 0:
            raise CheckerError("sr_dist_allreduce_f64")
        return list(arr)

    def close(self):
        if getattr(self, "handle", None):
            self._lib.sr_dist_free(self.handle)
            self.handle = None
        path = getattr(self, "_uid_path", None)
        if path:
            try:
                os.remove(path)
            except OSError:
                pass
            self._uid_path = None

    def __del__(self):
        self.close()
