"""Multi-GPU partitioned search: one process per GPU, RCCL over xGMI.

    import torch.distributed as dist
    from stateright_amd import TwoPhaseSys
    from stateright_amd.distributed import Communicator
    dist.init_process_group("nccl")                      # torchrun / torch.distributed.run
    comm = Communicator.from_torch(device=local_rank)
    checker = TwoPhaseSys(11).checker().comm(comm).spawn_bfs().join()   # global counts on every rank

The RCCL communicator is created natively (sr_dist_init); torch.distributed only carries the
128-byte unique id from rank 0 to the others.
"""
import ctypes

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

    def close(self):
        if getattr(self, "handle", None):
            self._lib.sr_dist_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
