"""world_size-2 gloo run of the partitioned level loop (CPU restatement of dist.hpp's protocol):
global unique / state counts / depth equal the single-process oracle, and the two visited-set
partitions are disjoint and cover the state space."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from oracle_lib import TWO_PHASE, OracleRun


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out, mode="sync", cmin=8192, head_max=0):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dist_protocol_ref import partitioned_bfs, pipelined_bfs
    out[rank] = partitioned_bfs(n) if mode == "sync" else pipelined_bfs(n, cmin=cmin, head_max=head_max)
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [2, 3, 4])
def test_two_rank_partitioned_protocol(n):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    o = OracleRun(TWO_PHASE, [n])
    for r in range(world):
        unique, state_count, depth, _ = out[r]
        assert (unique, state_count, depth) == (o.unique_state_count, o.state_count, o.max_depth)
    # the partitions are disjoint and together hold every state
    assert sum(out[r][3] for r in range(world)) == o.unique_state_count


@pytest.mark.parametrize("n", [3, 5])
def test_two_rank_pipelined_protocol(n):
    # The pipelined loop: counts equal the oracle's and both ranks planned the same bucket
    # capacity for every level (RCCL would hang on a mismatch).
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out, "pipelined"), nprocs=world, join=True)
    o = OracleRun(TWO_PHASE, [n])
    for r in range(world):
        unique, state_count, depth, _, plan = out[r]
        assert (unique, state_count, depth) == (o.unique_state_count, o.state_count, o.max_depth)
        assert not any(ov for _, _, ov in plan)
    assert out[0][4] == out[1][4]
    assert sum(out[r][3] for r in range(world)) == o.unique_state_count


def test_two_rank_pipelined_overflow_is_collective():
    # Buckets far too small: both ranks see the overflow in the same level (from the rows every
    # rank receives) and stop together.
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), 5, out, "pipelined", 4), nprocs=world, join=True)
    p0, p1 = out[0][4], out[1][4]
    assert p0 == p1 and p0[-1][2]


@pytest.mark.parametrize("head_max", [1, 30, 10**6])
def test_two_rank_pipelined_with_replicated_head(head_max):
    # The replicated head hands over at different levels (10**6: the whole 2pc N=4 space runs
    # replicated); counts equal the oracle's and both ranks plan identically.
    n, world = 4, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out, "pipelined", 8192, head_max), nprocs=world, join=True)
    o = OracleRun(TWO_PHASE, [n])
    for r in range(world):
        unique, state_count, depth, _, plan = out[r]
        assert (unique, state_count, depth) == (o.unique_state_count, o.state_count, o.max_depth)
    assert out[0][4] == out[1][4]
    assert sum(out[r][3] for r in range(world)) == o.unique_state_count
