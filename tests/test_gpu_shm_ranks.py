"""The one-process-per-GPU path (what `bench.py --gpus N` runs on a node) as separate PROCESSES on
one MI355X: two ranks joined by the shared-memory communicator (RCCL refuses two ranks on one
device), each a fresh interpreter started with subprocess (tests/shm_rank_worker.py). The
partitioned levels use the direct exchange across processes (IPC handles of pool buffers, device
flags), its set-up reused over consecutive checks and redone when buffers grow; SR_DIRECT=0 runs
the collective exchange instead. Counts must equal the oracle's on every rank."""
import json
import os
import subprocess
import sys
import uuid

import pytest

from oracle_lib import INCREMENT_LOCK, TWO_PHASE, OracleRun

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run_ranks(checks, world=2, distinct=False, env=None, timeout=240, name=None, stagger=None):
    name = name or f"/sr_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    e = dict(os.environ, **(env or {}))
    procs = []
    for r in (range(world) if stagger is None else reversed(range(world))):  # stagger: rank 0 last
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "shm_rank_worker.py"), str(r), str(world), name,
                                       "1" if distinct else "0", *checks], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=e))
        if stagger is not None:
            import time
            time.sleep(stagger)
    if stagger is not None:
        procs.reverse()
    outs = []
    for p in procs:
        try:
            o, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, err[-2000:]
        outs.append([json.loads(line) for line in o.splitlines() if line.startswith("{")])
    return outs


def expect(spec):
    model, n = spec.split(":")
    if model == "pingpong":
        from actor_golden import PINGPONG, pingpong_params
        o = OracleRun(PINGPONG, pingpong_params(int(n), lossy=True))
    else:
        o = OracleRun(TWO_PHASE if model == "2pc" else INCREMENT_LOCK, [int(n)])
    return o.unique_state_count, o.state_count, o.max_depth, o.discovery_names()


def test_stale_segment_of_a_crashed_run():
    # A crashed run left its segment under this name, full size and marked READY. Rank 1
    # starts first and opens it; rank 0 starts later, replaces it with a fresh one, and the attach
    # handshake brings rank 1 over to the live segment: the ranks meet and count right.
    import struct
    name = f"/sr_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    slot_bytes, world = 32 << 20, 2
    path = "/dev/shm" + name
    with open(path, "wb") as f:
        f.truncate(4096 + slot_bytes * world)
        f.seek(20)
        f.write(struct.pack("<I", 0x53524844))  # READY
    try:
        outs = run_ranks(["2pc:5"], env={"SR_HEAD_MAX": "0"}, name=name, stagger=3.0)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    for rank_out in outs:
        assert [(r["unique"], r["states"], r["depth"], r["discoveries"]) for r in rank_out] == [expect("2pc:5")]


@pytest.mark.parametrize("direct", ["1", "0"], ids=["direct", "collective"])
def test_processes_match_oracle(direct):
    # consecutive checks on the same ranks: the direct exchange's set-up is reused (2pc 5 twice),
    # grows with a larger check (2pc 7, increment_lock 7) and is reused again; ping-pong's
    # `eventually` properties across processes (one more word per record)
    checks = ["2pc:5", "2pc:5", "2pc:7", "inclock:7", "2pc:5", "pingpong:5"]
    outs = run_ranks(checks, env={"SR_DIRECT": direct, "SR_HEAD_MAX": "0"})
    for rank_out in outs:
        assert [r["check"] for r in rank_out] == checks
        for r in rank_out:
            assert (r["unique"], r["states"], r["depth"], r["discoveries"]) == expect(r["check"])
            assert r["pipelined"] == (2 if direct == "1" else 1)


def test_processes_corrupt_slot_falls_back():
    # A received record flipped AFTER its source checksummed it (rank 0's owner slots, level 2): the
    # owner's insert reports it, every rank votes, and the check is redone on the collective
    # exchange with the oracle's counts. The communicator keeps the collective exchange afterwards.
    checks = ["2pc:6", "2pc:5"]
    outs = run_ranks(checks, env={"SR_HEAD_MAX": "0", "SR_DX_CORRUPT_LEVEL": "2"})
    for rank_out in outs:
        first, second = rank_out
        for r in rank_out:
            assert (r["unique"], r["states"], r["depth"], r["discoveries"]) == expect(r["check"])
        assert first["exchange_fallbacks"] == 1 and first["pipelined"] == 1
        assert second["exchange_fallbacks"] == 0 and second["pipelined"] == 1


def test_processes_bench_config_with_head():
    # the bench's configuration (2pc N=9, replicated head, then partitioned levels), twice
    n = 9
    outs = run_ranks(["2pc:9", "2pc:9"])
    for rank_out in outs:
        for r in rank_out:
            assert r["unique"] == 6 ** n + 4 ** n + 2 ** n and r["depth"] == 3 * n + 1
            assert r["pipelined"] == 2 and r["restarts"] == 0


def test_processes_fused_wait():
    # ranks declared on distinct devices: the insert grid polls the flags itself (what one process
    # per GPU runs). On ONE shared GPU this is safe only for tiny grids (a spinning insert grid must
    # not hold the CUs the other process's expand grid needs): 2pc N=4, every level a few blocks.
    outs = run_ranks(["2pc:4", "2pc:4"], distinct=True, env={"SR_HEAD_MAX": "0"})
    for rank_out in outs:
        for r in rank_out:
            assert (r["unique"], r["states"], r["depth"], r["discoveries"]) == expect(r["check"])
            assert r["pipelined"] == 2


def test_bench_two_ranks_rehearsal():
    # bench.py's multi-process flow (torch.distributed.run as a child, one rank per process, timing
    # barrier, max over ranks, the replicas leg) with both ranks on this GPU over the shared-memory
    # transport: one JSON line from rank 0, the partitioned check on the direct exchange.
    root = os.path.dirname(HERE)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--comm", "shm", "--steps", "2",
                        "--warmup", "1", "--config4-steps", "0"], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size"] == 2 and d["config"]["comm"] == "shm"
    assert "direct exchange" in d["config"]["parallelism"]
    assert d["replicas"]["n_gpus"] == 2 and d["value"] > 0
