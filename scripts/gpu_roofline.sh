#!/bin/bash
# Memory-side (beyond-L2) request rates of the expand kernel against the measured request ceilings,
# from rocprofv3 PMC counters (separate passes, counters only with --kernel-trace, per the pool
# rules). Run from the repo root on the GPU box:  bash scripts/gpu_roofline.sh
#   1. the ceiling: scripts/microbench_random (random 8-byte loads with 1/4/8 in flight per lane,
#      random CAS and stores over tables of 8 MiB .. 4 GiB) with TCC_EA0_{RDREQ,WRREQ,ATOMIC}_sum:
#      the largest EA read / write / atomic request rate any dispatch reached;
#   2. per bench configuration, three passes over `bench.py` (EA request counts; read bytes by
#      request size; WRITE_SIZE) on the non-counting expand_fast dispatches.
# scripts/pmc_requests.py writes profiles/pmc_ceiling.json and profiles/pmc_traffic.json, stamped
# with the engine's source digest (bench.py ignores a file measured on other sources).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/roofline
mkdir -p $O
REQ="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum"
timeout -k 10 120 rocprofv3 --pmc $REQ --kernel-trace --output-format csv -d $O/ceiling -o c -- ./scripts/microbench_random > $O/ceiling.log 2>&1 || { echo "ceiling pass failed"; tail -5 $O/ceiling.log; exit 1; }
run() {  # label, bench args
    local tag=$1; shift
    local B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 $*"
    timeout -k 10 180 rocprofv3 --pmc $REQ --kernel-trace --output-format csv -d $O/$tag/req -o r -- python3 $B > $O/$tag.req.log 2>&1 || { echo "$tag req pass failed"; tail -5 $O/$tag.req.log; return 1; }
    timeout -k 10 180 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d $O/$tag/rd -o r -- python3 $B > $O/$tag.rd.log 2>&1 || { echo "$tag rd pass failed"; return 1; }
    timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/$tag/wr -o r -- python3 $B > $O/$tag.wr.log 2>&1 || { echo "$tag wr pass failed"; return 1; }
    echo "$tag ok"
}
run 2pc9 --rm-count 9 && run 2pc10 --rm-count 10 && run 2pc11 --rm-count 11 && \
run inclock10 --model increment_lock --threads 10 && run inclock11 --model increment_lock --threads 11 && \
run paxos3 --model paxos --clients 3 && python3 scripts/pmc_requests.py $O
