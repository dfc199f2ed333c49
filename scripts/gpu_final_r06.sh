#!/bin/bash
# Round 6 last pass at the current sources, in two gpurun calls:
#   scripts/gpu_final_r06.sh <tag> pmc    PMC ceilings and traffic stamped with the source digest
#   scripts/gpu_final_r06.sh <tag> bench  bench lines (they read the stamped PMC files), the rocprofv3
#                                         kernel stats of 2pc N=9 and paxos C=3, the shm rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06final}
O=gpurun_out/$T
mkdir -p $O
if [ "$2" = pmc ]; then
    bash scripts/gpu_roofline.sh > $O/roofline.log 2>&1 || { tail -20 $O/roofline.log; exit 1; }
    tail -3 $O/roofline.log
    exit 0
fi
bash scripts/gpu_round.sh $T bench || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --config4-steps 0 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_paxos3 -o bench -- python3 bench.py --model paxos --clients 3 --steps 10 --warmup 2 --cpu-baseline 0 --config4-steps 0 > $O/prof_paxos3.log 2>&1 || { echo "rocprof paxos failed"; tail -20 $O/prof_paxos3.log; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 --comm shm --steps 10 --warmup 2 --config4-steps 1 > $O/bench_rehearsal_shm_n2.json 2> $O/bench_rehearsal_shm_n2.err || { tail -20 $O/bench_rehearsal_shm_n2.err; exit 1; }
tail -1 $O/bench_rehearsal_shm_n2.json
echo "final bench ok"
