set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 300 python -u bench.py --model paxos --clients 3 > $O/paxos3.json 2> $O/paxos3.err || { tail -5 $O/paxos3.err; exit 1; }
tail -1 $O/paxos3.json | cut -c1-300
timeout -k 10 300 python -u bench.py --model paxos --clients 6 --steps 5 --cpu-baseline 0 > $O/paxos6.json 2> $O/paxos6.err || { tail -5 $O/paxos6.err; exit 1; }
tail -1 $O/paxos6.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_paxos3 -o ks -- python3 bench.py --model paxos --clients 3 --steps 10 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > $O/ks_paxos3.log 2>&1 || { tail -5 $O/ks_paxos3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_2pc9 -o ks -- python3 bench.py --steps 10 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > $O/ks_2pc9.log 2>&1 || { tail -5 $O/ks_2pc9.log; exit 1; }
find $O -name "*stats*.csv"
echo done
