# scripts/sweep_env.sh VAR "v1 v2 ..." <bench args...>: one bench line per value of env VAR.
set -o pipefail
cd $GRAFT_REPO_ROOT
var=$1; vals=$2; shift 2
for v in $vals; do
  r=$(env $var=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 "$@" 2>/dev/null) || exit 1
  echo "$var=$v $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("value=%.4g ms_per_step=%.3f kernel_ms=%.3f" % (d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"]*d["roofline"]["launches_per_step"]))')"
done
