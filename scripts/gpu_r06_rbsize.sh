#!/bin/bash
# Round 6: rehash_ranges' LDS per range (16 / 32 / 64 KB builds in gpurun_ab/lib_rb*.so), unhinted
# 2pc N=10 and increment_lock N=11 (bench.py's no_hint line).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export SR_LIB_DIGEST_CHECK=0
O=gpurun_out/r06rb
mkdir -p "$O"
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_new.so || exit 1
for r in 1 2; do
  for v in rb16 rb32 rb64; do
    cp "gpurun_ab/lib_$v.so" "$LIB" || exit 1
    for args in "--rm-count 10 --no-hint-steps 4" "--model increment_lock --threads 11 --no-hint-steps 2"; do
      tag=$(echo "$args" | tr -d ' -' | cut -c1-12)
      timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 1 --warmup 1 $args \
          > "$O/${v}_${tag}_$r.json" 2> "$O/${v}_${tag}_$r.err" || { tail -5 "$O/${v}_${tag}_$r.err"; cp gpurun_ab/lib_new.so "$LIB"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${tag}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('$v r$r $args', 'no_hint', round(n['ms_per_step'],3))"
    done
  done
done
cp gpurun_ab/lib_new.so "$LIB"
echo "rb ok"
