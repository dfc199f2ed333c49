#!/bin/bash
# Round 6: config 4 at T = 2 and 4: the sent cache off (SR_SEND_CACHE=0) and the route kernel's
# per-lane queues (SR_ROUTE_QUEUE=1, needs no sent cache), against the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for T in 2 4; do
bash scripts/gpu_okey_sweep.sh 11 $T "SR_X=0" "SR_SEND_CACHE=0" "SR_SEND_CACHE=0 SR_ROUTE_QUEUE=1" "SR_SEND_CACHE=0 SR_ROUTE_QUEUE=0" || exit 1
done
echo "c4 t24 ok"
