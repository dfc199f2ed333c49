#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/n11_probe.py 11 > gpurun_out/n11_default.log 2>&1 || { tail -20 gpurun_out/n11_default.log; exit 1; }
SR_GRID_MAX=1000000 timeout -k 10 200 python -u scripts/n11_probe.py 11 > gpurun_out/n11_nocap.log 2>&1 || { tail -20 gpurun_out/n11_nocap.log; exit 1; }
grep "^check" gpurun_out/n11_default.log gpurun_out/n11_nocap.log
