#!/bin/bash
# Round 2: multi-rank (in-process ranks) tests, small-grid parity, then the N=1 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_dist_ranks.py::test_ranks_deferred_paths_are_collective" tests/test_gpu_dist_ranks.py::test_ranks_overflow_restart_is_collective tests/test_gpu_dist_ranks.py::test_ranks_bench_config tests/test_gpu_dist_ranks.py::test_config4_2pc11_partitioned_8_full_size \
  "tests/test_gpu_parity.py::test_small_grid_strides" > gpurun_out/r02a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02a_tests.log; exit 1; }
tail -3 gpurun_out/r02a_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err || { echo "bench failed"; tail -20 gpurun_out/r02a_bench.err; exit 1; }
cat gpurun_out/r02a_bench.json
