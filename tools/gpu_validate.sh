#!/bin/bash
# GPU validation pass: parity tests, smoke, default bench, single-env compat bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit 30
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 31
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit 32
timeout -k 10 300 python tools/bench_compat.py --seconds 4 > gpurun_out/compat.log 2>&1 || exit 33
tail -3 gpurun_out/gpu_tests.log
