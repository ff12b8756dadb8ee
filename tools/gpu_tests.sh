#!/bin/bash
# GPU parity tests (+ optional bench): each step time-limited, stop at the first failure. Libraries are prebuilt in-tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/gpu_tests.log 2>&1 || exit 30
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 31
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > gpurun_out/bench.log 2>&1 || exit 32
fi
tail -3 gpurun_out/gpu_tests.log
