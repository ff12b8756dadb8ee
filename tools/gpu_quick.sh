#!/bin/bash
# quick check after a kernel change: rollout parity tests, bench lines (no CPU baseline / Philox), Leduc WRITE_SIZE
#   GAMES="leduc-holdem limit-holdem" PYK="rollout" bash tools/gpu_quick.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_refill.py -x -q -k "${PYK:-rollout}" --timeout 300 --timeout-method thread > gpurun_out/quick/tests.log 2>&1 || exit 30
for g in ${GAMES:-leduc-holdem limit-holdem no-limit-holdem}; do
  timeout -k 10 300 python bench.py --game $g --no-cpu-baseline --no-philox > gpurun_out/quick/bench_$g.log 2>&1 || exit 31
done
if [ -n "$PMC" ]; then
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/quick/write -o p -- python3 tools/ab_rollout.py ${PMC} 0 > gpurun_out/quick/pmc.log 2>&1 || exit 32
fi
