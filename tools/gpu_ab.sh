#!/bin/bash
# build, GPU tests, then A/B of kernel variants (interleaved in one process per game)
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 30
: > gpurun_out/ab.log
for spec in "leduc-holdem 1048576" "limit-holdem 262144" "blackjack 262144"; do
  timeout -k 10 200 python tools/ab_rollout.py $spec 16 ${AB_FLAGS:-0 2} >> gpurun_out/ab.log 2>&1 || exit 34
done
