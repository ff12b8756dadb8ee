#!/bin/bash
# Round evidence: GPU tests, smoke, bench line per config, rocprofv3 kernel trace + FETCH/WRITE passes per config.
#   TAG=r01 bash tools/gpu_measure.sh            (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 31
for g in ${GAMES:-leduc-holdem doudizhu limit-holdem}; do
  timeout -k 10 300 python bench.py --game $g > gpurun_out/bench_$g.jsonl 2> gpurun_out/bench_$g.err || exit 32
  bash tools/profile.sh $g --game $g --steps 10 --warmup 2 || exit 33
done
