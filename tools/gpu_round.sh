#!/bin/bash
# one GPU session: build, pytest -m gpu, smoke, bench(es) (each step time-limited; stop at the first failure)
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 30
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 31
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 32
for g in $BENCH_EXTRA; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --game $g > gpurun_out/bench_$g.log 2>&1 || exit 33
done
