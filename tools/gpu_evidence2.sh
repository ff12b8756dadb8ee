#!/bin/bash
# One evidence session: counter calibration, the default bench line, then the rocprofv3 profile of the same
# configuration (timed launches only) for each game in GAMES_PROF (default: leduc-holdem).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_calib.sh > gpurun_out/calib.log 2>&1 || exit 50
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 32
for g in ${GAMES_PROF:-leduc-holdem}; do
  STEPS=${STEPS:-100} bash tools/profile.sh $g --game $g || exit 40
done
echo done
