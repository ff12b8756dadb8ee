#!/bin/bash
# staggered ring seeding: the full GPU suite on the new build, then same-box A/B against the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_stagger.log 2>&1 || { tail -40 gpurun_out/gpu_tests_stagger.log; exit 30; }
tail -2 gpurun_out/gpu_tests_stagger.log
for g in leduc-holdem limit-holdem blackjack; do
  REPS=2 bash tools/gpu_ab_game.sh $g libcardsim.so libcardsim_r16.so || exit 31
done
