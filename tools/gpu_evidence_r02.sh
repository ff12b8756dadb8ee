#!/bin/bash
# Round-2 evidence: bench line per game (cpu_baseline, reference_cpu, rng_philox), then tools/profile.sh (kernel trace
# + stats, one PMC pass each for FETCH_SIZE / WRITE_SIZE at the bench's timed launches) -> gpurun_out/final/<game>/
set -o pipefail
for g in "$@"; do
  mkdir -p gpurun_out/final/$g
  timeout -k 10 300 python -u bench.py --game $g > gpurun_out/final/$g/bench.jsonl 2> gpurun_out/final/$g/bench.err || exit 40
  STEPS=40 bash tools/profile.sh $g --game $g || exit 41
done
