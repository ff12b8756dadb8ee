#!/bin/bash
# fused steps per launch on the final build: Limit / No-limit T 256 vs 512, alternating, 2 rounds (bench.py lines)
set -o pipefail
mkdir -p gpurun_out/abT
for rep in 1 2; do
  for g in limit-holdem no-limit-holdem; do
    for T in 256 512; do
      timeout -k 10 300 python bench.py --game $g --T $T --no-cpu-baseline --no-philox > gpurun_out/abT/${g}_T${T}_$rep.log 2>&1 || exit 31
    done
  done
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob('gpurun_out/abT/*.log')):
    ls = [l for l in open(f) if l.startswith('{')]
    if ls:
        d = json.loads(ls[-1]); print('%-32s %.4g env-steps/s  %.3f ms/launch' % (os.path.basename(f), d['value'], d['ms_per_step']))
PY
