#!/bin/bash
# Leduc split: product vs profiling builds (CARDSIM_LIB) and the Philox stream, same box
set -o pipefail
mkdir -p gpurun_out/abL
for rep in 1 2; do
  for lib in libcardsim.so libcardsim_noobs.so libcardsim_nosmall.so libcardsim_noreset.so; do
    CARDSIM_LIB=$lib timeout -k 10 300 python bench.py --game leduc-holdem --no-cpu-baseline --no-philox --steps 150 > gpurun_out/abL/${lib%.so}_$rep.log 2>&1 || exit 31
  done
  timeout -k 10 300 python bench.py --game leduc-holdem --no-cpu-baseline --steps 150 > gpurun_out/abL/philox_$rep.log 2>&1 || exit 32
done
python3 - <<'PY'
import glob, json, os, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/abL/*.log')):
    ls = [l for l in open(f) if l.startswith('{')]
    if ls:
        d = json.loads(ls[-1]); k = os.path.basename(f).rsplit('_', 1)[0]
        r[k].append(d['roofline']['kernel_ms_per_launch'])
        if k == 'philox': r['philox_mode'].append(d['rng_philox']['kernel_ms_per_launch'])
for k, v in sorted(r.items()):
    print(k, ' '.join('%.3f' % x for x in v))
PY
