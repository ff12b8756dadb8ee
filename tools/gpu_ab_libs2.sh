#!/bin/bash
# same-box A/B of library builds on bench.py (alternating runs): LIBS="libcardsim.so libcardsim_x.so" GAMES="..." 
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for g in ${GAMES:-leduc-holdem limit-holdem}; do
    for lib in ${LIBS}; do
      CARDSIM_LIB=$lib timeout -k 10 300 python bench.py --game $g --no-cpu-baseline --no-philox --steps ${STEPS:-200} > gpurun_out/ab/${g}_${lib%.so}_$rep.log 2>&1 || exit 31
    done
  done
done
python3 - <<'PY'
import glob, json, os, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab/*.log')):
    ls = [l for l in open(f) if l.startswith('{')]
    if ls:
        d = json.loads(ls[-1]); k = os.path.basename(f).rsplit('_', 1)[0]
        r[k].append(d['roofline']['kernel_ms_per_launch'])
for k, v in sorted(r.items()):
    print(k, ' '.join('%.3f' % x for x in v))
PY
