#!/bin/bash
# same-box A/B of fused steps per launch (bench.py --T), alternating: SPEC="leduc-holdem:256 leduc-holdem:512 ..."
set -o pipefail
mkdir -p gpurun_out/abT
for rep in 1 2; do
  for s in $SPEC; do
    g=${s%%:*}; T=${s##*:}
    timeout -k 10 300 python bench.py --game $g --T $T --no-cpu-baseline --no-philox > gpurun_out/abT/${g}_T${T}_$rep.log 2>&1 || exit 31
  done
done
python3 - <<'PY'
import glob, json, os, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/abT/*.log')):
    ls = [l for l in open(f) if l.startswith('{')]
    if ls:
        d = json.loads(ls[-1]); k = os.path.basename(f).rsplit('_', 1)[0]
        r[k].append((d['value'], d['roofline']['frac']))
for k, v in sorted(r.items()):
    print(k, ' '.join('%.4g (%.3f)' % x for x in v))
PY
