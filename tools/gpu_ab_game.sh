#!/bin/bash
# Same-box A/B of library builds for one game: optional parity tests first (TESTK=pytest -k expr), then
#   bench.py per library (CARDSIM_LIB), REPS rounds; prints per-launch kernel ms per library.
#   TESTK=blackjack REPS=2 bash tools/gpu_ab_game.sh <game> <lib.so> [<lib.so> ...]
set -o pipefail
G=$1; shift
REPS=${REPS:-2}
O=gpurun_out/ab_$G
mkdir -p $O
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$TESTK" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 30; }
  tail -2 $O/tests.log
fi
for rep in $(seq $REPS); do
  for lib in "$@"; do
    CARDSIM_LIB=$lib timeout -k 10 300 python bench.py --game $G --no-cpu-baseline --no-philox $BENCH_ARGS > $O/${lib%.so}_$rep.log 2>&1 || exit 31
  done
done
python3 - "$O" <<'PY'
import glob, json, os, sys, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + '/*.log')):
    ls = [l for l in open(f) if l.startswith('{')]
    if ls:
        d = json.loads(ls[-1])
        r[os.path.basename(f).rsplit('_', 1)[0]].append(d['roofline']['kernel_ms_per_launch'])
for k, v in sorted(r.items()):
    print('%-28s %s' % (k, ' '.join('%.3f' % x for x in v)))
PY
