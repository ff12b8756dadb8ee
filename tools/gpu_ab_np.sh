#!/bin/bash
# N-player hold'em A/B of library builds (tools/ab_rollout.py with AB_PLAYERS), after the N-player parity tests
#   bash tools/gpu_ab_np.sh <lib.so> [<lib.so> ...]
set -o pipefail
O=gpurun_out/ab_np
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_nplayer.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 30; }
tail -1 $O/tests.log
for cfg in "limit-holdem 6 262144 256" "no-limit-holdem 6 262144 256" "limit-holdem 10 131072 256"; do
  set -- $cfg
  for lib in $LIBS; do
    echo -n "$lib P=$2: "
    AB_PLAYERS=$2 CARDSIM_LIB=$lib timeout -k 10 300 python tools/ab_rollout.py $1 $3 $4 0 | tail -1 || exit 31
  done
done
