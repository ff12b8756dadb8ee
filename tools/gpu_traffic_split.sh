#!/bin/bash
# Leduc traffic split: FETCH_SIZE and WRITE_SIZE (separate passes) of k_rollout for the product library
# and profiling builds that drop outputs (CS_PROF_NO_SMALL: legal / player / reward / done; CS_PROF_NO_OBS: obs rows)
#   bash tools/gpu_traffic_split.sh   -> gpurun_out/split/<lib>_<counter>/
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in libcardsim.so libcardsim_nosmall.so libcardsim_noobs.so libcardsim_noout.so; do
  for c in FETCH_SIZE WRITE_SIZE; do
    O=$R/gpurun_out/split/${lib%.so}_$c
    mkdir -p $O
    CARDSIM_LIB=$lib AB_WARM=12 timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O -o p -- python3 tools/ab_rollout.py leduc-holdem 1048576 256 0 > $O/run.log 2>&1 || exit 20
  done
done
