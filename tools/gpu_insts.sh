#!/bin/bash
# Instruction-mix counters (one PMC pass) of k_rollout for several prebuilt libraries:
#   bash tools/gpu_insts.sh "GAME N T" lib...      -> gpurun_out/insts/<lib>/ + summary.txt
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
SPEC=$1; shift
O=$R/gpurun_out/insts
mkdir -p $O
: > $O/summary.txt
for lib in "$@"; do
  CARDSIM_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d $O/$lib -o p -- python3 tools/ab_rollout.py $SPEC 0 > $O/$lib.log 2>&1 || exit 30
  echo "== $lib" >> $O/summary.txt
  python3 tools/pmc_summary.py $O/$lib >> $O/summary.txt 2>&1
done
