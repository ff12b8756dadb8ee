#!/bin/bash
# SQ/TA counters for one rollout config (one PMC pass per counter group, no tracing beside --pmc)
#   bash tools/gpu_counters.sh TAG GAME N T
set -o pipefail
TAG=$1; GAME=$2; N=$3; T=$4
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cnt_$TAG
mkdir -p $O
# libraries prebuilt in-tree
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM" \
           "TD_BUSY_sum TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- python3 tools/ab_rollout.py $GAME $N $T 0 > $O/run$i.log 2>&1 || { echo "pass $i failed" >> $O/errors.log; exit 20; }
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1
