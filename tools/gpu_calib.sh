#!/bin/bash
# HBM counter calibration (tools/calib.py): one PMC pass per counter over known byte counts.
set -o pipefail
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/calib
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 tools/calib.py > $O/fetch.log 2>&1 || exit 51
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 tools/calib.py > $O/write.log 2>&1 || exit 52
python3 tools/calib.py --report $O > $O/calib.json 2>&1 || exit 53
cat $O/calib.json
