#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (k_rollout), at an explicit timed-launch count: kernel trace +
# stats, then one PMC pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no tracing beside
# --pmc). tools/pmc_traffic.py then averages the last STEPS dispatches (the timed launches) only.
#   STEPS=100 bash tools/profile.sh <tag> [bench args...]      (libraries prebuilt in-tree)
set -o pipefail
TAG=${1:-leduc}; shift
ARGS="$@"
STEPS=${STEPS:-100}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu-baseline --no-philox --steps $STEPS $ARGS > $O/bench_kt.log 2>&1 || exit 41
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 bench.py --no-cpu-baseline --no-philox --steps $STEPS $ARGS > $O/bench_fetch.log 2>&1 || exit 42
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 bench.py --no-cpu-baseline --no-philox --steps $STEPS $ARGS > $O/bench_write.log 2>&1 || exit 43
find $O -name "*.csv" | head -20 > $O/files.txt
