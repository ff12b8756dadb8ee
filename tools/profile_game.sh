#!/bin/bash
# One game's round evidence on the GPU box, all under gpurun_out/prof/<tag>/ (merged back by gpurun): the bench line
# under rocprofv3 --kernel-trace --stats, then one PMC pass each for FETCH_SIZE and WRITE_SIZE (separate runs: they
# cannot share a pass). Afterwards, on the build host:
#   python tools/pmc_traffic.py profiles/<round>/<tag> <game:envs:T> profiles/<round>/<tag> gpurun_out/prof/<tag>/pmc_*
#   bash tools/profile_game.sh GAME TAG [extra bench args]
set -euo pipefail
G=$1; TAG=$2; shift 2
export TMPDIR=/tmp
W=gpurun_out/prof/$TAG
rm -rf "$W"; mkdir -p "$W"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/trace" -o run -- python3 bench.py --game "$G" "$@" \
    > "$W/bench.jsonl" 2> "$W/trace.err"
cp "$(find "$W/trace" -name '*kernel_stats.csv' | head -n 1)" "$W/kernel_stats.csv"
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$W/pmc_$C" -o run -- python3 bench.py --game "$G" --steps 5 \
        --no-cpu-baseline "$@" > "$W/pmc_$C.out" 2> "$W/pmc_$C.err"
done
