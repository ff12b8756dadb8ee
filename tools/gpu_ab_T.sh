#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
: > gpurun_out/abT.log
for T in 8 16 32 64 128; do
  timeout -k 10 200 python tools/ab_rollout.py leduc-holdem 1048576 $T 0 >> gpurun_out/abT.log 2>&1 || exit 34
done
for T in 16 64; do
  timeout -k 10 200 python tools/ab_rollout.py limit-holdem 262144 $T 0 >> gpurun_out/abT.log 2>&1 || exit 35
done
for N in 262144 2097152 4194304; do
  timeout -k 10 200 python tools/ab_rollout.py leduc-holdem $N 32 0 >> gpurun_out/abT.log 2>&1 || exit 36
done
