#!/bin/bash
# build -> GPU tests -> A/B of kernel flags (one process per game) -> A/B of compile-time variants ($LIBS on $SPEC)
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
make -s -j4 -C rlcard_amd/csrc variants >> gpurun_out/build.log 2>&1 || exit 11
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 30
: > gpurun_out/ab.log
for spec in $AB_SPECS; do
  timeout -k 10 200 python tools/ab_rollout.py ${spec//:/ } ${AB_FLAGS:-0 2} >> gpurun_out/ab.log 2>&1 || exit 34
done
: > gpurun_out/ablibs.log
if [ -n "$LIBS" ]; then
for rnd in 1 2 3; do
  for lib in $LIBS; do
    echo "round $rnd $lib" >> gpurun_out/ablibs.log
    CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py ${SPEC//:/ } 0 >> gpurun_out/ablibs.log 2>&1 || exit 35
  done
done
fi
