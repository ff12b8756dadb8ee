#!/bin/bash
# GPU tests, then A/B of compile-time variants: LIBS x SPECS ("game:N:T ..."), alternating rounds, one process per
# (lib, spec) run on one device
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
make -s -j4 -C rlcard_amd/csrc variants >> gpurun_out/build.log 2>&1 || exit 11
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 30
fi
: > gpurun_out/ablibs.log
for rnd in 1 2 3; do
  for spec in $SPECS; do
    for lib in $LIBS; do
      echo "round $rnd $lib" >> gpurun_out/ablibs.log
      CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py ${spec//:/ } 0 >> gpurun_out/ablibs.log 2>&1 || exit 34
    done
  done
done
