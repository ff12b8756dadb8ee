# all GPU tests (default library), Leduc tests against VARIANT_LIB, then A/B on Leduc (LEDUC_LIBS) and Limit (LIMIT_LIBS)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || exit 30
if [ -n "$VARIANT_LIB" ]; then
  CARDSIM_LIB=$VARIANT_LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q -k leduc --timeout 200 --timeout-method thread > gpurun_out/ab/tests_variant.log 2>&1 || exit 31
fi
: > gpurun_out/ab/ab.log
for rnd in 1 2; do
  for lib in $LEDUC_LIBS; do
    echo "round $rnd $lib" >> gpurun_out/ab/ab.log
    CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py leduc-holdem 1048576 128 0 >> gpurun_out/ab/ab.log 2>&1 || exit 34
  done
  for lib in $LIMIT_LIBS; do
    echo "round $rnd $lib" >> gpurun_out/ab/ab.log
    CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py limit-holdem 262144 64 0 >> gpurun_out/ab/ab.log 2>&1 || exit 35
  done
done
