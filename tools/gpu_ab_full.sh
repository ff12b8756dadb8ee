# all GPU tests, then A/B of prebuilt libraries on the Leduc and Limit bench shapes (2 rounds each)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || exit 30
: > gpurun_out/ab/ab.log
for spec in "leduc-holdem 1048576 128" "limit-holdem 262144 64"; do
  for rnd in 1 2; do
    for lib in "$@"; do
      echo "round $rnd $lib" >> gpurun_out/ab/ab.log
      CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py $spec 0 >> gpurun_out/ab/ab.log 2>&1 || exit 34
    done
  done
done
