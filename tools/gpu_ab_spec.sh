# A/B of prebuilt libraries on one rollout spec, 2 alternating rounds (no tests): bash tools/gpu_ab_spec.sh "GAME N T" lib...
set -o pipefail
mkdir -p gpurun_out/ab
SPEC=$1; shift
: > gpurun_out/ab/ab_spec.log
for rnd in 1 2; do
  for lib in "$@"; do
    echo "round $rnd $lib" >> gpurun_out/ab/ab_spec.log
    CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py $SPEC 0 >> gpurun_out/ab/ab_spec.log 2>&1 || exit 34
  done
done
