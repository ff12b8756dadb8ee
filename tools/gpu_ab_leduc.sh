# A/B of prebuilt library variants on one rollout spec: bash tools/gpu_ab_leduc.sh "GAME N T" lib1 lib2 ...
set -o pipefail
SPEC=$1; shift
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.log
for rnd in 1 2; do
  for lib in "$@"; do
    echo "round $rnd $lib" >> gpurun_out/ab/ab.log
    CARDSIM_LIB=$lib timeout -k 10 120 python tools/ab_rollout.py $SPEC 0 >> gpurun_out/ab/ab.log 2>&1 || exit 34
  done
done
