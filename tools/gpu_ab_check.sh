# parity tests selected by GAME_K (pytest -k expression), then A/B of prebuilt libraries on one rollout spec
#   GAME_K=leduc bash tools/gpu_ab_check.sh "GAME N T" lib1 lib2 ...
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$GAME_K" --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || exit 30
bash tools/gpu_ab_leduc.sh "$@"
