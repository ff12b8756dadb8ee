set -o pipefail
mkdir -p gpurun_out/cfr
timeout -k 10 300 python -u -m pytest tests/test_cfr.py tests/test_envs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/cfr/tests.log 2>&1 || exit 30
timeout -k 10 300 python -u tools/bench_cfr.py > gpurun_out/cfr/bench_cfr.jsonl 2> gpurun_out/cfr/bench_cfr.err || exit 31
