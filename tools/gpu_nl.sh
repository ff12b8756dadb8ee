set -o pipefail
mkdir -p gpurun_out/nl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/nl/gpu_tests.log 2>&1 || exit 30
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/nl/smoke.log 2>&1 || exit 31
timeout -k 10 200 python -u bench.py --game no-limit-holdem > gpurun_out/nl/bench_nl.jsonl 2> gpurun_out/nl/bench_nl.err || exit 32
