set -e
mkdir -p gpurun_out/v1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v1/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.log 2>&1
for g in leduc-holdem limit-holdem doudizhu; do
  timeout -k 10 200 python -u bench.py --game $g > gpurun_out/v1/bench_$g.jsonl 2> gpurun_out/v1/bench_$g.err
done
