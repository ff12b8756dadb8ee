set -e
mkdir -p gpurun_out/v2
for n in 786432 1048576 1179648 1572864 2097152; do
  timeout -k 10 120 python -u bench.py --game leduc-holdem --envs $n --steps 10 --no-cpu-baseline >> gpurun_out/v2/sweep_leduc.jsonl 2>/dev/null
done
for n in 163840 262144 327680 393216 524288; do
  timeout -k 10 120 python -u bench.py --game limit-holdem --envs $n --steps 10 --no-cpu-baseline >> gpurun_out/v2/sweep_limit.jsonl 2>/dev/null
done
bash tools/profile_game.sh limit-holdem limit-holdem
