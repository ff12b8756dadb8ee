# Round evidence per game: the bench line (with cpu_baseline), then tools/profile.sh (kernel trace + stats, one PMC
# pass each for FETCH_SIZE and WRITE_SIZE) -> gpurun_out/final/<game>/ and gpurun_out/prof_<game>/
set -o pipefail
for g in "$@"; do
  mkdir -p gpurun_out/final/$g
  timeout -k 10 300 python -u bench.py --game $g > gpurun_out/final/$g/bench.jsonl 2> gpurun_out/final/$g/bench.err || exit 40
  bash tools/profile.sh $g --game $g || exit 41
done
