#!/bin/bash
# Round-2 final: full GPU suite, smoke, then per game the bench line and the rocprofv3 evidence (tools/profile.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 30
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 31
bash tools/gpu_evidence_r02.sh leduc-holdem limit-holdem doudizhu no-limit-holdem blackjack || exit 32
