#!/bin/bash
# diagnostic: native ABI driver (no torch) at several sizes, then python probes by load order (riskiest last)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/diag.log
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 10
make -s -C tools >> gpurun_out/build.log 2>&1 || exit 11
python tools/keys.py 42 200 > /tmp/k200 && python tools/keys.py 42 1048576 > /tmp/k1m && python tools/keys.py 7 262144 > /tmp/k256k || exit 12
echo "== native leduc 200" > $L
timeout -k 10 120 ./tools/abi_driver 1 200 8 < /tmp/k200 >> $L 2>&1 || exit 21
echo "== native leduc 1M" >> $L
timeout -k 10 300 ./tools/abi_driver 1 1048576 16 512 < /tmp/k1m >> $L 2>&1 || exit 22
echo "== native limit 256K" >> $L
timeout -k 10 300 ./tools/abi_driver 2 262144 16 512 < /tmp/k256k >> $L 2>&1 || exit 23
echo "== native blackjack 256K" >> $L
timeout -k 10 300 ./tools/abi_driver 0 262144 16 512 < /tmp/k256k >> $L 2>&1 || exit 24
echo "== python lib-first" >> $L
timeout -k 10 300 python tools/gpu_probe.py --lib-first leduc-holdem 200 1 1048576 >> $L 2>&1 || exit 25
echo "== python torch-first" >> $L
timeout -k 10 300 python tools/gpu_probe.py --torch-first leduc-holdem 200 1 >> $L 2>&1 || exit 26
