"""Per-allocation kernel time vs address-translation counters (diagnostic for the Leduc 3.5 / 4.3 ms box split,
VERDICT r03 next #2): fresh VecEnv + trajectory allocations in ONE process, each preconditioned like bench.py and
then timed over a few launches. Run it under `rocprofv3 --pmc ...` and pair every k_rollout dispatch's counters with
its own Start/End timestamps (tools/tlb_summary.py); without a profiler it prints the per-instance event times.

  python tools/tlb_probe.py GAME [instances] [timed launches]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402

game = sys.argv[1]
inst = int(sys.argv[2]) if len(sys.argv) > 2 else 4
timed = int(sys.argv[3]) if len(sys.argv) > 3 else 6
g = bench.GAMES[game]
n, T = g['envs'], g['T']
keep = []   # AP_KEEP=1: keep every instance alive (each new one lands on other physical pages)
for i in range(inst):
    v = VecEnv(game, n, seed=42, device=0)
    v.reset()
    tr = v.new_traj_out(T, select=1)
    pre = bench.precondition_launches(game, T, v)
    for c in range(pre):
        v.rollout(T, 5, c * T, out=tr)
    torch.cuda.synchronize()
    ms = []
    for k in range(timed):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v.rollout(T, 5, (pre + k) * T, out=tr)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print('instance %d: %d precondition + %d timed launches, median %.3f ms (min %.3f max %.3f)  mt@%x obs@%x' % (
        i, pre, timed, statistics.median(ms), min(ms), max(ms), v.mt_address() if hasattr(v, 'mt_address') else 0,
        tr['obs'].data_ptr()), flush=True)
    if os.environ.get('AP_KEEP'):
        keep.append((v, tr))
    else:
        del tr, v
        torch.cuda.empty_cache()
