"""In-process A/B of library builds over the SAME trajectory buffers.

  python tools/ab_libs.py GAME N T LIB1 LIB2 ...      (LIBs: file names under rlcard_amd/, e.g. libcardsim.so)

Where a trajectory lands in HBM sets how fast a launch writes it (placement), and a fresh process or a fresh
allocation draws a new placement. So this tool loads every library into ONE process (each its own ctypes handle and
HIP module), gives each its own VecEnv (same seeds), and has every library write into the same trajectory
allocation, interleaved round by round: the placement is common to the variants and drops out of the comparison.
AB_INST (3) trajectory allocations in turn (each the probe-ranked best of AB_SELECT (3) candidates, as VecEnv.new_traj_out
chooses by default; 1: unselected), AB_ROUNDS (5) rounds each, AB_K (5) timed launches per round and
library, AB_WARM (40) untimed launches per library first (the MT streams reach their steady refill rate).
Prints per-allocation medians and the overall median per library (ms per launch of T steps), and flags libraries whose
trajectories differ (a checksum of one more launch per allocation, from identical env states)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
from rlcard_amd import _abi, VecEnv  # noqa: E402

game, n, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
libs = sys.argv[4:]
inst = int(os.environ.get('AB_INST', '3'))
rounds = int(os.environ.get('AB_ROUNDS', '5'))
K = int(os.environ.get('AB_K', '5'))
warm = int(os.environ.get('AB_WARM', '40'))
flags = int(os.environ.get('AB_FLAGS', '0'))
sel = int(os.environ.get('AB_SELECT', '3'))   # the allocation: the fastest of this many by the placement probe

handles = {}
for p in libs:
    _abi.LIB_PATH = os.path.join(_abi._HERE, p)
    _abi._lib = None
    handles[p] = _abi.lib()


def use(p):
    _abi._lib = handles[p]


envs, t = {}, {}
for p in libs:
    use(p)
    v = VecEnv(game, n, seed=42, device=0)
    v.set_kernel_flags(flags)
    v.reset()
    envs[p], t[p] = v, 0
allt = {p: [] for p in libs}
for i in range(inst):
    use(libs[0])
    tr = envs[libs[0]].new_traj_out(T, select=sel, rank='probe')   # one allocation, written by every library
    for p in libs:
        use(p)
        for _ in range(warm if i == 0 else 3):
            envs[p].rollout(T, 5, t[p], out=tr)
            t[p] += T
    torch.cuda.synchronize()
    per = {p: [] for p in libs}
    for r in range(rounds):
        for p in libs:
            use(p)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                envs[p].rollout(T, 5, t[p], out=tr)
                t[p] += T
            e1.record()
            torch.cuda.synchronize()
            per[p].append(e0.elapsed_time(e1) / K)
    # the same launch (same env states, policy seed and step counter in every library) -> a checksum of the whole
    # trajectory per library: a variant that is faster but writes other outputs shows up here
    sums = {}
    for p in libs:
        use(p)
        envs[p].rollout(T, 5, t[p], out=tr)
        t[p] += T
        sums[p] = sum(int(x.view(torch.uint8).to(torch.int64).sum()) * (k + 1) for k, x in enumerate(tr.values()))
    if len(set(sums.values())) != 1:
        print('  OUTPUTS DIFFER across libraries: %s' % sums, flush=True)
    for p in libs:
        allt[p] += per[p]
        print('  allocation %d %-26s median %.3f ms/launch (min %.3f)' % (i, p, statistics.median(per[p]),
                                                                      min(per[p])), flush=True)
    del tr
    torch.cuda.empty_cache()
base = statistics.median(allt[libs[0]])
for p in libs:
    med = statistics.median(allt[p])
    print('%s %s n=%d T=%d: median %.3f ms/launch (%+.1f %% vs %s) -> %.3g env-steps/s' % (
        game, p, n, T, med, 100.0 * (med / base - 1.0), libs[0], n * T / (med * 1e-3)), flush=True)
