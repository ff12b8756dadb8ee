"""A/B timing of k_rollout kernel variants (cs_debug_set_kernel_flags) interleaved in ONE process (rule 24).
  python tools/ab_rollout.py GAME N T flagsA flagsB ...
AB_PLAYERS (env): game_num_players. AB_WARM (env, default 40) launches run first so the MT streams reach their steady block-refill rate (every env starts
at stream position 0 after seeding, so the first refills all come ~624 draws in)."""
import os
import sys
import statistics

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402

game, n, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = [int(x) for x in sys.argv[4:]] or [0, 2, 4, 6]
# AB_TS=T1,T2,..: the variants are fused-step counts (kernel flags 0) instead of kernel flags; T is ignored
Ts = [int(x) for x in os.environ.get('AB_TS', '').split(',') if x]
if Ts:
    variants = Ts
np_ = int(os.environ.get('AB_PLAYERS', '0'))   # game_num_players (0: the game's default)
inst = int(os.environ.get('AB_INST', '1'))       # fresh VecEnv allocations, variants interleaved in each (box / run
allt = {f: [] for f in variants}                 # variance follows the allocation: compare within one)
for i in range(inst):
    v = VecEnv(game, n, seed=42 + i, device=0, config={'game_num_players': np_} if np_ else None)
    v.reset()
    Tv = {f: (f if Ts else T) for f in variants}
    # one allocation of the largest T; smaller T launches write its leading steps (same buffers, no allocation effect)
    big = v.new_traj_out(max(Tv.values()), select=1) if Ts else None
    trs = {f: {k: x[:Tv[f]] for k, x in big.items()} for f in variants} if Ts else None
    tr = v.new_traj_out(T, select=1) if not Ts else trs[variants[0]]
    t = 0   # absolute step of the policy stream
    for _ in range(int(os.environ.get('AB_WARM', '40'))):
        v.rollout(Tv[variants[0]], 5, t, out=tr); t += Tv[variants[0]]
    for f in variants:            # warm-up each variant
        if not Ts:
            v.set_kernel_flags(f)
        v.rollout(Tv[f], 5, t, out=trs[f] if Ts else tr); t += Tv[f]
    torch.cuda.synchronize()
    times = {f: [] for f in variants}
    for rnd in range(6):
        for f in variants:
            if not Ts:
                v.set_kernel_flags(f)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(5):
                v.rollout(Tv[f], 5, t, out=trs[f] if Ts else tr); t += Tv[f]
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / 5 / (Tv[f] / T))   # per T steps
    for f in variants:
        allt[f] += times[f]
        if inst > 1:
            print('  instance %d flags=%d: median %.3f ms/launch' % (i, f, statistics.median(times[f])), flush=True)
    del v, tr, trs, big
    torch.cuda.empty_cache()
for f in variants:
    med = statistics.median(allt[f])
    print('%s n=%d T=%d flags=%d: median %.3f ms/launch (min %.3f) -> %.3g env-steps/s' % (
        game, n, T, f, med, min(allt[f]), n * T / (med * 1e-3)), flush=True)
