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
np_ = int(os.environ.get('AB_PLAYERS', '0'))   # game_num_players (0: the game's default)
inst = int(os.environ.get('AB_INST', '1'))       # fresh VecEnv allocations, variants interleaved in each (box / run
allt = {f: [] for f in variants}                 # variance follows the allocation: compare within one)
for i in range(inst):
    v = VecEnv(game, n, seed=42 + i, device=0, config={'game_num_players': np_} if np_ else None)
    v.reset()
    tr = v.new_traj_out(T)
    t = 0
    for _ in range(int(os.environ.get('AB_WARM', '40'))):
        v.rollout(T, 5, t * T, out=tr); t += 1
    for f in variants:            # warm-up each variant
        v.set_kernel_flags(f)
        v.rollout(T, 5, t * T, out=tr); t += 1
    torch.cuda.synchronize()
    times = {f: [] for f in variants}
    for rnd in range(6):
        for f in variants:
            v.set_kernel_flags(f)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(5):
                v.rollout(T, 5, t * T, out=tr); t += 1
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / 5)
    for f in variants:
        allt[f] += times[f]
        if inst > 1:
            print('  instance %d flags=%d: median %.3f ms/launch' % (i, f, statistics.median(times[f])), flush=True)
    del v, tr
    torch.cuda.empty_cache()
for f in variants:
    med = statistics.median(allt[f])
    print('%s n=%d T=%d flags=%d: median %.3f ms/launch (min %.3f) -> %.3g env-steps/s' % (
        game, n, T, f, med, min(allt[f]), n * T / (med * 1e-3)), flush=True)
