"""What a library user's trajectory placement costs: K fresh trajectories from VecEnv.new_traj_out() (the default:
candidates cut by the probe and ranked by one rollout launch each, DESIGN.md placement; PD_RANK=probe: the probe
alone) next to K unselected ones (select=1), each timed by rollout launches
in this process. Cached blocks are released between draws (torch.cuda.empty_cache), so every draw is a fresh device
allocation, as in a new process.
  python tools/placement_default.py GAME N T K      -> one JSON line per draw, then a summary line"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402

game, n, T, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rank = os.environ.get('PD_RANK', 'rollout')
v = VecEnv(game, n, seed=42, device=0)
v.reset()
t = 0
warm = v.new_traj_out(T, select=1)
for _ in range(20):   # the streams past their first refills (bench.py preconditions longer)
    v.rollout(T, 5, t * T, out=warm)
    t += 1
del warm
torch.cuda.synchronize()
torch.cuda.empty_cache()


def timed(traj):
    global t
    ms = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v.rollout(T, 5, t * T, out=traj)
        e1.record()
        t += 1
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return statistics.median(ms)


res = {'default': [], 'unselected': []}
for k in range(K):
    for mode in ('unselected', 'default') if k % 2 else ('default', 'unselected'):
        tr = v.new_traj_out(T, rank=rank) if mode == 'default' else v.new_traj_out(T, select=1)
        ms = timed(tr)
        res[mode].append(ms)
        va = {key: x.data_ptr() for key, x in tr.items()}   # virtual addresses: does the class follow any VA bits?
        print(json.dumps(dict(game=game, draw=k, mode=mode, kernel_ms=round(ms, 4), probe_ms=v.placement_probe_ms,
                              trial_ms=v.placement_trial_ms,
                              select_ms=round(v.placement_select_ms, 1), va=va)), flush=True)
        del tr
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
fast = min(res['default'] + res['unselected'])
print(json.dumps(dict(game=game, n=n, T=T, draws=K, rank=rank, fastest_ms=fast,
                      default_ms=res['default'], unselected_ms=res['unselected'],
                      default_max_over_fastest=max(res['default']) / fast,
                      unselected_max_over_fastest=max(res['unselected']) / fast)), flush=True)
