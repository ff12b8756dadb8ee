"""Launch-time spread of one rollout across fresh VecEnv allocations in ONE process (diagnostic for box / run
variance): python tools/alloc_probe.py GAME N T [instances]"""
import os
import sys
import statistics

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402

game, n, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
inst = int(sys.argv[4]) if len(sys.argv) > 4 else 4
for i in range(inst):
    v = VecEnv(game, n, seed=42 + i, device=0)
    v.reset()
    tr = v.new_traj_out(T, select=1)
    for t in range(int(os.environ.get('AB_WARM', '30'))):
        v.rollout(T, 5, t * T, out=tr)
    torch.cuda.synchronize()
    ms = []
    for k in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v.rollout(T, 5, (100 + k) * T, out=tr)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print('instance %d: median %.3f ms, min %.3f, max %.3f  obs@%x legal@%x' % (
        i, statistics.median(ms), min(ms), max(ms), tr['obs'].data_ptr(), tr['legal'].data_ptr()), flush=True)
    del tr, v
    torch.cuda.empty_cache()
