"""Which buffer's placement sets the k_rollout time? Several allocations of ONE kind, all kept
alive (so each is its own physical memory), timed in interleaved rounds in one process:

  python tools/place_probe.py GAME traj K    one VecEnv (MT streams + state), K trajectory buffers
  python tools/place_probe.py GAME env K     K VecEnvs (same seeds), one trajectory buffer
  python tools/place_probe.py GAME both K    K (VecEnv, trajectory) pairs

Each line: the allocation, its median launch time per round (HIP events), and the buffers' device addresses.
"""
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402

game, mode, K = sys.argv[1], sys.argv[2], int(sys.argv[3])
g = bench.GAMES[game]
n, T = g['envs'], g['T']


def make_env():
    v = VecEnv(game, n, seed=42, device=0)
    v.reset()
    return v


envs = [make_env() for _ in range(K if mode in ('env', 'both') else 1)]
trajs = [envs[0].new_traj_out(T, select=1) for _ in range(K if mode in ('traj', 'both') else 1)]
pairs = [(envs[i if len(envs) > 1 else 0], trajs[i if len(trajs) > 1 else 0]) for i in range(K)]
pre = bench.precondition_launches(game, T, envs[0])
t = {id(v): 0 for v in envs}
for v in envs:
    for c in range(pre):
        v.rollout(T, 5, c * T, out=trajs[0])
    t[id(v)] = pre * T
torch.cuda.synchronize()
res = [[] for _ in range(K)]
for rnd in range(4):
    for i, (v, tr) in enumerate(pairs):
        ms = []
        for k in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            v.rollout(T, 5, t[id(v)], out=tr)
            e1.record()
            t[id(v)] += T
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        res[i].append(statistics.median(ms))
for i, (v, tr) in enumerate(pairs):
    print('%s %d: rounds %s ms  obs@%x reward@%x done@%x' % (
        mode, i, ' '.join('%.3f' % x for x in res[i]), tr['obs'].data_ptr(), tr['reward'].data_ptr(),
        tr['done'].data_ptr()), flush=True)
