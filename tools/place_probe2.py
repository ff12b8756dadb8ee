"""Which trajectory tensor's placement sets the k_rollout time? One VecEnv, K variants of the trajectory in which only
the named tensors are fresh allocations (the rest shared with variant 0), all kept alive, timed in interleaved rounds:

  python tools/place_probe2.py GAME WHAT K     WHAT: obs | reward | small (legal/player/action/done) | single
                                               (single: every tensor carved from ONE allocation per variant) |
                                               skew (the same, tensor k shifted by k x 352 KiB) | alt (both, alternating)
"""
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402

game, what, K = sys.argv[1], sys.argv[2], int(sys.argv[3])
g = bench.GAMES[game]
n, T = g['envs'], g['T']
v = VecEnv(game, n, seed=42, device=0)
v.reset()
base = v.new_traj_out(T, select=1)


SKEW = 352 << 10   # skew mode: tensor k starts k x 352 KiB past a 2 MiB boundary (spread over the 2 MiB page)


def carve(like, skew=0):
    """every tensor of `like` as a view of one uint8 allocation (piece k at a 2 MiB boundary + k * skew)"""
    sizes = {k: x.numel() * x.element_size() for k, x in like.items()}
    al = lambda s: (s + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    buf = torch.empty(sum(al(s + skew) for s in sizes.values()) + len(sizes) * skew + (2 << 20), dtype=torch.uint8,
                      device=like['obs'].device)
    out, off = {}, 0
    for i, (k, x) in enumerate(like.items()):
        o = off + i * skew
        out[k] = buf[o:o + sizes[k]].view(x.dtype).view(x.shape)
        off += al(sizes[k] + skew)
    return out


variants = [base]
for i in range(1, K):
    if what in ('single', 'skew'):
        variants.append(carve(base, SKEW if what == 'skew' else 0))
        continue
    if what == 'alt':    # alternate unskewed / skewed single allocations
        variants.append(carve(base, SKEW if i % 2 else 0))
        continue
    fresh = v.new_traj_out(T, select=1)
    d = dict(base)
    keys = {'obs': ['obs'], 'reward': ['reward'], 'small': ['legal', 'player', 'action', 'done']}[what]
    for k in keys:
        d[k] = fresh[k]
    del fresh
    variants.append(d)
if what in ('single', 'skew', 'alt'):
    variants[0] = carve(base, SKEW if what == 'skew' else 0)
pre = bench.precondition_launches(game, T, v)
t = 0
for c in range(pre):
    v.rollout(T, 5, t, out=variants[0])
    t += T
torch.cuda.synchronize()
res = [[] for _ in range(K)]
for rnd in range(4):
    for i, tr in enumerate(variants):
        ms = []
        for k in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            v.rollout(T, 5, t, out=tr)
            e1.record()
            t += T
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        res[i].append(statistics.median(ms))
for i, tr in enumerate(variants):
    print('%s %d: rounds %s ms  %s' % (what, i, ' '.join('%.3f' % x for x in res[i]),
                                       ' '.join('%s@%x' % (k, x.data_ptr()) for k, x in tr.items())), flush=True)
