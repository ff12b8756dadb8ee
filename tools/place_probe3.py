"""Placement spread of one library build (round 5): ONE VecEnv, K trajectory allocations from
torch's caching allocator and C physically contiguous ones (hipExtMallocWithFlags(hipDeviceMallocContiguous): the
slow placement class every time), all kept alive, the rollout timed on each in interleaved rounds after the bench's
preconditioning.

  CARDSIM_LIB=libcardsim_x.so python tools/place_probe3.py GAME [K] [C]
"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402


class _Dev:
    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = dict(shape=tuple(shape), typestr=typestr, data=(ptr, False), version=2,
                                             strides=None)


def contiguous_traj(v, T, hip, keep):
    """the trajectory tensors of new_traj_out, each in its own physically contiguous allocation"""
    out = {}
    for k, x in v.new_traj_out(T, select=1).items():
        nbytes = x.numel() * x.element_size()
        p = C.c_void_p()
        assert hip.hipExtMallocWithFlags(C.byref(p), nbytes, 0x4) == 0, 'hipExtMallocWithFlags'
        keep.append(p)
        ts = {torch.uint8: '|u1', torch.int16: '<i2', torch.float32: '<f4'}[x.dtype]
        out[k] = torch.as_tensor(_Dev(p.value, x.shape, ts), device='cuda')
        del x
    torch.cuda.empty_cache()
    return out


def main():
    game = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    Cn = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    g = bench.GAMES[game]
    n, T = g['envs'], g['T']
    hip = C.CDLL('libamdhip64.so')
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    v = VecEnv(game, n, seed=42, device=0)
    v.reset()
    keep = []
    pad = [int(x) for x in os.environ.get('PP_PAD', '').split(',') if x]   # legal, obs row strides of a padded build

    def padded(tr):
        if pad:
            tr['legal'] = torch.empty((T, n, pad[0]), dtype=torch.uint8, device=0)
            tr['obs'] = torch.empty((T, n, pad[1]), dtype=torch.uint8, device=0)
        return tr
    trajs = [('torch%d' % i, padded(v.new_traj_out(T, select=1))) for i in range(K)]
    trajs += [('contig%d' % i, contiguous_traj(v, T, hip, keep)) for i in range(Cn if not pad else 0)]
    t = 0
    for _ in range(bench.precondition_launches(game, T, v)):
        v.rollout(T, 5, t, out=trajs[0][1])
        t += T
    torch.cuda.synchronize()
    res = {nm: [] for nm, _ in trajs}
    for rnd in range(3):
        for nm, tr in trajs:
            ms = []
            for k in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                v.rollout(T, 5, t, out=tr)
                e1.record()
                t += T
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            res[nm].append(statistics.median(ms))
    lib = os.environ.get('CARDSIM_LIB', 'libcardsim.so')
    for nm, _ in trajs:
        print('%s %s %s: %s ms  median %.3f' % (lib, game, nm, ' '.join('%.3f' % x for x in res[nm]),
                                                statistics.median(res[nm])), flush=True)
    tv = [statistics.median(res[nm]) for nm, _ in trajs if nm.startswith('torch')]
    print('%s %s torch spread: min %.3f max %.3f (%.1f %%)' % (lib, game, min(tv), max(tv), 100 * (max(tv) / min(tv) - 1)),
          flush=True)
    del trajs
    torch.cuda.synchronize()
    for p in keep:
        hip.hipFree(p)


if __name__ == '__main__':
    main()
