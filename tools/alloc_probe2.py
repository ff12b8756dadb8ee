"""Allocation-variance probe, part 2: the same rollout timed with its trajectory buffers from the torch caching allocator
and from hipExtMallocWithFlags(hipDeviceMallocContiguous), interleaved over fresh allocations in ONE process.
  python tools/alloc_probe2.py GAME N T [instances]"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402

game, n, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
inst = int(sys.argv[4]) if len(sys.argv) > 4 else 4
hip = C.CDLL('libamdhip64.so')
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipFree.argtypes = [C.c_void_p]


class Raw:
    """a device allocation seen by torch through __cuda_array_interface__ (no copy)"""

    def __init__(self, shape, typestr, itemsize, flags):
        nbytes = itemsize
        for s in shape:
            nbytes *= s
        self.p = C.c_void_p()
        assert hip.hipExtMallocWithFlags(C.byref(self.p), nbytes, flags) == 0, 'hipExtMallocWithFlags'
        self.__cuda_array_interface__ = dict(shape=tuple(shape), typestr=typestr, data=(self.p.value, False),
                                             version=2, strides=None)

    def free(self):
        hip.hipFree(self.p)


def raw_traj(v, T, flags):
    keep = []

    def mk(shape, typestr, itemsize, dtype):
        r = Raw(shape, typestr, itemsize, flags)
        keep.append(r)
        return torch.as_tensor(r, device='cuda')
    N = v.num_envs
    o = dict(obs=mk((T, N, v.obs_dim), '|u1', 1, torch.uint8), legal=mk((T, N, v.legal_bytes), '|u1', 1, torch.uint8),
             player=mk((T, N), '|u1', 1, torch.uint8), reward=mk((T, N, v.num_players), '<f4', 4, torch.float32),
             done=mk((T, N), '|u1', 1, torch.uint8),
             action=mk((T, N), '|u1' if v.action_dtype == torch.uint8 else '<i2', 1 if v.action_dtype == torch.uint8 else 2,
                       v.action_dtype))
    return o, keep


def time_it(v, tr, t, k=10):
    ms = []
    for _ in range(k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v.rollout(T, 5, t, out=tr)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        t += T
    return statistics.median(ms), t


for i in range(inst):
    v = VecEnv(game, n, seed=42 + i, device=0)
    v.reset()
    order = os.environ.get('AP_ORDER', 'torch,contiguous,hipdefault').split(',')
    bufs, keep = {}, []
    for name in order:   # allocated in this order
        if name == 'torch':
            bufs[name] = v.new_traj_out(T, select=1)
        else:
            bufs[name], k = raw_traj(v, T, 0x4 if name == 'contiguous' else 0x0)
            keep += k
    tt = bufs[order[0]]
    t = 0
    for _ in range(int(os.environ.get('AB_WARM', '20'))):
        v.rollout(T, 5, t, out=tt)
        t += T
    torch.cuda.synchronize()
    res = {name: [] for name in order}
    for rnd in range(3):
        for name in order:
            m, t = time_it(v, bufs[name], t)
            res[name].append(m)
    print('instance %d: ' % i + '  '.join('%s %.3f' % (k, statistics.median(x)) for k, x in res.items()), flush=True)
    del v, tt, bufs
    torch.cuda.synchronize()
    for r in keep:
        r.free()
    torch.cuda.empty_cache()
