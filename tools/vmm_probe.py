"""Does physical placement set the rollout's write rate? (round 5, VERDICT r04 next #1.) One VecEnv, trajectory
allocations of several kinds, all alive at once, timed in interleaved rounds after bench.py's preconditioning:
  torch    torch's caching allocator (what new_traj_out gives)
  contig   hipExtMallocWithFlags(hipDeviceMallocContiguous): physically contiguous (the slow class every time)
  vmm_id   HIP virtual memory: one VA range, CHUNK-byte physical allocations (hipMemCreate) mapped in order
  vmm_shuf the same with the chunks mapped in a random order (physically scattered at CHUNK granularity)

  VMM_KINDS=torch,vmm_shuf,.. python tools/vmm_probe.py GAME [CHUNK_MB] [ROUNDS]
"""
import ctypes as C
import os
import random
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402


class MemLocation(C.Structure):
    _fields_ = [('type', C.c_int), ('id', C.c_int)]


class AllocFlags(C.Structure):
    _fields_ = [('compressionType', C.c_ubyte), ('gpuDirectRDMACapable', C.c_ubyte), ('usage', C.c_ushort)]


class AllocProp(C.Structure):
    _fields_ = [('type', C.c_int), ('requestedHandleType', C.c_int), ('location', MemLocation),
                ('win32HandleMetaData', C.c_void_p), ('allocFlags', AllocFlags)]


class AccessDesc(C.Structure):
    _fields_ = [('location', MemLocation), ('flags', C.c_int)]


class _Dev:
    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = dict(shape=tuple(shape), typestr=typestr, data=(ptr, False), version=2,
                                             strides=None)


TYPESTR = {torch.uint8: '|u1', torch.int16: '<i2', torch.float32: '<f4', torch.int8: '|i1'}


def hip():
    h = C.CDLL('libamdhip64.so')
    vp, sz = C.c_void_p, C.c_size_t
    h.hipMemGetAllocationGranularity.argtypes = [C.POINTER(sz), C.POINTER(AllocProp), C.c_int]
    h.hipMemAddressReserve.argtypes = [C.POINTER(vp), sz, sz, vp, C.c_ulonglong]
    h.hipMemCreate.argtypes = [C.POINTER(vp), sz, C.POINTER(AllocProp), C.c_ulonglong]
    h.hipMemMap.argtypes = [vp, sz, sz, vp, C.c_ulonglong]
    h.hipMemSetAccess.argtypes = [vp, sz, C.POINTER(AccessDesc), sz]
    h.hipExtMallocWithFlags.argtypes = [C.POINTER(vp), sz, C.c_uint]
    return h


def carve(like, base):
    """the trajectory tensors of `like` laid out from device address base (each 4 KiB aligned)"""
    out, off = {}, 0
    for k, x in like.items():
        nb = x.numel() * x.element_size()
        out[k] = torch.as_tensor(_Dev(base + off, x.shape, TYPESTR[x.dtype]), device='cuda')
        off += (nb + 4095) // 4096 * 4096
    return out


def span(like):
    return sum((x.numel() * x.element_size() + 4095) // 4096 * 4096 for x in like.values())


def vmm_traj(h, like, chunk, shuffle, rng):
    prop = AllocProp(1, 0, MemLocation(1, 0), None, AllocFlags(0, 0, 0))
    g = C.c_size_t()
    assert h.hipMemGetAllocationGranularity(C.byref(g), C.byref(prop), 1) == 0, 'granularity'
    chunk = max(chunk, g.value) // g.value * g.value
    total = (span(like) + chunk - 1) // chunk * chunk
    va = C.c_void_p()
    assert h.hipMemAddressReserve(C.byref(va), total, chunk, None, 0) == 0, 'reserve'
    order = list(range(total // chunk))
    if shuffle:
        rng.shuffle(order)
    handles = [None] * len(order)
    for i in range(len(order)):   # physical chunk i created in this order, mapped at slot order[i]
        hd = C.c_void_p()
        assert h.hipMemCreate(C.byref(hd), chunk, C.byref(prop), 0) == 0, 'create'
        handles[i] = hd
        assert h.hipMemMap(C.c_void_p(va.value + order[i] * chunk), chunk, 0, hd, 0) == 0, 'map'
    acc = AccessDesc(MemLocation(1, 0), 3)
    assert h.hipMemSetAccess(va, total, C.byref(acc), 1) == 0, 'access'
    return carve(like, va.value), (va, handles, total, chunk)


def contig_traj(h, like):
    p = C.c_void_p()
    assert h.hipExtMallocWithFlags(C.byref(p), span(like), 0x4) == 0, 'contiguous'
    return carve(like, p.value), p


def main():
    game = sys.argv[1]
    chunk = int(float(sys.argv[2]) * (1 << 20)) if len(sys.argv) > 2 else 2 << 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    g = bench.GAMES[game]
    n, T = g['envs'], g['T']
    h = hip()
    rng = random.Random(7)
    v = VecEnv(game, n, seed=42, device=0)
    v.reset()
    like = v.new_traj_out(T, select=1)
    keep = []
    trajs = []
    kinds = os.environ.get('VMM_KINDS', 'torch,vmm_shuf,vmm_id,torch,vmm_shuf,vmm_id,torch,contig').split(',')
    for i, kind in enumerate(kinds):
        if kind == 'torch':
            tr = v.new_traj_out(T, select=1)
        elif kind == 'contig':
            tr, p = contig_traj(h, like)
            keep.append(p)
        else:
            tr, k = vmm_traj(h, like, chunk, kind == 'vmm_shuf', rng)
            keep.append(k)
        trajs.append(('%d_%s' % (i, kind), tr))
    print('chunk %.1f MiB, trajectory span %.2f GB' % (chunk / 2 ** 20, span(like) / 1e9), flush=True)
    t = 0
    for _ in range(bench.precondition_launches(game, T, v)):
        v.rollout(T, 5, t, out=trajs[0][1])
        t += T
    torch.cuda.synchronize()
    res = {nm: [] for nm, _ in trajs}
    for nm, tr in trajs:   # one untimed probe each first: the first touch of fresh pages is not the placement
        v.probe_traj(tr, T)
    probe = {nm: v.probe_traj(tr, T) for nm, tr in trajs}
    for rnd in range(rounds):
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
        print('round %d done' % rnd, flush=True)
    for nm, _ in trajs:
        print('%s %s: %s ms  median %.3f  probe %.3f' % (game, nm, ' '.join('%.3f' % x for x in res[nm]),
                                                       statistics.median(res[nm]), probe[nm]), flush=True)
    torch.cuda.synchronize()
    os._exit(0)   # the VMM mappings and contiguous buffers die with the process


if __name__ == '__main__':
    main()
