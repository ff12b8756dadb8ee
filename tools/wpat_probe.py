"""Trajectory-layout probe over HBM placements (tools/wpat.hip).

K buffers are allocated and kept alive -- torch's caching allocator (fresh segments) and hipExtMallocWithFlags with
hipDeviceMallocContiguous (physically contiguous: the slow placement every time) -- and every layout mode is
timed on every buffer in interleaved rounds, so a layout's placement spread is read off one column and layouts are
compared on the same placement along a row.

  python tools/wpat_probe.py [--n 1048576] [--T 256] [--torch 4] [--contig 2] [--modes 0,1,2,3,4] [--work 0,300]
                             [--pads 0,4160] [--lds 26000]
"""
import argparse
import ctypes as C
import os
import statistics

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: 'split', 1: 'packed', 2: 'wavemajor', 3: 'packedlane', 4: 'blockmajor', 5: 'obsonly', 6: 'split_nt0',
         7: 'work', 8: 'grouped', 9: 'packed_nt0', 10: 'torchfill', 11: 'chunks', 12: 'planes', 13: 'ddz', 14: 'ddz_nt'}


class _Dev:
    """a raw device allocation seen by torch (no copy)"""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = dict(shape=(nbytes,), typestr='|u1', data=(ptr, False), version=2,
                                             strides=None)


class WArgs(C.Structure):
    _fields_ = [('base', C.c_void_p), ('off_legal', C.c_int64), ('off_player', C.c_int64), ('off_action', C.c_int64),
                ('off_done', C.c_int64), ('off_reward', C.c_int64), ('n', C.c_int64), ('ts', C.c_int64),
                ('T', C.c_int32), ('work', C.c_int32), ('mode', C.c_int32), ('R', C.c_int32),
                ('dm', C.c_int32), ('xcd', C.c_int32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--T', type=int, default=256)
    ap.add_argument('--torch', type=int, default=4)
    ap.add_argument('--contig', type=int, default=2)
    ap.add_argument('--modes', default='0,1,2,3,4')
    ap.add_argument('--work', default='0,300')
    ap.add_argument('--pads', default='0')
    ap.add_argument('--lds', default='26000', help='LDS bytes per block (occupancy); comma list')
    ap.add_argument('--groups', default='', help='mode 8: waves per group, comma list')
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--xcd', default='0', help='1: XCD-aware block -> env-block map; comma list')
    ap.add_argument('--data', default='0', help='written data: 0 varying, 1 zeros, 2 constant, 3 per-env; comma list')
    ap.add_argument('--shapes', default='', help='extra NxT shapes timed on the same buffers, comma list')
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(ROOT, 'libwpat.so'))
    lib.wpat_run.argtypes = [C.POINTER(WArgs), C.c_int, C.c_void_p]
    hip = C.CDLL('libamdhip64.so')
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    modes = [int(x) for x in a.modes.split(',')]
    works = [int(x) for x in a.work.split(',')]
    pads = [int(x) for x in a.pads.split(',')]
    ldss = [int(x) for x in a.lds.split(',')]
    groups = [int(x) for x in a.groups.split(',')] if a.groups else [0]
    n, T = a.n, a.T
    shapes = [(n, T)] + [tuple(int(v) for v in x.split('x')) for x in a.shapes.split(',') if x]
    al = lambda s: (s + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    size = max(al(t_ * (n_ + max(pads)) * 36) + 4 * al(t_ * (n_ + max(pads))) + al(t_ * (n_ + max(pads)) * 8)
               for n_, t_ in shapes) + (2 << 20)
    if 13 in modes or 14 in modes:
        size = max(size, max(al(t_ * (n_ + max(pads)) * 901) + al(t_ * (n_ + max(pads)) * 3434) + (8 << 20)
                             for n_, t_ in shapes))
    bufs, raws = [], []
    for i in range(a.torch):
        t = torch.empty(size, dtype=torch.uint8, device=0)
        bufs.append(('torch%d' % i, t.data_ptr(), t))
    for i in range(a.contig):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), size, 0x4)
        if rc != 0:
            print('contiguous allocation %d failed: rc %d' % (i, rc), flush=True)
            break
        raws.append(p)
        bufs.append(('contig%d' % i, p.value, torch.as_tensor(_Dev(p.value, size), device='cuda')))
    print('buffers: %s, %.1f GB each; n %d T %d' % (
        ' '.join('%s@%x' % (nm, ptr) for nm, ptr, _ in bufs), size / 1e9, n, T), flush=True)
    stream = torch.cuda.current_stream()

    def launch(ptr, mode, work, pad, lds=26000, R=0, si=0, dm=0, xcd=0):
        n, T = shapes[si]
        if mode == 10:   # torch fill_ of the same bytes (default-policy stores, one linear sweep)
            views[ptr][:T * n * 12].fill_(float(work))
            return
        ts = n + pad
        if mode in (13, 14):   # DouDizhu rows: n envs = 2 per wave (grid n / 2 envs' lanes), legal after the obs rows
            ts = n + pad   # rows per step: a padded step stride (pad rows), the env count stays n
            w = WArgs(ptr, al(T * ts * 901) + (2 << 20), 0, 0, 0, 0, 32 * n, ts, T, work, mode, R, dm, xcd)   # n / 2 waves
            assert w.off_legal + T * ts * 3434 + 4096 <= size, 'ddz rows exceed the buffer'
            rc = lib.wpat_run(C.byref(w), lds, C.c_void_p(stream.cuda_stream))
            assert rc == 0, rc
            return
        if mode == 11:   # the same bytes as one sweep of R-KB wave pieces
            assert (T * n * 48) % (R * 1024 * 2048) == 0, 'chunk size must tile the sweep'
            n, T, ts = T * n * 48 // (R * 1024) * 64, 1, 0
        w = WArgs(ptr, 0, 0, 0, 0, 0, n, ts, T, work, mode, R, dm, xcd)
        o = al(T * ts * 36)
        w.off_legal, w.off_player, w.off_action, w.off_done = o, o + al(T * ts), o + 2 * al(T * ts), o + 3 * al(T * ts)
        w.off_reward = o + 4 * al(T * ts)
        rc = lib.wpat_run(C.byref(w), lds, C.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    views = {ptr: t.view(torch.float32) for _, ptr, t in bufs}
    for n_, _ in shapes:   # mode 8 spans ((w / R) T + t) R + w % R: R must divide the wave count or the last group overruns
        assert n_ % 2048 == 0, 'whole blocks, a multiple of 8 (xcd map)'
        for r in groups:
            assert r == 0 or 11 in modes or (n_ // 64) % r == 0, 'group %d does not divide %d waves' % (r, n_ // 64)
    dms = [int(x) for x in a.data.split(',')]
    xcds = [int(x) for x in a.xcd.split(',')]
    cfgs = [(m, w, p, l, r, si, dm, xcd) for si in range(len(shapes)) for l in ldss for w in works for m in modes
            for p in (pads if m in (0, 1, 3, 5, 6, 12, 13, 14) else [0]) for r in (groups if m in (8, 11) else [0])
            for dm in (dms if m != 10 else [0]) for xcd in (xcds if m != 10 else [0])]
    lab = lambda c: '%s/w%d/p%d/l%d%s%s%s' % (NAMES[c[0]][:8], c[1], c[2], c[3] // 1000,
                                             '/R%d' % c[4] if c[0] in (8, 11) else '', '/s%d' % c[5] if c[5] else '',
                                             '/d%d' % c[6] if c[6] else '') + ('/X' if c[7] else '')
    res = {}
    for nm, ptr, _ in bufs:   # warm every buffer once (first-touch)
        for c in cfgs[:1]:
            launch(ptr, *c)
    torch.cuda.synchronize()
    for rnd in range(a.rounds):
        for nm, ptr, _ in bufs:
            for c in cfgs:
                ms = []
                for k in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    launch(ptr, *c)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                res.setdefault((nm, c), []).append(statistics.median(ms))
        print('round %d done' % rnd, flush=True)
    print('%-26s' % 'config' + ''.join('%10s' % nm for nm, _, _ in bufs))
    for c in cfgs:
        print('%-26s' % lab(c) + ''.join('%10.3f' % statistics.median(res[(nm, c)]) for nm, _, _ in bufs), flush=True)
    print('shapes: %s' % ' '.join('s%d=%dx%d' % (i, a_, b_) for i, (a_, b_) in enumerate(shapes)))
    for c in cfgs:
        gb = shapes[c[5]][0] * shapes[c[5]][1] * 48 / 1e9
        v = [statistics.median(res[(nm, c)]) for nm, _, _ in bufs]
        print('%-26s min %.3f max %.3f spread %.1f %%  best %.2f TB/s (48-B rows)' % (
            lab(c), min(v), max(v), 100 * (max(v) / min(v) - 1), gb / min(v)))
    for p in raws:
        hip.hipFree(p)


if __name__ == '__main__':
    main()
