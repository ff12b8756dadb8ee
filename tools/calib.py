#!/usr/bin/env python3
"""Drive the HBM counter calibration kernels (tools/calib.hip -> tools/libcalib.so) on known byte counts; run under
rocprofv3 --pmc FETCH_SIZE and, separately, --pmc WRITE_SIZE (tools/gpu_calib.sh), then tools/calib.py --report DIR
prints counter bytes / true bytes per access shape (the correction factors DESIGN's traffic account uses).

Measurement infrastructure only."""
import csv
import collections
import ctypes as C
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
GIB = 1 << 30
ROWS = 1 << 24                     # seg64: 16 M rows of 64 B = 1 GiB
REPS = 4


def true_bytes():
    return {'k_read16': ('FETCH_SIZE', GIB), 'k_read4': ('FETCH_SIZE', GIB),
            'k_seg64': ('FETCH_SIZE', ROWS * 64 + ROWS * 4),
            'k_write16': ('WRITE_SIZE', GIB), 'k_write1': ('WRITE_SIZE', GIB), 'k_write4': ('WRITE_SIZE', GIB)}


def run():
    import torch
    L = C.CDLL(os.path.join(HERE, 'libcalib.so'))
    for f in ('calib_read16', 'calib_read4', 'calib_seg64', 'calib_write16', 'calib_write1', 'calib_write4'):
        getattr(L, f).restype = C.c_int
    dev = torch.device('cuda', 0)
    a = torch.zeros(2 * GIB + 4096, dtype=torch.uint8, device=dev)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    g = torch.Generator(device='cpu').manual_seed(1)
    off = (torch.randint(0, (2 * GIB - 64) // 4, (ROWS,), generator=g, dtype=torch.int64) * 4).to(torch.int32).to(dev)
    P = lambda t: C.c_void_p(t.data_ptr())
    torch.cuda.synchronize()
    for _ in range(REPS):
        assert L.calib_read16(P(a), GIB, P(out)) == 0
        assert L.calib_read4(P(a[GIB:]), GIB, P(out)) == 0
        assert L.calib_seg64(P(a), P(off), ROWS, P(out)) == 0
        for nt in (0, 1):        # dispatch order within a rep: write16 nt0, nt1; write1 nt0, nt1; write4 nt0, nt1
            assert L.calib_write16(P(a), GIB, nt) == 0
            assert L.calib_write1(P(a[GIB:]), GIB, nt) == 0
            assert L.calib_write4(P(a), GIB, nt) == 0
    print('calibration kernels done: %d reps' % REPS)


def report(d):
    tb = true_bytes()
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].strip()
            if k in tb and r['Counter_Name'] == tb[k][0]:
                rows[k].append((int(r.get('Dispatch_Id', 0) or 0), float(r['Counter_Value'])))
    res = {}
    for k, v in sorted(rows.items()):
        v.sort()
        vals = [x for _, x in v]
        if k.startswith('k_write'):      # alternating default / nontemporal dispatches
            for nt, sub in ((0, vals[0::2]), (1, vals[1::2])):
                res['%s%s' % (k, 'nt' if nt else '')] = dict(counter=tb[k][0], true_bytes=tb[k][1],
                                                            ratio=sum(sub) / len(sub) * 1024 / tb[k][1], n=len(sub))
        else:
            res[k] = dict(counter=tb[k][0], true_bytes=tb[k][1], ratio=sum(vals) / len(vals) * 1024 / tb[k][1],
                          n=len(vals))
    print(json.dumps(res, indent=1))
    return res


def ceiling():
    """Achievable HBM rates of plain streams (the practical ceiling beside the 8 TB/s spec): the calibration kernels
    timed with HIP events on the null stream (they launch there; each call also synchronizes), 2 GiB per dispatch, plus torch's fill_."""
    import torch
    L = C.CDLL(os.path.join(HERE, 'libcalib.so'))
    L.calib_read16.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
    for f in ('calib_write16', 'calib_write4', 'calib_write1'):
        getattr(L, f).argtypes = [C.c_void_p, C.c_int64, C.c_int]
    dev = torch.device('cuda', 0)
    a = torch.zeros(2 * GIB + 4096, dtype=torch.uint8, device=dev)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    P = lambda t: C.c_void_p(t.data_ptr())
    cases = [('read16', lambda: L.calib_read16(P(a), 2 * GIB, P(out))),
             ('write16', lambda: L.calib_write16(P(a), 2 * GIB, 0)),
             ('write16nt', lambda: L.calib_write16(P(a), 2 * GIB, 1)),
             ('write4', lambda: L.calib_write4(P(a), 2 * GIB, 0)),
             ('write4nt', lambda: L.calib_write4(P(a), 2 * GIB, 1)),
             ('write1', lambda: L.calib_write1(P(a), 2 * GIB, 0)),
             ('write1nt', lambda: L.calib_write1(P(a), 2 * GIB, 1)),
             ('torch_fill', lambda: a[:2 * GIB].fill_(7))]
    res = {}
    for name, f in cases:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[name] = {'ms': ms, 'GB/s': 2 * GIB / ms / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == '--ceiling':
        ceiling()
    elif len(sys.argv) > 2 and sys.argv[1] == '--report':
        report(sys.argv[2])
    else:
        run()
