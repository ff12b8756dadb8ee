"""Plain HBM write / read rates of K separate allocations of the same size, all kept alive, timed in interleaved rounds
(torch fill_ = streaming 16-B stores; sum = streaming reads). Tells whether the per-allocation k_rollout times
(tools/place_probe*.py) are a property of where the buffer landed in HBM, independent of the kernel:

  python tools/fill_probe.py [GiB per buffer] [K]
"""
import statistics
import sys

import torch

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 9.0
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = int(gib * (1 << 30))
bufs = [torch.empty(n, dtype=torch.uint8, device=0) for _ in range(K)]
f32 = [b.view(torch.float32) for b in bufs]
res_w = [[] for _ in range(K)]
res_r = [[] for _ in range(K)]
for b in f32:
    b.fill_(1.0)
torch.cuda.synchronize()
for rnd in range(4):
    for i, b in enumerate(f32):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        b.fill_(float(rnd))
        e1.record()
        s = b.sum()
        e2.record()
        torch.cuda.synchronize()
        res_w[i].append(n / (e0.elapsed_time(e1) * 1e-3) / 1e12)
        res_r[i].append(n / (e1.elapsed_time(e2) * 1e-3) / 1e12)
        del s
for i in range(K):
    print('buffer %d @%x: fill %s TB/s  sum %s TB/s' % (
        i, bufs[i].data_ptr(), ' '.join('%.2f' % x for x in res_w[i]), ' '.join('%.2f' % x for x in res_r[i])),
        flush=True)
