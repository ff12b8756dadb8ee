"""Does a write-only probe of a trajectory allocation predict the rollout's time on it? K Leduc trajectory allocations
(VecEnv.new_traj_out), each timed with the real k_rollout and with the synthetic split-layout write pattern of
tools/wpat.hip (mode 0: the same six tensors, obs rows of 36 B, no game logic) writing into the same tensors.

  python tools/place_corr.py [K]
"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from rlcard_amd import VecEnv  # noqa: E402
from tools.wpat_probe import WArgs  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    game = 'leduc-holdem'
    n, T = bench.GAMES[game]['envs'], bench.GAMES[game]['T']
    lib = C.CDLL(os.path.join(ROOT, 'libwpat.so'))
    lib.wpat_run.argtypes = [C.POINTER(WArgs), C.c_int, C.c_void_p]
    v = VecEnv(game, n, seed=42, device=0)
    v.reset()
    trajs = [v.new_traj_out(T, select=1) for _ in range(K)]
    stream = torch.cuda.current_stream()
    t = 0
    for _ in range(bench.precondition_launches(game, T, v)):
        v.rollout(T, 5, t, out=trajs[0])
        t += T
    torch.cuda.synchronize()

    def probe(tr):
        b = tr['obs'].data_ptr()
        w = WArgs(b, tr['legal'].data_ptr() - b, tr['player'].data_ptr() - b, tr['action'].data_ptr() - b,
                  tr['done'].data_ptr() - b, tr['reward'].data_ptr() - b, n, n, T, 0, 0, 0, 0, 0)
        assert lib.wpat_run(C.byref(w), 26000, C.c_void_p(stream.cuda_stream)) == 0

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    roll = [[] for _ in trajs]
    prb = [[] for _ in trajs]
    for rnd in range(3):
        for i, tr in enumerate(trajs):
            for _ in range(2):
                def go():
                    v.rollout(T, 5, t, out=tr)
                roll[i].append(timed(go))
                t += T
                prb[i].append(timed(lambda: probe(tr)))
    for i in range(K):
        print('allocation %d: rollout %.3f ms  write probe %.3f ms' % (i, statistics.median(roll[i]),
                                                                       statistics.median(prb[i])), flush=True)


if __name__ == '__main__':
    main()
