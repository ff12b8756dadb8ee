"""Does the last, partial round of waves cost a full round? k_rollout time per env-step at env counts that fill the
resident wave slots a whole number of times and at the bench's count in between.

  python tools/tail_probe.py GAME T N1,N2,... [INST]

Leduc at 6 waves per SIMD holds 256 CUs x 24 = 6 144 waves = 393 216 envs at once: 2^20 envs are 2.67 rounds of
waves, 786 432 / 1 179 648 exactly 2 / 3. If a round's time is set by each wave's own latency, 2^20 costs what 3 rounds
cost; if it is set by HBM bandwidth, time follows the env count. Each N gets INST (2) fresh trajectory allocations,
chosen by VecEnv.new_traj_out (placement), 40 warm-up launches and 10 timed ones each."""
import statistics
import sys

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402

game, T = sys.argv[1], int(sys.argv[2])
ns = [int(x) for x in sys.argv[3].split(',')]
inst = int(sys.argv[4]) if len(sys.argv) > 4 else 2
for n in ns:
    per = []
    for i in range(inst):
        v = VecEnv(game, n, seed=42 + i, device=0)
        v.reset()
        tr = v.new_traj_out(T)
        for k in range(40):
            v.rollout(T, policy_seed=1, t0=k * T, out=tr)
        torch.cuda.synchronize()
        ts = []
        for k in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(torch.cuda.current_stream())
            v.rollout(T, policy_seed=1, t0=(40 + k) * T, out=tr)
            b.record(torch.cuda.current_stream())
            b.synchronize()
            ts.append(a.elapsed_time(b))
        per.append(statistics.median(ts))
        del tr, v
        torch.cuda.empty_cache()
    ms = statistics.median(per)
    print('%s n=%d T=%d: %.3f ms per launch (allocations %s), %.3f ns per env-step' %
          (game, n, T, ms, ' '.join('%.3f' % x for x in per), ms * 1e6 / (n * T)), flush=True)
