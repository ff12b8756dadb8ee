"""Throughput of the post-rollout kernels (cs_transitions, cs_legal_lists, cs_action_features) on bench-sized
trajectories; one JSON line per measurement.  python tools/bench_traj.py"""
import json
import sys

import torch

sys.path.insert(0, '.')
from rlcard_amd import VecEnv  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for game, n in (('leduc-holdem', 1 << 20), ('limit-holdem', 262144), ('doudizhu', 65536)):
    T = 16
    v = VecEnv(game, n, seed=42)
    v.reset()
    tr = v.rollout(T, policy_seed=5)
    rows = T * n
    ms = timed(lambda: v.transitions(tr))
    # bytes: player + done + reward in, next_t + end_t + reward + done + ret out
    B = rows * (1 + 1 + 4 * v.num_players + 4 + 4 + 4 + 1 + 4)
    print(json.dumps(dict(kernel='cs_transitions', game=game, rows=rows, ms=ms, rows_per_s=rows / ms * 1e3,
                          gbs=B / ms / 1e6)), flush=True)
    counts, offsets, ids = v.legal_lists(tr['legal'])
    ms = timed(lambda: v.legal_lists(tr['legal']))   # includes the host read of the total between the two passes
    B = rows * (v.legal_bytes * 2 + 4 + 8) + ids.numel() * 4
    print(json.dumps(dict(kernel='cs_legal_lists', game=game, rows=rows, ids=int(ids.numel()), ms=ms,
                          rows_per_s=rows / ms * 1e3, gbs=B / ms / 1e6)), flush=True)
    acts = tr['action'].reshape(-1).to(torch.int32)
    ms = timed(lambda: v.action_features(acts))
    B = rows * (4 + v.info.action_feature_dim)
    print(json.dumps(dict(kernel='cs_action_features', game=game, rows=rows, ms=ms, gbs=B / ms / 1e6)), flush=True)
    del v, tr
    torch.cuda.empty_cache()
