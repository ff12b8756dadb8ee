"""Timing of chance-sampling CFR on Leduc (cs_cfr_train) on the GPU, next to the CPU oracle (oracle/or_cfr.c).
  python tools/bench_cfr.py            -> one JSON line per configuration
B = envs = deals per player per iteration (B = 1 is the reference agent's algorithm); tree walks/s counts one full
betting-tree traversal per (deal, player)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]
from rlcard_amd import VecEnv, seeding  # noqa: E402
from rlcard_amd.agents import CFRAgent  # noqa: E402


def gpu(B, K):
    agent = CFRAgent(VecEnv('leduc-holdem', B, seed=0))
    agent.train(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.train(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return dict(engine='gpu', deals_per_player=B, iterations=K, s=el, iterations_per_s=K / el,
                tree_walks_per_s=2 * B * K / el)


def cpu(B, K):
    import oracle_lib
    keys, lens = seeding.seed_keys(range(B))
    c = oracle_lib.CFR(keys, lens)
    t0 = time.perf_counter()
    c.train(K)
    el = time.perf_counter() - t0
    return dict(engine='cpu oracle (1 core)', deals_per_player=B, iterations=K, s=el, iterations_per_s=K / el,
                tree_walks_per_s=2 * B * K / el)


if __name__ == '__main__':
    for r in (gpu(1, 2000), cpu(1, 2000), gpu(4096, 20), gpu(262144, 5), cpu(256, 20)):
        print(json.dumps(r), flush=True)
