#!/usr/bin/env python3
"""cProfile of the compat env-only loop (rlcard_amd.make + reset/step), to split host overhead from the GPU round trip."""
import cProfile
import os
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rlcard_amd  # noqa: E402

game = sys.argv[1] if len(sys.argv) > 1 else 'leduc-holdem'
env = rlcard_amd.make(game, config={'seed': 42})
rng = random.Random(0)


def loop(n):
    steps = 0
    while steps < n:
        state, _ = env.reset()
        while not env.is_over():
            state, _ = env.step(rng.choice(list(state['legal_actions'].keys())))
            steps += 1


loop(200)
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
loop(3000)
pr.disable()
print('%.1f us/step under cProfile' % ((time.perf_counter() - t) / 3000 * 1e6))
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
