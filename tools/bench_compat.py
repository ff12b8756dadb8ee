#!/usr/bin/env python3
"""Single-env compat path (rlcard_amd.make(...)) speed: env.run(is_training=False) with RandomAgent, exactly as the
reference's examples/run_random.py drives it, plus the env-only loop (reset / step a uniform legal id) -- the same
two loops tools/ref_cpu_baseline.py times on the reference (profiles/ref_cpu_baseline.json). One process, one env.

  python tools/bench_compat.py [--seconds 5] [--games leduc-holdem ...]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seconds', type=float, default=5.0)
    ap.add_argument('--games', nargs='*', default=['blackjack', 'leduc-holdem', 'limit-holdem', 'doudizhu',
                                                     'no-limit-holdem'])
    args = ap.parse_args()
    import rlcard_amd
    from rlcard_amd.agents import RandomAgent
    from rlcard_amd.utils import set_seed
    ref = {}
    try:
        with open(os.path.join(ROOT, 'profiles', 'ref_cpu_baseline.json')) as f:
            ref = json.load(f)['games']
    except (OSError, ValueError, KeyError):
        pass
    for g in args.games:
        env = rlcard_amd.make(g, config={'seed': 42})
        set_seed(42)
        env.set_agents([RandomAgent(num_actions=env.num_actions) for _ in range(env.num_players)])
        env.run(is_training=False)                      # warm-up (first launches, allocations)
        t0, s0 = time.perf_counter(), env.timestep
        while time.perf_counter() - t0 < args.seconds:
            env.run(is_training=False)
        run_rate = (env.timestep - s0) / (time.perf_counter() - t0)
        rng = random.Random(42)
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.seconds:
            state, _ = env.reset()
            while not env.is_over():
                state, _ = env.step(rng.choice(list(state['legal_actions'].keys())))
                steps += 1
        env_rate = steps / (time.perf_counter() - t0)
        r = ref.get(g, {})
        print(json.dumps({'game': g, 'run_steps_per_s': run_rate, 'env_only_steps_per_s': env_rate,
                          'reference_run_one_core': r.get('one_core', {}).get('value'),
                          'reference_env_only_one_core': r.get('env_only_one_core', {}).get('value')}), flush=True)


if __name__ == '__main__':
    main()
