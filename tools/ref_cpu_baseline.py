#!/usr/bin/env python3
"""The reference's own CPU path timed on this container's cores (SURVEY 8(d) "CPU baseline timing").

Runs pmcgannon22/rlcard's `env.run(is_training=False)` with `RandomAgent` exactly as examples/run_random.py:12-27
does (env seed, set_seed, one RandomAgent per player), repeatedly, for a fixed wall budget per process:
  * one process per core of os.sched_getaffinity(0), each with its own env seed (42 + process index),
    aggregate env-steps/s = sum of Env.timestep (envs/env.py:81 counts every step) / wall;
  * the same on one core;
  * the env-only loop (uniform legal id via random.choice, no agent) on one core.
The reference exists only in the build container (/root/reference), never on the GPU box, so bench.py cannot time it
there: this script writes profiles/ref_cpu_baseline.json (host, cores, numbers, provenance) and bench.py reports it as
`reference_cpu` next to its own `cpu_baseline` (the C port, timed on the GPU box's host).

Test / measurement infrastructure only: nothing in rlcard_amd/ imports it.

  python tools/ref_cpu_baseline.py [--seconds 10] [--games leduc-holdem ...]
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))

GAMES = ['blackjack', 'leduc-holdem', 'limit-holdem', 'doudizhu', 'no-limit-holdem']


def _use_reference_copy():
    """sys.path for the writable reference copy the parent set up (gen_golden.setup_reference)."""
    import typing
    import gen_golden
    if not hasattr(typing, 'Self'):
        typing.Self = typing.Any
    sys.path.insert(0, os.path.join(gen_golden.WORK, 'stubs'))
    sys.path.insert(0, gen_golden.WORK)
    sys.dont_write_bytecode = True


def _worker(game, seed, seconds, mode, q):
    _use_reference_copy()
    import random
    import rlcard
    from rlcard.agents import RandomAgent
    from rlcard.utils import set_seed
    env = rlcard.make(game, config={'seed': seed})
    set_seed(seed)
    rng = random.Random(seed)
    if mode == 'run':
        env.set_agents([RandomAgent(num_actions=env.num_actions) for _ in range(env.num_players)])
    steps, games = 0, 0
    t0 = time.perf_counter()
    while True:
        if mode == 'run':
            env.run(is_training=False)
            steps = env.timestep                # Env.timestep is cumulative: never reset by Env.reset
        else:                                   # env-only: reset + step a uniform legal id until over
            state, _ = env.reset()
            n = 0
            while not env.is_over():
                state, _ = env.step(rng.choice(list(state['legal_actions'].keys())))
                n += 1
            steps += n
        games += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    q.put((steps, games, el))


def measure(game, procs, seconds, mode):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(game, 42 + i, seconds, mode, q)) for i in range(procs)]
    t0 = time.perf_counter()
    for p in ps:
        p.start()
    res = [q.get(timeout=seconds * 10 + 300) for _ in ps]
    for p in ps:
        p.join()
    wall = max(r[2] for r in res)
    steps = sum(r[0] for r in res)
    return dict(value=steps / wall, unit='env-steps/s', processes=procs, env_steps=steps,
                games=sum(r[1] for r in res), seconds=wall, launch_s=time.perf_counter() - t0)


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seconds', type=float, default=10.0)
    ap.add_argument('--games', nargs='*', default=GAMES)
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'ref_cpu_baseline.json'))
    args = ap.parse_args()
    import gen_golden
    gen_golden.setup_reference()                # one writable copy, before any worker starts
    cores = len(os.sched_getaffinity(0))
    out = {'host': {'cpu': cpu_model(), 'cores': cores, 'python': platform.python_version(),
                    'machine': 'build container (no GPU); the reference does not exist on the GPU box'},
           'method': 'rlcard env.run(is_training=False) + RandomAgent per player as examples/run_random.py:12-27 '
                     '(config {"seed": 42 + process}, set_seed), repeated for %.0f s per process; env-steps = '
                     'Env.timestep (envs/env.py:81); env_only = reset/step with a uniform legal id, no agent'
                     % args.seconds,
           'script': 'tools/ref_cpu_baseline.py', 'date': time.strftime('%Y-%m-%d %H:%M:%S'), 'games': {}}
    for g in args.games:
        r = {'all_cores': measure(g, cores, args.seconds, 'run'),
             'one_core': measure(g, 1, args.seconds, 'run'),
             'env_only_one_core': measure(g, 1, args.seconds, 'env')}
        out['games'][g] = r
        print(g, {k: round(v['value']) for k, v in r.items()}, flush=True)
    with open(args.out, 'w') as f:
        json.dump(out, f, indent=1)
    print('wrote', args.out)


if __name__ == '__main__':
    main()
