#!/usr/bin/env python3
"""Benchmark of the env.step hot path (BASELINE.json): env-steps/s (whole node) + achieved HBM GB/s.

One bench "step" = one cs_rollout launch: T fused lockstep env steps (default Leduc 128, the others 64) of the
uniform-random legal policy with auto-reset over every env of the rank's shard, writing the full trajectory (obs,
legal mask, player, action, reward, done) to HBM.
N>1: one process per GPU (torchrun), rank r owns envs [r*N, (r+1)*N) seeded 42 + global index -- the envs are
independent, so there is no data-path collective (weak scaling); --gather adds the optional RCCL all-gather of the
trajectory shards (timed separately, reported under "gather").

  python bench.py [--gpus N] [--steps K] [--warmup W] [--game leduc-holdem] [--envs N_PER_GPU] [--T STEPS]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (chip-level parameters)

# per game: default envs per GPU (BASELINE.json configs), default fused steps per launch, packed state bytes per env
# read + written once per launch (state words + the RNG control word), and the expected tempered-u32 MT19937 draws
# per env-step under random play (exact acceptance rates of random_interval x random-play game lengths).
# Fused steps per launch, measured on one box: Leduc 256 vs 128 +3 % (T >= 256), Limit / No-limit 128
# vs 64 +2.5 / +3 %, DouDizhu 128 vs 64 -7 %.
GAMES = {
    'leduc-holdem': dict(envs=1 << 20, T=256, state_bytes=2 * 4 + 4, draws_per_step=2.83),
    'limit-holdem': dict(envs=262144, T=128, state_bytes=12 * 4 + 4, draws_per_step=24.5),
    'blackjack': dict(envs=1 << 20, T=64, state_bytes=20 * 4 + 4, draws_per_step=57.0),
    'doudizhu': dict(envs=65536, T=64, state_bytes=20 * 4 + 4, draws_per_step=1.21),
    # not a BASELINE config; draws/step counted on the oracle (4096 envs x 256 random steps)
    'no-limit-holdem': dict(envs=262144, T=128, state_bytes=4 * 4 + 4, draws_per_step=26.3),
}


def alg_bytes_per_env_step(info, T, game):
    """B = O + ceil(A/8) + 4P + 1 (done) + 1 (player) + a + 2S/T + R, R = 8 B x draws/step
    (each MT word is read once by its lane, and each 624-word block is written and re-read once by the refill)."""
    g = GAMES[game]
    a = 1 if info.num_actions <= 256 else 2
    return (info.obs_dim + (info.num_actions + 7) // 8 + 4 * info.num_players + 1 + 1 + a
            + 2.0 * g['state_bytes'] / T + 8.0 * g['draws_per_step'])


def cpu_baseline(game, budget_s=12.0):
    """The CPU oracle (C restatement, oracle/) timed on this host, one core, on a bounded sample of the same
    workload (same env seeds, same policy)."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import oracle_lib
    from rlcard_amd import seeding
    n_s, T_s = (256, 8) if game == 'doudizhu' else (8192, 32)   # one chunk well under the budget
    keys, lens = seeding.seed_keys(range(42, 42 + n_s))
    b = oracle_lib.Batch(game, n_s, keys, lens)
    b.reset()
    steps, t0, chunk = 0, time.perf_counter(), 0
    while True:
        b.rollout(T_s, 5, chunk * T_s, 0)
        steps += n_s * T_s
        chunk += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return dict(value=steps / el, unit='env-steps/s', cores=1, kind='port',
                sample='%s: %d envs (seeds 42..%d) x %d lockstep steps, uniform-legal Philox policy, %.1f s, '
                       'oracle/liboracle.so scalar C' % (game, n_s, 41 + n_s, steps // n_s, el))


def measured_traffic(game, envs, T):
    """HBM bytes per k_rollout launch of this configuration from the committed rocprofv3 PMC profile
    (profiles/traffic.json, written by tools/pmc_traffic.py), or None."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'traffic.json')) as f:
            e = json.load(f).get('%s:%d:%d' % (game, envs, T))
    except (OSError, ValueError):
        return None
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--game', default='leduc-holdem', choices=sorted(GAMES))
    ap.add_argument('--envs', type=int, default=0, help='envs per GPU (default: the BASELINE config)')
    ap.add_argument('--T', type=int, default=0, help='fused env steps per launch (default: per game, GAMES)')
    ap.add_argument('--gather', action='store_true', help='also all-gather trajectory shards over RCCL')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-precondition', dest='precondition', action='store_false',
                    help='time from freshly seeded streams (optimistic: no MT block refills yet)')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from rlcard_amd.shard import ShardedVecEnv, gather_traj, new_gathered

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit('run N>1 under torchrun: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N')
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    def barrier():
        if world > 1:
            dist.barrier()

    game = args.game
    T = args.T or GAMES[game]['T']   # measured: longer launches amortise the state / staging traffic
    N = args.envs or GAMES[game]['envs']
    env = ShardedVecEnv(game, N, rank, seed=42, device=local)   # global envs [rank*N, (rank+1)*N)
    env.reset()
    traj = env.new_traj_out(T)
    gathered = new_gathered(traj, world) if args.gather and world > 1 else None

    stream = torch.cuda.current_stream()
    t_launch = 0
    # Precondition: every env's MT19937 stream starts at position 0 after seeding, so no env refills a block until
    # ~624 draws in; run (untimed) until each stream has crossed two blocks on average, so the timed launches see the
    # steady-state refill rate (measured on Leduc: launches are ~15-25 % slower once the refills start).
    pre = int(math.ceil(2 * 624 / (GAMES[game]['draws_per_step'] * T))) if args.precondition else 0
    for w in range(pre):
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        t_launch += 1
    for w in range(args.warmup):
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        t_launch += 1
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        ev[k][1].record(stream)
        t_launch += 1
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    gather_info = None
    if gathered is not None:
        torch.cuda.synchronize()
        barrier()
        g0 = time.perf_counter()
        for k in range(args.steps):
            env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
            t_launch += 1
            gather_traj(traj, gathered)
        torch.cuda.synchronize()
        barrier()
        gel = time.perf_counter() - g0
        gather_info = dict(ms_per_step=1e3 * gel / args.steps,
                           value=world * N * T * args.steps / gel,
                           bytes_per_rank_per_step=sum(v.numel() * v.element_size() for v in traj.values()))

    if world > 1:
        t = torch.tensor([elapsed], device='cuda', dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if gather_info is not None:
            t = torch.tensor([gather_info['ms_per_step']], device='cuda', dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            gather_info['ms_per_step'] = float(t.item())
            gather_info['value'] = world * N * T * 1e3 / gather_info['ms_per_step']

    if rank == 0:
        env_steps = world * N * T * args.steps
        value = env_steps / elapsed
        B = alg_bytes_per_env_step(env.info, T, game)
        achieved = B * N * T / (kernel_ms * 1e-3) / 1e9
        line = {
            'metric': 'env-steps/s (whole node) + achieved HBM GB/s, %s %d envs/GPU' % (game, N),
            'value': value,
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': 1e3 * elapsed / args.steps,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic: env i seeded 42+i (reference seeding), uniform-random legal policy (Philox); '
                    '%d untimed preconditioning launches (steady-state MT refill rate)' % pre,
            'config': {'workload': '%s, %d envs per GPU, %d fused lockstep steps per launch, auto-reset, full '
                                   'trajectory to HBM' % (game, N, T),
                       'game': game, 'envs_per_gpu': N, 'global_envs': world * N, 'fused_steps': T,
                       'parallelism': 'env-shard x%d (no data-path collective)' % world},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                         'alg_bytes_per_env_step': B, 'kernel_ms_per_launch': kernel_ms,
                         'kernel': 'k_rollout<%s>' % game},
        }
        tr = measured_traffic(game, N, T)
        if tr is not None:   # per launch, like `achieved`; from the profile of this exact configuration
            line['roofline']['traffic'] = tr['bytes_per_launch']
            line['roofline']['traffic_source'] = tr['source']
            line['roofline']['alg_bytes_per_launch'] = B * N * T
        if gather_info is not None:
            line['gather'] = gather_info
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(game)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
