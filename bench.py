#!/usr/bin/env python3
"""Benchmark of the env.step hot path (BASELINE.json): env-steps/s (whole node) + achieved HBM GB/s.

One bench "step" = one cs_rollout launch: T fused lockstep env steps (defaults per game in GAMES: Leduc, Limit and
No-limit 256, DouDizhu / Blackjack 64) of the uniform-random legal policy with auto-reset over every env of the
rank's shard, writing the full trajectory (obs, legal mask, player, action, reward, done) to HBM.
N>1: one process per GPU (torchrun), rank r owns envs [r*N, (r+1)*N) seeded 42 + global index -- the envs are
independent, so the timed loop has no data-path collective (weak scaling, `value`). A second timed phase adds the
one real exchange, returning the trajectory shards to their consumer: point-to-point RCCL into rank 0 over xGMI
("gather") and the all-gather into every rank that BASELINE config 5 names ("allgather"); both by default.

A third phase times the same workload with the engine's fast RNG mode (cs_config.rng_mode = CS_RNG_PHILOX: Philox
byte stream instead of numpy's MT19937, so NOT the reference's deals) and reports it under "rng_philox" -- `value`
is always the reference-compatible MT19937 stream.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--game leduc-holdem] [--envs N_PER_GPU] [--T STEPS]
"""
import argparse
import hashlib
import json
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (chip-level parameters)
MT_N = 624              # words per MT19937 block

# per game: default envs per GPU (BASELINE.json configs), default fused steps per launch, the expected tempered-u32
# MT19937 draws per env-step under random play (exact acceptance rates of random_interval x random-play game lengths). The
# stream geometry (draws before the first refill, draws per refill) comes from the built library (VecEnv.rng_period:
# the byte ring's CS_RING_SLOTS, or DouDizhu's two-block word window), see precondition_launches.
# Fused steps per launch, measured on one box: Leduc 256 vs 128 +3 % (T >= 256), 512 vs 256 -9 %;
# Limit / No-limit 512 vs 256 +1.5 % (round 3; 256 vs 128 +1.5 / +2 %), DouDizhu 128 vs 64 -5 %, 32 vs 64 -2 % (two-env
# kernel), Blackjack 128 vs 64 +2 %.
GAMES = {
    'leduc-holdem': dict(envs=1 << 20, T=256, draws_per_step=2.83),
    'limit-holdem': dict(envs=262144, T=512, draws_per_step=24.5),
    'blackjack': dict(envs=1 << 20, T=128, draws_per_step=57.0),
    'doudizhu': dict(envs=65536, T=64, draws_per_step=1.21),
    # not a BASELINE config; draws/step counted on the oracle (4096 envs x 256 random steps)
    'no-limit-holdem': dict(envs=262144, T=512, draws_per_step=26.3),
}
TIMED_TARGET_S = 2.0     # default --steps: enough launches for >= ~2 s of timed region (box variance, SMI sampler)


def state_bytes(info):
    """Packed state bytes per env read + written once per launch: the built library's state words (hold'em: the game
    words + the deal queue, whatever depth was compiled) + the RNG control word."""
    return 4 * info.state_words + 4


def alg_bytes_per_env_step(info, T, game):
    """B = O + ceil(A/8) + 4P + 1 (done) + 1 (player) + a + 2S/T + R, R = 8 B x draws/step
    (each MT word is read once by its lane, and each 624-word block is written and re-read once by the refill)."""
    g = GAMES[game]
    a = 1 if info.num_actions <= 256 else 2
    return (info.obs_dim + (info.num_actions + 7) // 8 + 4 * info.num_players + 1 + 1 + a
            + 2.0 * state_bytes(info) / T + 8.0 * g['draws_per_step'])


def alg_bytes_philox(info, T, game):
    """SURVEY 8(d) with R = 0 (Philox mode): the outputs and the packed state only."""
    return alg_bytes_per_env_step(info, T, game) - 8.0 * GAMES[game]['draws_per_step']


def precondition_launches(game, T, vec):
    """Untimed launches so that the timed ones run at the steady-state refill rate: a freshly seeded stream refills
    nothing for its first draws (VecEnv.rng_first_refill, the worst case over envs); run until the average env has
    also passed two refills (VecEnv.rng_per_refill), the geometry of the library actually built."""
    g = GAMES[game]
    return int(math.ceil((vec.rng_first_refill + 2 * vec.rng_per_refill) / (g['draws_per_step'] * T)))


def _code_only(text):
    """C++ source without its comments and blank space (a comment edit does not change the kernels)"""
    text = re.sub(r'/\*.*?\*/', ' ', text, flags=re.S)
    text = re.sub(r'//[^\n]*', '', text)
    return '\n'.join(' '.join(line.split()) for line in text.split('\n') if line.strip())


def kernel_source_digest():
    """sha256 (16 hex) of the engine's sources, comments stripped: a traffic profile is only reported for the kernels
    it measured."""
    d = os.path.join(ROOT, 'rlcard_amd', 'csrc')
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith(('.hip', '.h', '.cpp', '.bin')) or f == 'Makefile':
            h.update(f.encode())
            with open(os.path.join(d, f), 'rb') as fh:
                data = fh.read()
            h.update(_code_only(data.decode()).encode() if f.endswith(('.hip', '.h', '.cpp')) else data)
    return h.hexdigest()[:16]


def product_library():
    """The engine library this process loads, and whether it is the product build: rlcard_amd/libcardsim.so, which
    the Makefile builds with no -D options (A/B and profiling variants are libcardsim_<name>.so, loaded through
    CARDSIM_LIB). The kernel-source digest only identifies the product build's kernels, so a line measured on any other
    library cites no traffic profile and says so."""
    name = os.environ.get('CARDSIM_LIB', 'libcardsim.so')
    return name, name == 'libcardsim.so'


def measured_traffic(game, envs, T, kernel_ms=None):
    """HBM bytes per k_rollout launch of this configuration from the committed rocprofv3 profiles
    (profiles/traffic.json, written by tools/pmc_traffic.py), or None. An entry is one profile or a list of them
    (one per HBM placement class); the one measured on these kernel sources whose kernel time is closest to
    `kernel_ms` is returned. Entries measured on other kernel sources are returned with stale=True and are not used
    as `traffic`."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'traffic.json')) as f:
            e = json.load(f).get('%s:%d:%d' % (game, envs, T))
    except (OSError, ValueError):
        return None
    if e is None:
        return None
    digest = kernel_source_digest()
    es = [dict(x, stale=x.get('src_sha16') != digest) for x in (e if isinstance(e, list) else [e])]
    fresh = [x for x in es if not x['stale']] or es
    if kernel_ms is not None:
        fresh.sort(key=lambda x: abs(x.get('kernel_ns_timed_mean', 0) / 1e6 - kernel_ms))
    return fresh[0]


def under_profiler():
    """True when a profiler's library is preloaded into this process (rocprofv3 sets LD_PRELOAD / ROCPROF_*): then
    no child process may be started from here -- the amd-smi sampler's `env -> python3` hop would be an exec after
    the preloaded library initialised the GPU."""
    pre = os.environ.get('LD_PRELOAD', '')
    return 'rocprof' in pre or 'roctracer' in pre or any(k.startswith(('ROCPROF', 'ROCP_')) for k in os.environ)


def _cpu_worker(game, first, n, T, budget_s, q):
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import oracle_lib
    from rlcard_amd import seeding
    keys, lens = seeding.seed_keys(range(42 + first, 42 + first + n))
    b = oracle_lib.Batch(game, n, keys, lens)
    b.reset()
    steps, chunk = 0, 0
    t0 = time.perf_counter()
    while True:
        b.rollout(T, 5, chunk * T, first)
        steps += n * T
        chunk += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    q.put((steps, el))


def cpu_cores():
    """Host cores this process may use: the affinity set, capped by the job's CPU share where the launcher states
    one (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes, whose os.cpu_count() is the whole machine)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get('OMP_NUM_THREADS')
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline(game, budget_s=10.0):
    """The CPU oracle (C restatement, oracle/) on this host: one process per core, each on its own slice of the same
    workload (env seeds 42 + global id, same Philox policy), for a bounded wall budget."""
    import multiprocessing as mp
    cores = cpu_cores()
    n_s, T_s = (64, 8) if game == 'doudizhu' else (4096, 32)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_cpu_worker, args=(game, i * n_s, n_s, T_s, budget_s, q)) for i in range(cores)]
    for p in ps:
        p.start()
    res = [q.get(timeout=budget_s * 20 + 120) for _ in ps]
    for p in ps:
        p.join()
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return dict(value=steps / wall, unit='env-steps/s', cores=cores, kind='port',
                sample='%s: %d processes x %d envs (seeds 42 + global id) x lockstep chunks of %d steps, '
                       'uniform-legal Philox policy, %.1f s wall, oracle/liboracle.so scalar C, one process per '
                       'core' % (game, cores, n_s, T_s, wall))


def reference_cpu(game):
    """The reference's own env.run + RandomAgent, measured in the build container by tools/ref_cpu_baseline.py (the
    reference does not exist on the GPU box); None when that profile is absent."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'ref_cpu_baseline.json')) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    g = d.get('games', {}).get(game)
    if g is None:
        return None
    return dict(value=g['all_cores']['value'], unit='env-steps/s', cores=g['all_cores']['processes'],
                one_core=g['one_core']['value'], env_only_one_core=g['env_only_one_core']['value'],
                host=d['host']['cpu'], where=d['host']['machine'], date=d['date'],
                source='profiles/ref_cpu_baseline.json (%s)' % d['script'], method=d['method'])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=0,
                    help='timed launches (default: enough for ~%.0f s of timed region, at least 20)' % TIMED_TARGET_S)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--game', default='leduc-holdem', choices=sorted(GAMES))
    ap.add_argument('--envs', type=int, default=0, help='envs per GPU (default: the BASELINE config)')
    ap.add_argument('--T', type=int, default=0, help='fused env steps per launch (default: per game, GAMES)')
    ap.add_argument('--gather', choices=('both', 'rank0', 'all', 'none'), default='both',
                    help='N>1: trajectory exchange timed after the main loop: every shard into rank 0 ("gather"), '
                         'all-gathered into every rank (BASELINE config 5, "allgather"), or both (default)')
    ap.add_argument('--gather-steps', type=int, default=5)
    ap.add_argument('--recv-budget-gb', type=float, default=32.0,
                    help='N>1: receive-buffer budget per GPU of the exchange (GiB); the trajectory moves in T-slices '
                         'that fit it (rlcard_amd/shard.py exchange_traj)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-philox', dest='philox', action='store_false',
                    help='skip the CS_RNG_PHILOX phase (reported under "rng_philox")')
    ap.add_argument('--no-precondition', dest='precondition', action='store_false',
                    help='time from freshly seeded streams (optimistic: no MT block refills yet)')
    ap.add_argument('--select', type=int, default=None,
                    help='trajectory placement selection: VecEnv.new_traj_out(select=...) allocates this many '
                         'candidate trajectories and keeps the fastest (1: off); default: what the library does '
                         '(PLACEMENT_CANDIDATES); reported under "placement"')
    ap.add_argument('--select-by', choices=('rollout', 'probe'), default='rollout',
                    help="new_traj_out's rank: 'rollout' (the library default: the probe's fast class, then one timed "
                         "rollout launch each, env state saved and restored) or 'probe' (the placement probe alone)")
    ap.add_argument('--placement', type=int, default=3,
                    help='N=1: time a few launches into this many fresh trajectory allocations after the timed region '
                         '(untimed context under "placement"; 0: off)')
    ap.add_argument('--device-state', dest='device_state', action='store_true', default=None,
                    help='sample the box (HIP attributes + amd-smi, reported under "device"); default: on, except '
                         'under a profiler (no child processes there)')
    ap.add_argument('--no-device-state', dest='device_state', action='store_false')
    args = ap.parse_args()
    if args.device_state is None:
        args.device_state = not under_profiler()

    import torch
    import torch.distributed as dist
    from rlcard_amd import _abi
    from rlcard_amd.shard import ShardedVecEnv, rank_max, time_exchange, whole_job_rate

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit('run N>1 under torchrun: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N')
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)

    # the box's state: HIP attributes + amd-smi's clocks / partition modes, queried by a host
    # thread while the envs are built and preconditioned, joined BEFORE the timed region (so even a 20-launch driver
    # run records it and the queries never overlap the timed launches)
    import threading
    dev_state, dev_state_lock = {}, threading.Lock()
    state_thread = None
    if rank == 0 and args.device_state:
        from tools.device_state import device_state

        def sample_state():
            d = device_state(local)
            with dev_state_lock:
                dev_state.update(d)
        state_thread = threading.Thread(target=sample_state, daemon=True)
        state_thread.start()

    def barrier():
        if world > 1:
            dist.barrier()

    game = args.game
    T = args.T or GAMES[game]['T']   # measured: longer launches amortise the state / staging traffic
    N = args.envs or GAMES[game]['envs']
    env = ShardedVecEnv(game, N, rank, seed=42, device=local)   # global envs [rank*N, (rank+1)*N)
    env.reset()
    traj = env.new_traj_out(T, select=args.select, rank=args.select_by)   # the library's choice (DESIGN.md placement)
    probe_ms = list(getattr(env, 'placement_probe_ms', None) or [])
    trial_ms = getattr(env, 'placement_trial_ms', None)
    select_ms = getattr(env, 'placement_select_ms', None)

    stream = torch.cuda.current_stream()
    t_launch = 0
    pre = precondition_launches(game, T, env) if args.precondition else 0
    for w in range(pre):
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        t_launch += 1
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    for w in range(args.warmup):
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        t_launch += 1
    torch.cuda.synchronize()
    steps = args.steps
    if steps <= 0:   # same K on every rank: from the slowest rank's warm-up
        per = rank_max((time.perf_counter() - w0) / max(1, args.warmup), dev)
        steps = int(min(4000, max(20, math.ceil(TIMED_TARGET_S / max(per, 1e-6)))))

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    pw = None
    state_snapshot = {}
    if state_thread is not None:
        state_thread.join(timeout=90)   # device_state's amd-smi queries are bounded at 25 + 25 + 15 s
        with dev_state_lock:
            state_snapshot = dict(dev_state) if not state_thread.is_alive() else {}
    if rank == 0 and args.device_state:
        # the power window over the timed launches -- average power, package-power-limit (PPT) residency, XCD clocks
        # -- from in-process gpu_metrics reads (sysfs through the amdsmi library: no child process), sampled every
        # 20 ms so that even a short timed region gets clock samples
        from tools.device_state import PowerWindow
        pw = PowerWindow(local)
        stop_sampling = threading.Event()

        def sample():
            pw.mid()
            while not stop_sampling.wait(0.02):
                pw.mid()
        sampler = threading.Thread(target=sample, daemon=True)
    barrier()
    torch.cuda.synchronize()
    if pw is not None:
        pw.start()
        sampler.start()
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record(stream)
        env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
        ev[k][1].record(stream)
        t_launch += 1
    torch.cuda.synchronize()
    power = None
    if pw is not None:
        power = pw.stop()
        stop_sampling.set()
    barrier()
    elapsed = rank_max(time.perf_counter() - t0, dev)
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    if pw is not None:
        sampler.join(timeout=5)

    # the timed allocation's write ceiling (untimed): the placement probe writes the rollout's trajectory bytes (zeros,
    # the same tensors and order, no game logic), so its rate is what this allocation takes writes at
    write_probe = None
    if (args.select is None or args.select > 0) and hasattr(_abi.lib(), 'cs_traj_probe'):   # (old A/B builds lack it)
        wp_ms = sorted(env.probe_traj(traj, T) for _ in range(3))[1]
        wbytes = sum(traj[k].numel() * traj[k].element_size() for k in ('obs', 'legal', 'player', 'action', 'reward', 'done'))
        write_probe = dict(ms=wp_ms, bytes=wbytes, gbs=wbytes / (wp_ms * 1e-3) / 1e9, kernel_over_probe=kernel_ms / wp_ms,
                           note='untimed: cs_traj_probe on the timed trajectory after the timed region (median of 3): '
                                'the trajectory bytes alone at this allocation\'s write rate')
    placement = None
    if world == 1 and args.placement > 0:
        # untimed context for `value` ("the 3.5 / 4.3 ms split"): the same launches into fresh trajectory
        # allocations -- the kernel time follows where the output buffers land in HBM, so a single allocation's
        # time is one draw from this spread
        per = [kernel_ms]
        other_probe = []
        for _ in range(args.placement):
            other = env.new_traj_out(T, select=1)
            other_probe.append(env.probe_traj(other, T))
            ms = []
            for k in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                env.rollout(T, policy_seed=5, t0=t_launch * T, out=other)
                e1.record(stream)
                t_launch += 1
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            per.append(sorted(ms)[len(ms) // 2] if len(ms) % 2 else sum(sorted(ms)[1:3]) / 2)
            del other
        placement = dict(kernel_ms_per_allocation=per, probe_ms_per_allocation=[None] + other_probe,
                         note='untimed: kernel ms per launch of the timed allocation (first) and of %d fresh '
                              'trajectory allocations without selection (median of 4 launches each; their placement '
                              'probe ms beside); not part of value' % args.placement)
        torch.cuda.empty_cache()

    gather_info = {}
    if world > 1 and args.gather != 'none':
        # the trajectory exchange: rollout + exchange per step, timed like the main loop
        for mode in (('rank0', 'all') if args.gather == 'both' else (args.gather,)):
            def produce():
                nonlocal t_launch
                env.rollout(T, policy_seed=5, t0=t_launch * T, out=traj)
                t_launch += 1
            info, gathered = time_exchange(produce, traj, mode, args.gather_steps, N, T, torch.cuda.synchronize, dev,
                                            budget_bytes=int(args.recv_budget_gb * (1 << 30)))
            gather_info['allgather' if mode == 'all' else 'gather'] = info
            del gathered
            torch.cuda.empty_cache()

    philox_info = None
    if args.philox:
        # the engine's fast RNG mode on the same workload (not the reference's deals): own envs, same buffers
        del env
        penv = ShardedVecEnv(game, N, rank, seed=42, device=local, config={'rng_mode': 'philox'})
        penv.reset()
        for w in range(pre + args.warmup):
            penv.rollout(T, policy_seed=5, t0=w * T, out=traj)
        psteps = max(10, steps // 2)
        pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(psteps)]
        torch.cuda.synchronize()
        barrier()
        p0 = time.perf_counter()
        for k in range(psteps):
            pev[k][0].record(stream)
            penv.rollout(T, policy_seed=5, t0=(pre + args.warmup + k) * T, out=traj)
            pev[k][1].record(stream)
        torch.cuda.synchronize()
        barrier()
        pel = rank_max(time.perf_counter() - p0, dev)
        pkms = sum(a.elapsed_time(b) for a, b in pev) / psteps
        Bp = alg_bytes_philox(penv.info, T, game)
        philox_info = dict(value=whole_job_rate(N, T, psteps, pel, world), unit='env-steps/s', steps=psteps,
                           ms_per_step=1e3 * pel / psteps, kernel_ms_per_launch=pkms,
                           alg_bytes_per_env_step=Bp,
                           roofline_frac=Bp * N * T / (pkms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           note='cs_config.rng_mode = CS_RNG_PHILOX: Philox4x32-10 byte stream keyed by the seed '
                                'key (same games, rules and policy; not the reference deals); alg bytes = SURVEY '
                                '8(d) with R = 0')
        env = penv

    if rank == 0:
        value = whole_job_rate(N, T, steps, elapsed, world)
        B = alg_bytes_per_env_step(env.info, T, game)
        achieved = B * N * T / (kernel_ms * 1e-3) / 1e9
        line = {
            'metric': 'env-steps/s (whole node) + achieved HBM GB/s, %s %d envs/GPU' % (game, N),
            'value': value,
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': steps,
            'warmup': args.warmup,
            'ms_per_step': 1e3 * elapsed / steps,
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
                         'alg_bytes_per_env_step': B, 'alg_bytes_per_launch': B * N * T,
                         'kernel_ms_per_launch': kernel_ms, 'kernel': 'k_rollout<%s>' % game},
        }
        if write_probe is not None:
            line['roofline']['write_probe'] = write_probe
        lib_name, is_product = product_library()
        if not is_product:
            line['non_product_build'] = lib_name
        tr = measured_traffic(game, N, T, kernel_ms) if is_product else None
        if not is_product:
            line['roofline']['traffic_stale'] = 'non-product build %s: no traffic profile cited' % lib_name
        if tr is not None:   # per launch, like `achieved`; from the profile of this exact configuration and kernels
            if tr['stale']:
                line['roofline']['traffic_stale'] = '%s measured other kernel sources' % tr['source']
            else:
                line['roofline']['traffic'] = tr['bytes_per_launch']
                line['roofline']['traffic_source'] = tr['source']
                # the counter-based HBM rate beside `frac`: where the byte ring moves fewer bytes than the
                # algorithmic count (traffic / alg < 1), this is the kernel's real share of the HBM peak
                line['roofline']['traffic_over_alg'] = tr['bytes_per_launch'] / (B * N * T)
                line['roofline']['traffic_frac'] = tr['bytes_per_launch'] / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                # the cited profile's own kernel time (rocprofv3 kernel trace of its timed launches) next to this
                # line's HIP-event time: a profile is evidence for the line only if they agree
                pk = tr.get('kernel_ns_timed_mean')
                if pk:
                    pk = pk / 1e6
                    line['roofline']['profile_kernel_ms'] = pk
                    line['roofline']['profile_frac'] = B * N * T / (pk * 1e-3) / 1e9 / HBM_PEAK_GBS
                    line['roofline']['profile_mismatch'] = abs(pk - kernel_ms) > 0.05 * kernel_ms
        if state_snapshot or power:
            smi = state_snapshot.get('smi') or {}
            keep = ('bus', 'gfx_0_mhz', 'gfx_0_max_mhz', 'mem_0_mhz', 'fclk_0_mhz', 'power_w', 'power_cap_static',
                    'temp_hotspot', 'temp_mem', 'driver')
            line['device'] = dict(name=state_snapshot.get('name'), arch=state_snapshot.get('arch'),
                                  hip=state_snapshot.get('hip'), smi={k: smi.get(k) for k in keep},
                                  partition=(smi.get('partition') or {}).get('current_partition'),
                                  timed_window=power)
        if placement is not None or probe_ms:
            line['placement'] = dict(placement or {})
            line['placement']['selection'] = dict(
                candidates=len(probe_ms) or 1, by=args.select_by, probe_ms=probe_ms or None, trial_ms=trial_ms,
                select_ms=select_ms, library_default=args.select is None and args.select_by == 'rollout',
                note='the timed trajectory is VecEnv.new_traj_out\'s choice, made before the preconditioning: '
                     'candidate allocations probed (cs_traj_probe: the rollout\'s writes, zeros, no game logic), '
                     'those in the fast class timed by one rollout launch each with the env state saved and restored '
                     '(cs_state_save / cs_state_load), the fastest kept -- what a library user gets (DESIGN.md '
                     'placement)')
        line.update(gather_info)
        if philox_info is not None:
            line['rng_philox'] = philox_info
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(game)
            ref = reference_cpu(game)
            if ref is not None:
                line['reference_cpu'] = ref
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
