"""Multi-rank layout on CPU (gloo, world size 2): rank r replays its env shard [r*N, (r+1)*N) -- seeds 42 + global
id, policy counter on the global id -- and the gathered trajectory equals one process running all 2N envs. The
producer here is the CPU oracle (test infrastructure); the shard arithmetic and the gather are the product's
(rlcard_amd/shard.py, used by bench.py)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip('torch')
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
GAMES = [('leduc-holdem', 96, 24), ('limit-holdem', 64, 16), ('blackjack', 64, 16), ('doudizhu', 8, 8)]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _oracle_traj(game, env_base, n, T, chunks):
    sys.path.insert(0, HERE)
    import oracle_lib
    from rlcard_amd import seeding
    keys, lens = seeding.seed_keys(range(42 + env_base, 42 + env_base + n))
    b = oracle_lib.Batch(game, n, keys, lens)
    b.reset()
    out = [b.rollout(T, 5, c * T, env_base) for c in range(chunks)]
    return {k: np.concatenate([o[k] for o in out], 0) for k in out[0]}


def _worker(rank, world, port, game, n, T, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rlcard_amd.shard import shard_range, gather_traj, new_gathered
        base, m = shard_range(n, rank)
        mine = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in _oracle_traj(game, base, m, T, 2).items()}
        got = gather_traj(mine, new_gathered(mine, world))
        if rank == 0:
            q.put({k: v.numpy() for k, v in got.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('game,n,T', GAMES)
def test_two_rank_shards_gather_to_the_single_process_trajectory(oracle, game, n, T):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, game, n, T, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = _oracle_traj(game, 0, 2 * n, T, 2)
    for k, v in full.items():
        # gathered [world, T', n, ...] -> [T', world * n, ...]
        g = np.concatenate([got[k][r] for r in range(2)], axis=1)
        assert np.array_equal(g, v), k


def _worker_rank0(rank, world, port, game, n, T, q):
    """gather_traj_to(dst=0) + the bench's cross-rank timing: rank_max of per-rank times, whole_job_rate."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rlcard_amd.shard import shard_range, gather_traj_to, new_gathered, rank_max, whole_job_rate
        base, m = shard_range(n, rank)
        mine = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in _oracle_traj(game, base, m, T, 1).items()}
        out = new_gathered(mine, world) if rank == 0 else None
        got = gather_traj_to(mine, out, dst=0)
        elapsed = rank_max(0.5 + rank)                         # rank r "took" 0.5 + r s
        rate = whole_job_rate(m, T, 3, elapsed, world)
        if rank == 0:
            q.put(({k: v.numpy() for k, v in got.items()}, elapsed, rate))
        else:
            assert got is None
            q.put((None, elapsed, rate))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('game,n,T', [('leduc-holdem', 96, 24), ('doudizhu', 8, 8)])
def test_two_rank_gather_to_rank0_and_timing(oracle, game, n, T):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker_rank0, args=(r, world, port, game, n, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for got, elapsed, rate in res:
        assert elapsed == 1.5                                 # the slowest rank's time, on every rank
        assert rate == world * n * T * 3 / 1.5                # every rank's env-steps over that time
    got = [g for g, _, _ in res if g is not None]
    assert len(got) == 1
    full = _oracle_traj(game, 0, world * n, T, 1)
    for k, v in full.items():
        g = np.concatenate([got[0][k][r] for r in range(world)], axis=1)
        assert np.array_equal(g, v), k


def _worker_exchange(rank, world, port, q):
    """bench.py's exchange phase (shard.time_exchange) in both modes with a CPU producer."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rlcard_amd.shard import time_exchange
        traj = {'obs': torch.zeros((4, 8, 3), dtype=torch.uint8), 'reward': torch.zeros((4, 8, 2))}
        calls = [0]

        def produce():
            calls[0] += 1
            traj['obs'].fill_(rank * 10 + calls[0])
            traj['reward'].fill_(float(rank))
        res = {}
        for mode in ('rank0', 'all'):
            info, g = time_exchange(produce, traj, mode, 3, 8, 4)
            held = None if g is None else {k: v.clone() for k, v in g.items()}
            res[mode] = (info, held)
        # a corrupted slice on the receiving side fails verification on every rank
        info, g = time_exchange(produce, traj, 'all', 1, 8, 4)
        from rlcard_amd.shard import verify_gathered
        g['obs'][1 - rank, 2, 3, 1] += 1
        corrupt_ok = verify_gathered(traj, g)
        q.put((rank, calls[0], {m: (i['mode'], i['steps'], i['value'] > 0, i['bytes_per_rank_per_step'],
                                    None if h is None else (h['obs'][:, 0, 0, 0].tolist(), h['reward'].shape),
                                    i['verified'])
                                for m, (i, h) in res.items()}, info['verified'], corrupt_ok))
    finally:
        dist.destroy_process_group()


def test_two_rank_exchange_phase_of_bench():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_exchange, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (c, m, v, bad)) for r, c, m, v, bad in [q.get(timeout=240) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        calls, m, v, bad = res[r]
        assert m['rank0'][5] and m['all'][5] and v, 'exchanged shards verified against their senders'
        assert not bad, 'a corrupted slice fails verification'
        assert calls == 7   # 3 + 3 exchanges, then the corrupted-slice round
        assert m['rank0'][:3] == ('rank0', 3, True) and m['all'][:3] == ('all', 3, True)
        assert m['rank0'][3] == 4 * 8 * 3 + 4 * 8 * 2 * 4
        # the last exchange of each mode holds every rank's last shard: rank r's obs = 10 r + call number
        assert m['all'][4] == ([3 + 3, 13 + 3], (2, 4, 8, 2))
    assert res[0][1]['rank0'][4] == ([3, 13], (2, 4, 8, 2))
    assert res[1][1]['rank0'][4] is None


@pytest.mark.gpu
def test_nccl_world1_exchange_on_device_trajectories():
    """bench.py's exchange phase over RCCL on the GPU (world size 1: the all_gather_into_tensor call on the uint8 /
    int16 / f32 trajectory tensors of a real DouDizhu rollout and the rank-0 copy path), with the shard verification.
    8-GPU runs are the driver's; this makes the RCCL calls run on hardware at least once."""
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU')
    port = _free_port()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    try:
        from rlcard_amd.shard import ShardedVecEnv, time_exchange
        env = ShardedVecEnv('doudizhu', 96, 0, seed=42, device=0)
        env.reset()
        traj = env.new_traj_out(8)
        t = [0]

        def produce():
            env.rollout(8, policy_seed=5, t0=8 * t[0], out=traj)
            t[0] += 1
        assert traj['action'].dtype == torch.int16 and traj['obs'].dtype == torch.uint8
        for mode in ('rank0', 'all'):
            info, g = time_exchange(produce, traj, mode, 2, 96, 8, torch.cuda.synchronize, torch.device('cuda', 0))
            assert info['verified'] and info['value'] > 0
            for k, v in traj.items():
                assert torch.equal(g[k][0], v), (mode, k)
    finally:
        dist.destroy_process_group()


def _worker_chunked(rank, world, port, q):
    """exchange_traj in T-slices through budget-bounded receive buffers (config 5's bounded all-gather), both modes:
    the consumed slices reassemble the whole exchange; a slice altered before verification is caught; shard sizes
    that are not a multiple of 8 bytes verify (digest of a misaligned slice); a budget below one step
    raises before anything is allocated."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rlcard_amd.shard import exchange_traj, exchange_chunk_steps, RecvBuffers, traj_bytes
        T, N = 7, 5   # uint8 [T, N] rows: 5 B per step, odd shard sizes
        g = torch.Generator().manual_seed(11 + rank)
        traj = {'done': torch.randint(0, 255, (T, N), dtype=torch.uint8, generator=g),
                'obs': torch.randint(0, 255, (T, N, 3), dtype=torch.uint8, generator=g),
                'reward': torch.randn((T, N, 2), generator=g)}
        row = traj_bytes(traj) // T
        budget = world * 3 * row + 1
        chunk = exchange_chunk_steps(traj, world, budget)
        out = {}
        for mode in ('rank0', 'all'):
            got = []

            def consume(t0, t1, views):
                got.append((t0, t1, {k: v.clone() for k, v in views.items()}))
            ok, recv = exchange_traj(traj, mode, consume=consume, verify=True, budget_bytes=budget)
            out[mode] = (ok, [(a, b) for a, b, _ in got],
                         None if not got else {k: torch.cat([v[k] for _, _, v in got], 1).numpy() for k in traj},
                         None if recv is None else recv.nbytes)

        def tamper(t0, t1, views):
            if t0 == 3:
                views['obs'][1 - rank, 0, 4, 2] ^= 1
        bad, _ = exchange_traj(traj, 'all', consume=tamper, verify=True, budget_bytes=budget)
        try:
            RecvBuffers(traj, world, 1, budget_bytes=world * row - 1)
            small = 'no error'
        except ValueError:
            small = 'ValueError'
        try:
            exchange_chunk_steps(traj, world, world * row - 1)
            small2 = 'no error'
        except ValueError:
            small2 = 'ValueError'
        q.put((rank, chunk, budget, out, bad, small, small2, {k: v.numpy() for k, v in traj.items()}))
    finally:
        dist.destroy_process_group()


def test_two_rank_chunked_exchange_within_budget():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_chunked, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in [q.get(timeout=240) for _ in range(2)]}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [res[r][-1] for r in (0, 1)]
    for r in (0, 1):
        chunk, budget, out, bad, small, small2, _ = res[r]
        assert chunk == 3
        assert not bad, 'a slice altered before verification fails on every rank'
        assert small == 'ValueError' and small2 == 'ValueError'
        for mode in ('rank0', 'all'):
            ok, spans, got, nbytes = out[mode]
            assert ok
            if mode == 'rank0' and r == 1:
                assert spans == [] and got is None and nbytes is None, 'a sender holds no receive buffers'
                continue
            assert spans == [(0, 3), (3, 6), (6, 7)]
            assert nbytes <= budget
            for k in shards[0]:
                for s in (0, 1):
                    assert np.array_equal(got[k][s], shards[s][k]), (mode, k, s)
