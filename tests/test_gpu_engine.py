"""HIP engine vs the reference (golden streams) and vs the CPU oracle, through the C ABI. Needs a GPU."""
import numpy as np
import pytest

import golden_replay as gr
from rlcard_amd import seeding

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

GAMES = [('leduc-holdem', 'leduc'), ('limit-holdem', 'limit'), ('blackjack', 'blackjack'), ('doudizhu', 'doudizhu'),
         ('no-limit-holdem', 'nolimit')]
# doudizhu runs one wave per env and its oracle scans the 27 472-id table per observation: smaller parity batches
STEP_SIZE = {'doudizhu': (256, 80)}            # (envs, steps); default (3000, 120)
ROLL_SIZE = {'doudizhu': (256, 48)}            # (envs, T); default (4197, 48)
FULL_SIZE = {'leduc-holdem': (1 << 20, 16, 384), 'limit-holdem': (262144, 16, 384), 'blackjack': (262144, 16, 384),
             'doudizhu': (65536, 8, 64), 'no-limit-holdem': (262144, 16, 384)}      # (envs, T, oracle window)


def _np(o):
    return {k: v.cpu().numpy() for k, v in o.items()}


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU (run them on the MI355X box)')


def _vec(game, n, **kw):
    from rlcard_amd import VecEnv
    return VecEnv(game, n, **kw)


@pytest.mark.parametrize('game,name', GAMES)
def test_single_env_replays_reference_stream(game, name):
    d = gr.load(name)

    class One:
        def __init__(self, ei, seed):
            self.v = _vec(game, 1, seeds=[seed], config=gr.env_config(d, ei))

        def reset(self):
            return {k: x[0] for k, x in _np(self.v.reset()).items()}

        def step(self, a):
            return {k: x[0] for k, x in _np(self.v.step([a])).items()}

        def observe(self, p):
            o = _np(self.v.observe(p))
            return o['obs'][0], o['legal'][0]

    num_actions = _vec(game, 1).num_actions
    assert gr.replay(d, One, num_actions) == len(d['ev_kind'])


@pytest.mark.parametrize('game,name', GAMES)
def test_batched_replay_with_lazy_reset(game, name):
    """All fixture seeds as one batch; a 'reset' event after a finished game is a step with any action (lazy reset)."""
    d = gr.load(name)
    for cfg, envs in gr.config_groups(d):
        _batched_replay(d, cfg, envs, game)


def _batched_replay(d, cfg, envs, game):
    seeds = [int(d['seeds'][i]) for i in envs]
    v = _vec(game, len(seeds), seeds=seeds, config=cfg)
    per_env = [np.nonzero(d['ev_env'] == i)[0] for i in envs]
    ticks = max(len(x) for x in per_env)
    out = _np(v.reset())
    for tick in range(ticks):
        if tick > 0:
            acts = np.zeros(len(seeds), np.int32)
            for i, ev in enumerate(per_env):
                if tick < len(ev) and d['ev_kind'][ev[tick]] == 1:
                    acts[i] = d['ev_act'][ev[tick]]
            out = _np(v.step(torch.from_numpy(acts).cuda()))
        for i, ev in enumerate(per_env):
            if tick >= len(ev):
                continue
            k = ev[tick]
            n = int(d['ev_obs_len'][k])
            assert np.array_equal(out['obs'][i][:n], d['ev_obs'][k][:n]), (i, tick)
            assert np.array_equal(out['legal'][i], gr.legal_bits_of(d, k, v.num_actions)), (i, tick)
            assert out['player'][i] == d['ev_player'][k] and out['done'][i] == d['ev_done'][k], (i, tick)
            if d['ev_done'][k]:
                exp_r = d['ev_payoff'][k][:v.num_players]   # fixture rows are padded to its largest table
                assert np.array_equal(out['reward'][i].astype(np.float64), exp_r), (i, tick)


def _oracle_batch(oracle, game, seeds):
    keys, lens = seeding.seed_keys(seeds)
    return oracle.Batch(game, len(seeds), keys, lens)


def _assert_same(got, exp, what):
    for k in exp:
        if k not in got:
            continue
        g, e = got[k], exp[k]
        if g.dtype != e.dtype:
            e = e.astype(g.dtype)
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)
            raise AssertionError('%s: %s differs at %d places, first %s: got %s expected %s'
                                 % (what, k, len(bad), bad[0], g[tuple(bad[0])], e[tuple(bad[0])]))


@pytest.mark.parametrize('game,name', GAMES)
def test_step_api_matches_oracle(oracle, game, name):
    n, steps = STEP_SIZE.get(game, (3000, 120))  # not a multiple of 64: exercises the tail wave
    seeds = list(range(100, 100 + n))
    v = _vec(game, n, seed=100)
    ob = _oracle_batch(oracle, game, seeds)
    rng = np.random.RandomState(0)
    exp = ob.reset()
    _assert_same(_np(v.reset()), exp, 'reset')
    for t in range(steps):
        acts = rng.randint(-1, v.num_actions + 1, size=n).astype(np.int32)   # includes illegal ids
        if game == 'doudizhu':   # half the envs play a legal id (random ids are almost never legal there)
            for i in range(0, n, 2):
                ids = np.nonzero(np.unpackbits(exp['legal'][i], bitorder='little'))[0]
                if len(ids):
                    acts[i] = ids[rng.randint(len(ids))]
        exp = ob.step(acts)
        _assert_same(_np(v.step(torch.from_numpy(acts).cuda())), exp, 'step %d' % t)
    for p in range(v.num_players):
        o = _np(v.observe(p))
        for i in (0, 1, n // 2, n - 1):
            obs, legal = ob.observe(i, p)
            assert np.array_equal(o['obs'][i], obs) and np.array_equal(o['legal'][i], legal)


@pytest.mark.parametrize('flags', [0, 1, 2, 4, 7])   # kernel variants: serial refill / per-draw loads / dword stores
@pytest.mark.parametrize('game,name', GAMES)
def test_rollout_matches_oracle(oracle, game, name, flags):
    if game == 'doudizhu' and flags not in (0, 1, 2):
        pytest.skip('doudizhu kernel variants: 1 = every legal set through the group pass (no following fast path), '
                    '2 = the whole legal image zeroed at every step')
    n, T = ROLL_SIZE.get(game, (4160 + 37, 48))
    seeds = list(range(7, 7 + n))
    v = _vec(game, n, seed=7)
    v.set_kernel_flags(flags)
    ob = _oracle_batch(oracle, game, seeds)
    v.reset()
    ob.reset()
    for chunk in range(3):   # state, RNG position and policy counter carry across launches
        got = _np(v.rollout(T, policy_seed=99, t0=chunk * T))
        exp = ob.rollout(T, 99, chunk * T, 0)
        _assert_same(got, exp, 'rollout chunk %d' % chunk)
    torch.cuda.synchronize()
    for i in sorted({0, 63, 64, 2000 % n, n - 1}):
        assert v.rng_position(i) == ob.draws(i) % v.rng_period


@pytest.mark.parametrize('flags', [0, 1, 2])
def test_doudizhu_odd_counts(oracle, flags):
    """The DouDizhu rollout gives each half-wave one env (k_rollout2, cs_doudizhu.hip), so an odd env count leaves the
    last pair's second half empty (masked). The reference is per env (doudizhu/game.py:23-81), so every env must
    come out as in any other batch: 257 envs -- reset, single steps, 3 chained rollouts and stream positions vs the
    oracle; 65 537 envs (the bench size + 1) -- 3 launches of the bench's T = 64 compared on windows at the start, an
    odd offset and the end (the half-empty pair). Flags 1 / 2 are the kernel variants of test_rollout_matches_oracle."""
    n = 257
    v = _vec('doudizhu', n, seed=11)
    v.set_kernel_flags(flags)
    ob = _oracle_batch(oracle, 'doudizhu', range(11, 11 + n))
    exp = ob.reset()
    _assert_same(_np(v.reset()), exp, 'reset')
    rng = np.random.RandomState(4)
    for t in range(6):
        acts = np.zeros(n, np.int32)
        for i in range(n):
            ids = np.nonzero(np.unpackbits(exp['legal'][i], bitorder='little'))[0]
            acts[i] = ids[rng.randint(len(ids))] if len(ids) else 0
        exp = ob.step(acts)
        _assert_same(_np(v.step(torch.from_numpy(acts).cuda())), exp, 'step %d' % t)
    for c in range(3):
        _assert_same(_np(v.rollout(48, policy_seed=13, t0=c * 48)), ob.rollout(48, 13, c * 48, 0), 'rollout %d' % c)
    torch.cuda.synchronize()
    for i in (0, 1, 128, 255, 256):
        assert v.rng_position(i) == ob.draws(i) % v.rng_period, i
    n, T, win = 65536 + 1, 64, 33
    v = _vec('doudizhu', n, seed=42)
    v.set_kernel_flags(flags)
    v.reset()
    out = v.new_traj_out(T)
    starts = (0, n // 2 - 3, n - win)
    obs = {s: _oracle_batch(oracle, 'doudizhu', range(42 + s, 42 + s + win)) for s in starts}
    for s in starts:
        obs[s].reset()
    for c in range(3):
        tr = v.rollout(T, policy_seed=5, t0=c * T, out=out)
        for s in starts:
            got = {k: x[:, s:s + win].cpu().numpy() for k, x in tr.items()}
            _assert_same(got, obs[s].rollout(T, 5, c * T, s), 'n %d launch %d window %d' % (n, c, s))
    for s in starts:
        assert v.rng_position(s + win - 1) == obs[s].draws(win - 1) % v.rng_period


def test_doudizhu_odd_count_past_mt_twists(oracle):
    """65 DouDizhu envs (an odd count: the last wave holds one env in its first half) for 22 x 64 = 1 408 steps,
    every env past its first word-window twist and the MT_WORDS wrap (test_gpu_refill's DouDizhu case, ragged)."""
    n = 65
    v = _vec('doudizhu', n, seed=9)
    ob = _oracle_batch(oracle, 'doudizhu', range(9, 9 + n))
    _assert_same(_np(v.reset()), ob.reset(), 'reset')
    out = v.new_traj_out(64)
    for c in range(22):
        _assert_same(_np(v.rollout(64, policy_seed=2, t0=c * 64, out=out)), ob.rollout(64, 2, c * 64, 0),
                     'launch %d' % c)
    torch.cuda.synchronize()
    d = np.array([ob.draws(i) for i in range(n)])
    assert d.min() >= 1300, d.min()
    for i in (0, 31, 32, 63, 64):
        assert v.rng_position(i) == d[i] % v.rng_period, i


@pytest.mark.parametrize('players,decks', [(2, 1), (4, 1), (1, 0), (3, 0)])
def test_blackjack_configs_match_oracle(oracle, players, decks):
    """Blackjack with 2-4 players and the infinite deck (num_decks 0: a dealt card stays in the deck), step API and
    rollout launches vs the oracle (the reference fixtures hold the default game only)."""
    n, T = 2000 + 7, 32
    seeds = list(range(500, 500 + n))
    v = _vec('blackjack', n, seed=500, config={'game_num_players': players, 'game_num_decks': decks})
    keys, lens = seeding.seed_keys(seeds)
    ob = oracle.Batch('blackjack', n, keys, lens, num_players=players, num_decks=decks)
    _assert_same(_np(v.reset()), ob.reset(), 'reset')
    rng = np.random.RandomState(5)
    for t in range(12):
        acts = rng.randint(0, 2, size=n).astype(np.int32)
        _assert_same(_np(v.step(torch.from_numpy(acts).cuda())), ob.step(acts), 'step %d' % t)
    for c in range(2):
        _assert_same(_np(v.rollout(T, policy_seed=3, t0=c * T)), ob.rollout(T, 3, c * T, 0), 'rollout %d' % c)


@pytest.mark.parametrize('game,cfg', [('limit-holdem', {}), ('no-limit-holdem', {}), ('leduc-holdem', {}),
                                      ('no-limit-holdem', {'chips_for_each': 12, 'dealer_id': 1})])
def test_rollout_step_reset_interleaved(oracle, game, cfg):
    """Rollout launches, single steps and resets on the same envs: the hold'em deal queue (deals the rollout drew
    ahead) is consumed by cs_step / cs_reset in stream order, and the host's stream position discounts it."""
    n, T = 1000 + 13, 24
    seeds = list(range(300, 300 + n))
    v = _vec(game, n, seed=300, config=cfg)
    keys, lens = seeding.seed_keys(seeds)
    ob = oracle.Batch(game, n, keys, lens, chips_for_each=cfg.get('chips_for_each', 100),
                      dealer_id=cfg.get('dealer_id', -1))
    rng = np.random.RandomState(3)
    _assert_same(_np(v.reset()), ob.reset(), 'reset')
    t0 = 0
    for rnd in range(3):
        _assert_same(_np(v.rollout(T, policy_seed=11, t0=t0)), ob.rollout(T, 11, t0, 0), 'rollout %d' % rnd)
        t0 += T
        for t in range(5):
            acts = rng.randint(0, v.num_actions, size=n).astype(np.int32)
            _assert_same(_np(v.step(torch.from_numpy(acts).cuda())), ob.step(acts), 'step %d.%d' % (rnd, t))
        torch.cuda.synchronize()
        for i in (0, 1, n // 2, n - 1):
            assert v.rng_position(i) == ob.draws(i) % v.rng_period
        if rnd == 1:
            _assert_same(_np(v.reset()), ob.reset(), 'reset %d' % rnd)


@pytest.mark.parametrize('game,name', GAMES)
def test_full_size_rollout_properties_and_sampled_parity(oracle, game, name):
    n, T, win = FULL_SIZE[game]
    v = _vec(game, n, seed=42)
    v.reset()
    tr = v.rollout(T, policy_seed=5)
    torch.cuda.synchronize()
    from rlcard_amd import legal_mask
    lm = legal_mask(tr['legal'], v.num_actions)                       # [T, N, A]
    a = tr['action'].long()
    assert bool((lm.sum(-1) > 0).all()), 'every acting state has a legal action'
    assert bool(lm.gather(-1, a.unsqueeze(-1)).all()), 'policy picks legal actions'
    done = tr['done'].bool()
    rsum = tr['reward'].sum(-1)
    if game == 'doudizhu':    # landlord wins -> [1, 0, 0], else [0, 1, 1]
        rd = tr['reward'][done]
        assert bool(((rd == torch.tensor([1., 0., 0.], device=rd.device)).all(-1) |
                     (rd == torch.tensor([0., 1., 1.], device=rd.device)).all(-1)).all())
        ll = tr['player'] == 0
        assert not bool(tr['obs'][ll][:, 790:].any()), 'landlord obs is 790 wide'
        hand = tr['obs'][..., :54].long().sum(-1)
        assert bool((hand >= 1).all()) and bool((hand <= 20).all())
    elif game == 'blackjack':   # player vs dealer: payoff in {-1, 0, 1}, not zero-sum
        assert bool(((tr['reward'][done] == -1) | (tr['reward'][done] == 0) | (tr['reward'][done] == 1)).all())
        assert bool((tr['obs'][..., 0] >= 4).all()) and bool((tr['obs'][..., 0] <= 21).all()), 'acting player not bust'
    else:
        assert bool((rsum[done].abs() < 1e-6).all()), 'zero-sum payoffs'
    assert bool((tr['reward'][~done] == 0).all())
    if game == 'leduc-holdem':
        assert bool((tr['obs'].sum(-1) >= 3).all())
    if game == 'limit-holdem':
        s = tr['obs'].long().sum(-1)
        assert bool(((s >= 6) & (s <= 11)).all()), 'limit obs: 2 hole + 0/3/4/5 board + 4 raise slots'
    if game == 'no-limit-holdem':
        s = tr['obs'][..., :52].long().sum(-1)
        assert bool(((s == 2) | (s == 5) | (s == 6) | (s == 7)).all()), 'no-limit obs: 2 hole + 0/3/4/5 board'
        mine, top = tr['obs'][..., 52].long(), tr['obs'][..., 53].long()
        assert bool(((mine >= 1) & (mine <= top) & (top <= 100)).all()), 'chips: 1 <= mine <= max <= stack'
        assert bool((tr['reward'][done].abs() <= 100).all())
    # exact parity on three windows (start, middle, end) replayed by the oracle with the same env ids
    for start in (0, n // 2 + 17, n - win):
        ob = _oracle_batch(oracle, game, range(42 + start, 42 + start + win))
        ob.reset()
        exp = ob.rollout(T, 5, 0, start)
        got = {k: x[:, start:start + win].cpu().numpy() for k, x in tr.items()}
        _assert_same(got, exp, 'window %d' % start)


@pytest.mark.parametrize('game,name', GAMES)
def test_env_shards_equal_one_gpu_run(game, name):
    """bench.py's multi-GPU layout on one GPU: two shards (env_base 0 and n) reproduce a single 2n-env run."""
    from rlcard_amd.shard import ShardedVecEnv
    n, T = (64, 8) if game == 'doudizhu' else (1000, 16)
    full = _vec(game, 2 * n, seed=42)
    full.reset()
    ref = [_np(full.rollout(T, policy_seed=5, t0=c * T)) for c in range(2)]
    shards = [ShardedVecEnv(game, n, r, seed=42) for r in range(2)]
    for s in shards:
        s.reset()
    for c in range(2):
        parts = [_np(s.rollout(T, policy_seed=5, t0=c * T)) for s in shards]
        for k in ref[c]:
            assert np.array_equal(np.concatenate([p[k] for p in parts], axis=1), ref[c][k]), (c, k)
