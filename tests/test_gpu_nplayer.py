"""3..22-player hold'em ('game_num_players') on the HIP engine vs the reference streams and the CPU oracle, through the
C ABI. Needs a GPU. Kernels: rlcard_amd/csrc/cs_holdem_n.h; oracle: oracle/or_leduc.c, or_limit.c, or_nolimit.c,
or_judger.c; fixtures: tests/golden/*_np.npz (tests/golden/gen_golden.py --only nplayer)."""
import numpy as np
import pytest

import golden_replay as gr
from rlcard_amd import seeding

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

FIXTURES = [('leduc-holdem', 'leduc_np'), ('limit-holdem', 'limit_np'), ('no-limit-holdem', 'nolimit_np')]
CASES = [('leduc-holdem', 3, {}), ('leduc-holdem', 5, {}), ('limit-holdem', 3, {}), ('limit-holdem', 6, {}),
         ('no-limit-holdem', 4, {}), ('no-limit-holdem', 6, {'chips_for_each': 10}),
         ('no-limit-holdem', 3, {'chips_for_each': 6, 'dealer_id': 2}), ('limit-holdem', 10, {}),
         ('no-limit-holdem', 8, {'chips_for_each': 15}), ('no-limit-holdem', 10, {'dealer_id': 9}),
         ('limit-holdem', 12, {}), ('limit-holdem', 22, {}), ('no-limit-holdem', 16, {'chips_for_each': 20}),
         ('no-limit-holdem', 22, {'dealer_id': 21})]


def _np(o):
    return {k: v.cpu().numpy() for k, v in o.items()}


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU (run them on the MI355X box)')


def _vec(game, n, **kw):
    from rlcard_amd import VecEnv
    return VecEnv(game, n, **kw)


def _oracle(oracle, game, seeds, np_, cfg):
    keys, lens = seeding.seed_keys(seeds)
    d = cfg.get('dealer_id')
    return oracle.Batch(game, len(seeds), keys, lens, num_players=np_, chips_for_each=cfg.get('chips_for_each', 100),
                        dealer_id=-1 if d is None else d)


def _same(got, exp, what):
    for k in exp:
        if k not in got:
            continue
        g, e = got[k], exp[k].astype(got[k].dtype)
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)
            raise AssertionError('%s: %s differs at %d places, first %s: got %s expected %s'
                                 % (what, k, len(bad), bad[0], g[tuple(bad[0])], e[tuple(bad[0])]))


@pytest.mark.parametrize('game,name', FIXTURES)
def test_single_env_replays_reference_nplayer_stream(game, name):
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

    assert gr.replay(d, One, 5 if game == 'no-limit-holdem' else 4) == len(d['ev_kind'])


@pytest.mark.parametrize('game,players,cfg', CASES)
def test_nplayer_step_api_matches_oracle(oracle, game, players, cfg):
    n, steps = 3000, 100
    v = _vec(game, n, seed=100, config=dict(cfg, game_num_players=players))
    assert v.num_players == players
    ob = _oracle(oracle, game, list(range(100, 100 + n)), players, cfg)
    rng = np.random.RandomState(1)
    _same(_np(v.reset()), ob.reset(), 'reset')
    for t in range(steps):
        acts = rng.randint(-1, v.num_actions + 1, size=n).astype(np.int32)   # includes illegal ids
        _same(_np(v.step(torch.from_numpy(acts).cuda())), ob.step(acts), 'step %d' % t)
    for p in range(players):
        o = _np(v.observe(p))
        for i in (0, 1, n // 2, n - 1):
            obs, legal = ob.observe(i, p)
            assert np.array_equal(o['obs'][i], obs) and np.array_equal(o['legal'][i], legal), (p, i)


@pytest.mark.parametrize('flags', [0, 1])   # 1: serial MT refill in-lane
@pytest.mark.parametrize('game,players,cfg', CASES)
def test_nplayer_rollout_matches_oracle(oracle, game, players, cfg, flags):
    """Three chained launches of 64 steps (Limit / No-limit cross several MT ring refills), then the stream
    positions; final observations of every player where a game ends."""
    n, T = 2000 + 37, 64
    v = _vec(game, n, seed=7, config=dict(cfg, game_num_players=players))
    v.set_kernel_flags(flags)
    ob = _oracle(oracle, game, list(range(7, 7 + n)), players, cfg)
    v.reset()
    ob.reset()
    for chunk in range(3):
        got = _np(v.rollout(T, policy_seed=99, t0=chunk * T, final_obs=True))
        exp = ob.rollout(T, 99, chunk * T, 0, final_obs=True)
        done = exp['done'].astype(bool)
        got['final_obs'] = got['final_obs'][done]
        exp['final_obs'] = exp['final_obs'][done]
        _same(got, exp, 'rollout chunk %d' % chunk)
        r = got['reward'][done]
        assert np.all(np.abs(r.sum(-1)) < 1e-4), 'zero-sum payoffs'
    torch.cuda.synchronize()
    for i in (0, 63, 64, n // 2, n - 1):
        assert v.rng_position(i) == ob.draws(i) % v.rng_period


@pytest.mark.parametrize('game,players', [('leduc-holdem', 4), ('limit-holdem', 5), ('no-limit-holdem', 6),
                                          ('limit-holdem', 22), ('no-limit-holdem', 17)])
def test_nplayer_compat_env(game, players):
    """rlcard_amd.make with game_num_players: shapes, raw_obs decoding of the N-player state words, Env.run."""
    import rlcard_amd
    from rlcard_amd.agents import RandomAgent
    env = rlcard_amd.make(game, config={'seed': 3, 'game_num_players': players})
    assert env.num_players == players and len(env.state_shape) == players
    env.set_agents([RandomAgent(num_actions=env.num_actions) for _ in range(players)])
    done = raised = 0
    while done < 5:
        try:
            traj, payoffs = env.run(is_training=False)
        except IndexError:   # as the reference's: Leduc's obs index passes 35 with 3+ players (leducholdem.py:63-64)
            assert game == 'leduc-holdem'
            raised += 1
            assert raised < 50
            continue
        done += 1
        assert len(traj) == players and len(payoffs) == players
        assert abs(float(np.sum(payoffs))) < 1e-6
        for p in range(players):
            raw = traj[p][-1]['raw_obs']
            assert len(raw['all_chips']) == players


def test_leduc_nplayer_payoffs_exact_float64_and_index_errors():
    """N-player Leduc through rlcard_amd.make, every event of leduc_np.npz (3..5 players):
    * Env.get_payoffs equals the reference's float64 payoffs exactly (float(total) / #winners,
      leducholdem/judger.py:50-56, / big blind), unrounded. The engine's reward rows are f32 (ABI); the compat Env
      rebuilds the float64 values with the reference's operations.
    * Env.step / Env.get_state raise IndexError exactly where the reference's _extract_state did
      (envs/leducholdem.py:63-64, the fixture's obs_len -1 events), after the game has advanced as the reference's
      has; every other observation equals the fixture's."""
    import rlcard_amd
    d = gr.load('leduc_np')
    fin_rows = {}
    for j, g in enumerate(d['fin_game']):
        fin_rows.setdefault(int(g), []).append(j)
    checked = raised = fin_raised = 0
    env, cur = None, -1
    for k in range(len(d['ev_env'])):
        ei = int(d['ev_env'][k])
        if ei != cur:
            env = rlcard_amd.make('leduc-holdem', config={'seed': int(d['seeds'][ei]),
                                                          'game_num_players': int(d['env_np'][ei])})
            cur = ei
        n = int(d['ev_obs_len'][k])
        if d['ev_kind'][k] == 0:
            state, _ = env.reset()
        elif n < 0:
            with pytest.raises(IndexError):
                env.step(int(d['ev_act'][k]))
            raised += 1
            state = None
        else:
            state, _ = env.step(int(d['ev_act'][k]))
        if state is not None:
            assert np.array_equal(state['obs'], d['ev_obs'][k][:36].astype(np.float64)), k
        assert int(env.is_over()) == int(d['ev_done'][k]) and env.get_player_id() == int(d['ev_player'][k]), k
        if d['ev_kind'][k] != 0 and d['ev_done'][k]:
            n = env.num_players
            got, exp = env.get_payoffs(), d['ev_payoff'][k][:n]
            assert got.dtype == np.float64 and np.array_equal(got, exp), (k, got, exp)
            checked += 1
            for p, j in enumerate(fin_rows[int(d['ev_game'][k])]):
                if int(d['fin_obs_len'][j]) < 0:
                    with pytest.raises(IndexError):
                        env.get_state(p)
                    fin_raised += 1
                else:
                    assert np.array_equal(env.get_state(p)['obs'], d['fin_obs'][j][:36].astype(np.float64)), (k, p)
    # a Leduc deck holds two cards per rank, so at most two players split: the values are multiples of 0.25
    assert checked > 100 and raised > 0 and fin_raised > 0, (checked, raised, fin_raised)
