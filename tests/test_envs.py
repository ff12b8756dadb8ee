"""rlcard-compatible Env layer (rlcard_amd.make): registry, shapes/dtypes, Env.run, and the reference's own
streams replayed through the single-env API."""
import hashlib
from collections import OrderedDict

import numpy as np
import pytest

import golden_replay as gr
import rlcard_amd
from rlcard_amd.envs import doudizhu as ddz_env

torch = pytest.importorskip('torch')
GAMES = [('leduc-holdem', 'leduc'), ('limit-holdem', 'limit'), ('blackjack', 'blackjack'), ('doudizhu', 'doudizhu'),
         ('no-limit-holdem', 'nolimit')]
SHAPES = {'leduc-holdem': (2, 4, [[36]] * 2, np.float64), 'limit-holdem': (2, 4, [[72]] * 2, np.float64),
          'no-limit-holdem': (2, 5, [[54]] * 2, np.float64),
          'blackjack': (1, 2, [[2]], np.int64), 'doudizhu': (3, 27472, [[790], [901], [901]], np.int8)}


def test_registry_errors():
    with pytest.raises(ValueError):
        rlcard_amd.make('no-such-game')
    with pytest.raises(ValueError):
        rlcard_amd.register('leduc-holdem', 'rlcard_amd.envs.leducholdem:LeducholdemEnv')


def test_doudizhu_action_strings_are_the_reference_action_space():
    d = gr.load('ddz_actions')
    assert len(ddz_env.ID_2_ACTION) == 27472 and ddz_env.ID_2_ACTION[ddz_env.PASS_ID] == 'pass'
    assert hashlib.sha256(' '.join(ddz_env.ID_2_ACTION).encode()).hexdigest() == str(d['action_space_sha256'])
    f = ddz_env.cards2array(ddz_env.COUNTS[ddz_env.ACTION_2_ID['3334']])
    assert f.dtype == np.int8 and f.shape == (54,)
    assert list(np.nonzero(f)[0]) == [0, 1, 2, 4]            # column-major 4 x 13: rank 3 x3, rank 4 x1
    assert list(np.nonzero(ddz_env.cards2array(ddz_env.COUNTS[ddz_env.ACTION_2_ID['BR']]))[0]) == [52, 53]


@pytest.mark.gpu
def test_blackjack_run_random_config1_matches_reference_trajectory():
    """BASELINE config 1: examples/run_random.py --env blackjack (env seed 42, global np.random seeded 42)."""
    from rlcard_amd.agents import RandomAgent
    from rlcard_amd.utils import set_seed
    d = gr.load('blackjack')
    env = rlcard_amd.make('blackjack', config={'seed': 42})
    set_seed(42)
    agent = RandomAgent(num_actions=env.num_actions)
    env.set_agents([agent for _ in range(env.num_players)])
    traj, payoffs = env.run(is_training=False)
    got_obs, got_act = [], []
    for item in traj[0]:
        if isinstance(item, dict):
            got_obs.append(np.asarray(item['obs'], dtype=np.int64))
            got_act.append(-1)
        else:
            got_obs.append(np.zeros(2, np.int64))
            got_act.append(int(item))
    assert np.array_equal(np.stack(got_obs), d['run42_obs'])
    assert np.array_equal(np.array(got_act), d['run42_act'])
    assert np.array_equal(np.asarray(payoffs), d['run42_payoffs'])
    assert env.timestep == int((d['run42_act'] >= 0).sum())


class _Adapter:
    """One compat Env in the shape golden_replay.replay expects."""
    def __init__(self, game, seed, config=None):
        self.env = rlcard_amd.make(game, config=dict(config or {}, seed=seed))

    def _pack(self, state, player, done):
        bits = np.zeros(self.env.num_actions, np.uint8)
        bits[list(state['legal_actions'].keys())] = 1
        r = self.env.get_payoffs() if done else np.zeros(self.env.num_players)
        return dict(obs=np.asarray(state['obs']), legal=np.packbits(bits, bitorder='little'), player=player,
                    reward=np.asarray(r, np.float64), done=int(done))

    def reset(self):
        s, p = self.env.reset()
        return self._pack(s, p, False)

    def step(self, a):
        s, p = self.env.step(a)
        return self._pack(s, p, self.env.is_over())

    def observe(self, p):
        s = self.env.get_state(p)
        return np.asarray(s['obs']), None


@pytest.mark.gpu
@pytest.mark.parametrize('game,name', GAMES)
def test_reference_stream_through_compat_env(game, name):
    d = gr.load(name)
    assert gr.replay(d, lambda ei, s: _Adapter(game, s, gr.env_config(d, ei)), SHAPES[game][1]) == len(d['ev_kind'])


@pytest.mark.gpu
@pytest.mark.parametrize('game,name', GAMES)
def test_env_run_layout_and_types(game, name):
    from rlcard_amd.agents import RandomAgent
    np_, na, shape, dt = SHAPES[game]
    env = rlcard_amd.make(game, config={'seed': 3})
    assert (env.num_players, env.num_actions, env.state_shape) == (np_, na, shape)
    env.set_agents([RandomAgent(env.num_actions) for _ in range(env.num_players)])
    np.random.seed(0)
    for _ in range(3):
        t0 = env.timestep
        traj, payoffs = env.run(is_training=False)
        assert len(payoffs) == np_ and env.is_over()
        n_actions = 0
        for p in range(np_):
            seq = traj[p]
            assert isinstance(seq[-1], dict)
            for k, item in enumerate(seq[:-1]):
                if isinstance(item, dict):
                    assert item['obs'].dtype == dt and list(item['obs'].shape) == shape[p]
                    assert isinstance(item['legal_actions'], OrderedDict)
                    assert len(item['raw_legal_actions']) == len(item['legal_actions'])
                else:
                    n_actions += 1
                    assert isinstance(seq[k - 1], dict) and int(item) in seq[k - 1]['legal_actions']
        assert env.timestep - t0 == n_actions
    if game == 'doudizhu':
        s = env.get_state(1)
        for a, feat in s['legal_actions'].items():
            assert np.array_equal(feat, env.get_action_feature(a))
        assert s['raw_obs']['self'] == 1 and len(s['raw_obs']['trace']) == len(env.action_recorder)


@pytest.mark.gpu
@pytest.mark.parametrize('game,name', GAMES)
def test_step_back_restores_the_game(game, name):
    """Env.step_back (env.py:88-108): the state before each step comes back exactly, and for Leduc, DouDizhu and
    Blackjack replaying the same actions reproduces the same states (Blackjack's history holds the dealer's
    RandomState, games/blackjack/game.py:66-70, so the hits redraw the undone cards). Not for the two Texas games,
    whose reference step_back leaves part of the game behind: limit hold'em keeps the undone steps' raise history
    (game.py:167-168), no-limit's round reads a detached dealer's pot from then on (game.py:137-143, 219), so raises
    after a step back can differ; tests/test_raw.py replays the reference's own streams through all of them."""
    env = rlcard_amd.make(game, config={'seed': 5, 'allow_step_back': True})
    rng = np.random.RandomState(1)

    def snap(s, p):   # limit hold'em: the raise-count bits show the list step_back leaves behind (see above)
        obs = s['obs'][:52] if game == 'limit-holdem' else s['obs']
        return (p, obs.tobytes(), tuple(s['legal_actions'].keys()))

    for _ in range(4):
        state, player = env.reset()
        assert env.step_back() is False
        seen, acts = [snap(state, player)], []
        while not env.is_over() and len(acts) < 12:
            a = int(rng.choice(list(state['legal_actions'].keys())))
            state, player = env.step(a)
            acts.append(a)
            seen.append(snap(state, player))
        k = len(acts)
        for j in range(k, 0, -1):
            state, player = env.step_back()
            assert snap(state, player) == seen[j - 1] and not env.is_over()
        assert env.step_back() is False
        if game in ('leduc-holdem', 'doudizhu', 'blackjack'):
            for j, a in enumerate(acts):
                state, player = env.step(a)
                assert snap(state, player) == seen[j + 1]


@pytest.mark.gpu
@pytest.mark.parametrize('game,name', GAMES)
def test_step_on_a_finished_game_starts_a_new_one_without_history(game, name):
    """A step on a finished game is the engine's lazy auto-reset (include/cardsim.h cs_step): a new game with an empty
    step_back history, so step_back returns False instead of restoring the old game into the new deal's host
    bookkeeping (DouDizhu's trace / No-limit's type stack raised IndexError there)."""
    env = rlcard_amd.make(game, config={'seed': 3, 'allow_step_back': True})
    rng = np.random.RandomState(2)
    state, _ = env.reset()
    while not env.is_over():
        state, _ = env.step(int(rng.choice(list(state['legal_actions'].keys()))))
    state, player = env.step(0)   # ignored: the engine deals the next game
    assert not env.is_over()
    assert env.step_back() is False
    a = int(rng.choice(list(state['legal_actions'].keys())))
    s1, p1 = env.step(a)
    s0, p0 = env.step_back()
    assert p0 == player and s0['obs'].tobytes() == state['obs'].tobytes()
    assert list(s0['legal_actions']) == list(state['legal_actions'])
    assert env.step_back() is False


def test_step_back_is_off_by_default():
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip('needs the GPU engine')
    env = rlcard_amd.make('leduc-holdem', config={'seed': 1})
    env.reset()
    with pytest.raises(Exception):
        env.step_back()


def test_reorganize_and_remove_illegal_follow_the_reference():
    """utils.py:153-198 on a hand-built trajectory (two players, player 1 acts last)."""
    from rlcard_amd.utils import reorganize, remove_illegal
    s = [{'k': i} for i in range(6)]
    traj = [[s[0], 1, s[2], 0, s[4]], [s[1], 2, s[3], 3, s[5]]]
    out = reorganize(traj, [1.5, -1.5])
    assert out[0] == [[s[0], 1, 0, s[2], False], [s[2], 0, 1.5, s[4], True]]
    assert out[1] == [[s[1], 2, 0, s[3], False], [s[3], 3, -1.5, s[5], True]]
    p = remove_illegal(np.array([0.5, 0.0, 0.25, 0.25]), [1, 2])
    assert np.array_equal(p, np.array([0.0, 0.0, 1.0, 0.0]))
    assert np.array_equal(remove_illegal(np.zeros(4), [0, 3]), np.array([0.5, 0.0, 0.0, 0.5]))


@pytest.mark.gpu
def test_tournament_runs_the_env():
    from rlcard_amd.agents import RandomAgent
    from rlcard_amd.utils import tournament
    env = rlcard_amd.make('leduc-holdem', config={'seed': 7})
    env.set_agents([RandomAgent(env.num_actions) for _ in range(env.num_players)])
    np.random.seed(0)
    pay = tournament(env, 50)
    assert len(pay) == 2 and abs(pay[0] + pay[1]) < 1e-9
