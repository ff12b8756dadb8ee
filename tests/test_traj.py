"""After the rollout: final observations, rlcard's reorganize + DMC targets, legal-id lists
and action features, on the device vs restatements here / the CPU oracle. Needs a GPU."""
import numpy as np
import pytest

from rlcard_amd import seeding

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

GAMES = ['leduc-holdem', 'limit-holdem', 'blackjack', 'doudizhu', 'no-limit-holdem']
SIZE = {'doudizhu': (70, 40)}   # (envs, T); default (700, 48)


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU (run them on the MI355X box)')


def _rollout(game, n, T, seed=7, chunks=1):
    from rlcard_amd import VecEnv
    v = VecEnv(game, n, seed=seed)
    v.reset()
    outs = [v.rollout(T, policy_seed=11, t0=c * T, final_obs=True) for c in range(chunks)]
    torch.cuda.synchronize()
    return v, outs


@pytest.mark.parametrize('game', GAMES)
def test_final_observations_match_oracle(oracle, game):
    n, T = SIZE.get(game, (700, 48))
    v, outs = _rollout(game, n, T, chunks=2)
    keys, lens = seeding.seed_keys(range(7, 7 + n))
    ob = oracle.Batch(game, n, keys, lens)
    ob.reset()
    for c, tr in enumerate(outs):
        exp = ob.rollout(T, 11, c * T, 0, final_obs=True)
        got = tr['final_obs'].cpu().numpy()
        done = exp['done'].astype(bool)
        assert done.any()
        assert np.array_equal(got[done], exp['final_obs'][done]), 'final_obs differs (chunk %d)' % c
        assert not got[~done].any(), 'rows without a finished game stay untouched'


def reorganize_rows(player, done, reward, P):
    """rlcard/utils/utils.py:153-179 restated on one env's rows: transition of the player acting at row t goes to its
    next turn in the same game, or to the game's final state (reward = its payoff, done) -- expected arrays in the
    layout of cs_transitions."""
    T = len(player)
    next_t = np.full(T, -2, np.int32)
    end_t = np.full(T, -1, np.int32)
    rew = np.zeros(T, np.float32)
    dn = np.zeros(T, np.uint8)
    ret = np.full(T, np.nan, np.float32)
    start = 0
    while start < T:
        end = start
        while end < T and not done[end]:
            end += 1
        rows = range(start, min(end, T - 1) + 1)
        ended = end < T
        turns = {}
        for t in rows:
            turns.setdefault(int(player[t]), []).append(t)
        for p, ts in turns.items():
            for j, t in enumerate(ts):
                if j + 1 < len(ts):
                    next_t[t] = ts[j + 1]
                elif ended:
                    next_t[t] = -1
                    rew[t] = reward[end][p]
                    dn[t] = 1
                if ended:
                    ret[t] = reward[end][p]
                    end_t[t] = end
        start = end + 1
    return next_t, end_t, rew, dn, ret


@pytest.mark.parametrize('game', GAMES)
def test_transitions_are_rlcard_reorganize(game):
    n, T = SIZE.get(game, (700, 48))
    v, (tr,) = _rollout(game, n, T)
    got = {k: x.cpu().numpy() for k, x in v.transitions(tr).items()}
    pl, dn, rw = (tr[k].cpu().numpy() for k in ('player', 'done', 'reward'))
    for e in range(n):
        nt, et, r, d, ret = reorganize_rows(pl[:, e], dn[:, e], rw[:, e], v.num_players)
        assert np.array_equal(got['next_t'][:, e], nt), e
        assert np.array_equal(got['end_t'][:, e], et), e
        assert np.array_equal(got['reward'][:, e], r), e
        assert np.array_equal(got['done'][:, e], d), e
        assert np.array_equal(np.isnan(got['ret'][:, e]), np.isnan(ret)), e
        m = ~np.isnan(ret)
        assert np.array_equal(got['ret'][m, e], ret[m]), e


@pytest.mark.parametrize('game', GAMES)
def test_legal_lists_and_action_features(game):
    n, T = SIZE.get(game, (700, 48))
    v, (tr,) = _rollout(game, n, T)
    counts, offsets, ids = v.legal_lists(tr['legal'])
    bits = np.unpackbits(tr['legal'].cpu().numpy().reshape(-1, v.legal_bytes), axis=1, bitorder='little')
    bits = bits[:, :v.num_actions]
    c, o, i = counts.cpu().numpy(), offsets.cpu().numpy(), ids.cpu().numpy()
    assert np.array_equal(c, bits.sum(1)) and o[0] == 0 and np.array_equal(np.diff(o), c)
    rows = np.nonzero(bits)
    assert np.array_equal(i, rows[1])                                 # row-major, ascending within a row
    # the policy's actions are legal ids and their features are Env.get_action_feature's
    acts = tr['action'].reshape(-1).to(torch.int32)
    feats = v.action_features(acts).cpu().numpy()
    a = acts.cpu().numpy()
    if game == 'doudizhu':
        from rlcard_amd.envs.doudizhu import COUNTS, cards2array
        exp = np.stack([cards2array(COUNTS[x]) for x in a]).astype(np.uint8)
        sample = v.action_features(ids[:5000]).cpu().numpy()
        exp_s = np.stack([cards2array(COUNTS[x]) for x in i[:5000]]).astype(np.uint8)
        assert np.array_equal(sample, exp_s)
    else:
        exp = np.eye(v.num_actions, dtype=np.uint8)[a]
    assert feats.shape == (len(a), v.info.action_feature_dim) and np.array_equal(feats, exp)
