"""Replays a reference game stream (tests/golden/<game>.npz) through any engine exposing reset/step/observe on a
single env; used for the oracle (CPU) and for the HIP engine (GPU tests)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


class Fixture(dict):
    """A fixture's arrays, decompressed once (an NpzFile re-reads its zip member on every item access)."""

    @property
    def files(self):
        return list(self.keys())


def load(name):
    with np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False) as z:
        return Fixture({k: z[k] for k in z.files})


def env_config(d, ei):
    """Game config of fixture env ei (nolimit*.npz / *_np.npz hold one per env; the other streams use the defaults)."""
    c = {}
    if 'env_np' in d.files:
        c['game_num_players'] = int(d['env_np'][ei])
    if 'env_decks' in d.files:
        c['game_num_decks'] = int(d['env_decks'][ei])
    if 'env_chips' in d.files:
        dealer = int(d['env_dealer'][ei])
        c.update({'chips_for_each': int(d['env_chips'][ei]), 'dealer_id': None if dealer < 0 else dealer})
    return c


def config_groups(d):
    """[(config, [env index, ...])]: fixture envs grouped by game config (a VecEnv has one config)."""
    groups = {}
    for ei in range(len(d['seeds'])):
        c = env_config(d, ei)
        groups.setdefault(tuple(sorted(c.items())), (c, []))[1].append(ei)
    return list(groups.values())


def legal_bits_of(d, k, num_actions):
    if 'ev_legal' in d.files:
        return d['ev_legal'][k]
    ids = d['ev_legal_ids'][d['ev_legal_ptr'][k]:d['ev_legal_ptr'][k + 1]]
    m = np.zeros(num_actions, np.uint8)
    m[ids] = 1
    return np.packbits(m, bitorder='little')


def replay(d, make_env, num_actions, check_final=True):
    """make_env(seed_index, seed) -> object with reset() / step(a) returning dict(obs, legal, player, reward, done)
    for one env (1-d arrays), and observe(player) -> (obs, legal). Returns the number of checked events."""
    env_idx = d['ev_env']
    n_checked = 0
    cur_env, env = None, None
    fin = {}
    for k in range(len(env_idx)):
        fin.setdefault(int(d['ev_game'][k]), None)
    fin_rows = {}
    for j, g in enumerate(d['fin_game']):
        fin_rows.setdefault(int(g), []).append(j)
    for k in range(len(env_idx)):
        ei = int(env_idx[k])
        if ei != cur_env:
            cur_env = ei
            env = make_env(ei, int(d['seeds'][ei]))
        kind = int(d['ev_kind'][k])
        out = env.reset() if kind == 0 else env.step(int(d['ev_act'][k]))
        ctx = 'event %d (env %d game %d kind %d act %d)' % (k, ei, d['ev_game'][k], kind, d['ev_act'][k])
        n = int(d['ev_obs_len'][k])   # -1: the reference's obs raised there (N-player Leduc), nothing to compare
        exp_obs = d['ev_obs'][k]
        got_obs = np.asarray(out['obs']).reshape(-1)
        if n >= 0:
            assert np.array_equal(got_obs[:n], exp_obs[:n]), ctx + ' obs\n%s\n%s' % (got_obs[:n], exp_obs[:n])
            assert not got_obs[n:].any(), ctx + ' obs padding'
        else:   # Leduc's others'-chips slot is past 35: the row holds hand, [public,] my chips and nothing in 21..35
            assert not got_obs[21:].any() and got_obs[:3].sum() == 1 and got_obs[6:21].sum() == 1, ctx + ' raised row'
        exp_legal = legal_bits_of(d, k, num_actions)
        got_legal = np.asarray(out['legal']).reshape(-1)
        assert np.array_equal(got_legal, exp_legal), ctx + ' legal %s vs %s' % (
            np.nonzero(np.unpackbits(got_legal, bitorder='little'))[0][:20],
            np.nonzero(np.unpackbits(exp_legal, bitorder='little'))[0][:20])
        assert int(np.asarray(out['player']).reshape(-1)[0]) == int(d['ev_player'][k]), ctx + ' player'
        assert int(np.asarray(out['done']).reshape(-1)[0]) == int(d['ev_done'][k]), ctx + ' done'
        if d['ev_done'][k]:
            got_r = np.asarray(out['reward'], dtype=np.float64).reshape(-1)
            exp_r = d['ev_payoff'][k][:len(got_r)].astype(np.float32).astype(np.float64)   # f32 rows (ABI)
            assert np.array_equal(got_r, exp_r), ctx + ' payoff %s vs %s' % (got_r, d['ev_payoff'][k])
            if check_final:
                for p, j in enumerate(fin_rows[int(d['ev_game'][k])]):
                    obs, _ = env.observe(p)
                    m = int(d['fin_obs_len'][j])
                    if m < 0:
                        continue
                    assert np.array_equal(np.asarray(obs).reshape(-1)[:m], d['fin_obs'][j][:m]), ctx + ' final obs p%d' % p
        n_checked += 1
    return n_checked
