"""The rlcard API's raw side through rlcard_amd.make, exactly against the reference: raw_obs, raw_legal_actions, the
legal_actions key order, action_record, get_perfect_information() and get_payoffs(), compared as canonical JSON
(tests/rawcanon.py: types, tuple / list, key order, enum members and numpy dtypes included) with the streams
tests/golden/gen_golden.py recorded from the reference (raw_<game>.npz): resets, steps with the recorded action ids
(illegal ones included, for Leduc / Limit), step_back calls, and every player's Env.get_state after each game.
These dicts are what use_raw agents read (rlcard/models/*_rule_models.py)."""
import json

import numpy as np
import pytest

import golden_replay as gr
import rawcanon
import rlcard_amd

GAMES = ['leduc', 'limit', 'nolimit', 'blackjack', 'doudizhu']


def test_raw_fixtures_are_canonical_json():
    for name in GAMES:
        d = gr.load('raw_' + name)
        n = len(d['kind'])
        assert n > 200 and len(d['state']) == n == len(d['perfect']) == len(d['payoffs'])
        for k in range(0, n, 37):
            json.loads(d['state'][k])
            json.loads(d['perfect'][k])
        assert set(np.unique(d['kind'])) <= {0, 1, 2, 3}


def test_canon_keeps_types():
    a = rawcanon.dumps({'a': (1, [2]), 3: np.int64(4), 'x': None, 'b': True, 'f': 0.1 + 0.2})
    b = rawcanon.dumps({'a': [1, [2]], 3: 4, 'x': None, 'b': 1, 'f': 0.3})
    assert a != b
    assert rawcanon.dumps(np.array([-0.5, 0.5])) == '{"__nd__":"float64","v":[-0.5,0.5]}'


@pytest.mark.gpu
@pytest.mark.parametrize('name', GAMES)
def test_raw_side_matches_reference(name):
    d = gr.load('raw_' + name)
    streams = [json.loads(s) for s in d['streams']]
    env, cur = None, -1
    bad = []
    for k in range(len(d['kind'])):
        si, kind, act = int(d['stream'][k]), int(d['kind'][k]), int(d['act'][k])
        if si != cur:
            s = streams[si]
            env = rlcard_amd.make(s['env_id'], dict(s['config'], seed=s['seed'], allow_step_back=s['step_back']))
            cur = si
        if kind == 0:
            state, player = env.reset()
        elif kind == 1:
            state, player = env.step(act)
        elif kind == 2:
            state, player = env.step_back()
        else:
            state, player = env.get_state(act), act
        where = '%s event %d (stream %d, kind %d, act %d)' % (name, k, si, kind, act)
        assert player == int(d['player'][k]), where
        assert int(env.is_over()) == int(d['done'][k]), where
        got = rawcanon.dumps(rawcanon.state_view(state))
        if got != d['state'][k]:
            bad.append((where, 'state', got, str(d['state'][k])))
        try:
            perfect = rawcanon.dumps(env.get_perfect_information())
        except NotImplementedError:
            perfect = '"NotImplementedError"'
        if perfect != d['perfect'][k]:
            bad.append((where, 'perfect', perfect, str(d['perfect'][k])))
        if d['payoffs'][k]:
            pay = rawcanon.dumps(env.get_payoffs())
            if pay != d['payoffs'][k]:
                bad.append((where, 'payoffs', pay, str(d['payoffs'][k])))
        if len(bad) >= 3:
            break
    assert not bad, '\n'.join('%s %s\n  got %s\n  ref %s' % b for b in bad)
