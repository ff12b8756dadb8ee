"""Canonical JSON of the rlcard API's raw outputs (state['raw_obs'], 'raw_legal_actions', the legal_actions key order,
'action_record', get_perfect_information(), get_payoffs()), shared by the fixture generator (tests/golden/gen_golden.py,
run against the reference) and the tests that compare rlcard_amd.make's Env with it.

Test infrastructure only. The encoding keeps every distinction a consumer of these dicts can observe: tuple vs list,
dict key order and key types, numpy scalar / array dtypes, enum members (by class and member name), bool vs int, and
floats exactly (json writes repr, which round-trips)."""
import json
from enum import Enum

import numpy as np


def canon(x):
    if isinstance(x, Enum):
        return {'__enum__': '%s.%s' % (type(x).__name__, x.name)}
    if isinstance(x, np.ndarray):
        return {'__nd__': x.dtype.name, 'v': x.tolist()}
    if isinstance(x, np.generic):
        return {'__np__': x.dtype.name, 'v': x.item()}
    if isinstance(x, tuple):
        return {'__tuple__': [canon(y) for y in x]}
    if isinstance(x, list):
        return [canon(y) for y in x]
    if isinstance(x, dict):
        return {'__dict__': [[canon(k), canon(v)] for k, v in x.items()]}
    if x is None or isinstance(x, (bool, int, float, str)):
        return x
    raise TypeError('no canonical form for %r (%s)' % (x, type(x).__name__))


def dumps(x):
    return json.dumps(canon(x), separators=(',', ':'))


def state_view(state):
    """The parts of an Env state dict that are not the numeric obs (pinned elsewhere): raw_obs, raw_legal_actions,
    the legal_actions keys in their order, action_record."""
    return {'raw_obs': state['raw_obs'], 'raw_legal_actions': state['raw_legal_actions'],
            'legal_keys': list(state['legal_actions'].keys()), 'action_record': state['action_record']}


def ddz_sort_leading(state, action_2_id):
    """DouDizhu's leading legal actions come from a Python set (games/doudizhu/judger.py:124-134), so their order in
    raw_obs['actions'], raw_legal_actions and the legal_actions keys depends on PYTHONHASHSEED: the fixtures store
    them by ascending action id, the order rlcard_amd emits. Following sets (get_gt_cards, utils.py:225-262, which
    starts with 'pass') have a defined order and are kept as the reference produced them."""
    acts = state['raw_obs'].get('actions')
    if acts and 'pass' not in acts:
        order = sorted(acts, key=lambda a: action_2_id[a])
        state = dict(state)
        state['raw_obs'] = dict(state['raw_obs'], actions=order)
        state['raw_legal_actions'] = list(order)
        state['legal_actions'] = {action_2_id[a]: state['legal_actions'][action_2_id[a]] for a in order}
    return state


def ddz_sort_perfect(info, action_2_id):
    acts = info.get('legal_actions')
    if acts and 'pass' not in acts:
        info = dict(info, legal_actions=sorted(acts, key=lambda a: action_2_id[a]))
    return info
