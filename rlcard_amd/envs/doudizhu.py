"""DouDizhu env (rlcard/envs/doudizhu.py:26-188) over the HIP engine (rlcard_amd/csrc/cs_doudizhu.hip).

The action ids and strings are the reference's action space (rlcard/games/doudizhu/jsondata.zip), compiled into the
engine from rlcard_amd/csrc/ddz_actions.bin; an action string lists its cards by rank, 3..A, 2, B(lack joker),
R(ed joker) (the joined id -> string list hashes to the reference's, tests/test_envs.py).
"""
import os
import struct

import numpy as np

from .env import Env

RANKS = '3456789TJQKA2BR'
_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'csrc', 'ddz_actions.bin')


def _load_table():
    raw = open(_TABLE, 'rb').read()
    assert raw[:4] == b'DDZT'
    na, pass_id, _ = struct.unpack('<III', raw[4:16])
    packed = np.frombuffer(raw, dtype='<u8', count=na, offset=16)
    counts = ((packed[:, None] >> (4 * np.arange(15, dtype=np.uint64))) & np.uint64(15)).astype(np.int8)
    names = [''.join(RANKS[r] * int(c) for r, c in enumerate(row)) for row in counts]
    names[pass_id] = 'pass'
    return counts, names, pass_id


COUNTS, ID_2_ACTION, PASS_ID = _load_table()
ACTION_2_ID = {a: i for i, a in enumerate(ID_2_ACTION)}


def cards2array(counts15):
    """_cards2array (envs/doudizhu.py:150-166): 4 x 13 rank-count one-hot (column-major) + the two jokers."""
    m = np.zeros((4, 13), dtype=np.int8)
    for r in range(13):
        m[:int(counts15[r]), r] = 1
    return np.concatenate([m.flatten('F'), np.array([counts15[13] > 0, counts15[14] > 0], dtype=np.int8)])


def _unpack(lo, hi):
    v = lo | (hi << 32)
    return np.array([(v >> (4 * r)) & 15 for r in range(15)], dtype=np.int64)


def counts_str(c):
    return ''.join(RANKS[r] * int(n) for r, n in enumerate(c))


class DoudizhuEnv(Env):
    name = 'doudizhu'
    actions = ID_2_ACTION

    def __init__(self, config):
        super().__init__(config)
        self.state_shape = [[790], [901], [901]]
        self.action_shape = [[54] for _ in range(self.num_players)]

    def _obs_of(self, obs_bytes, player_id):
        return obs_bytes[:790 if player_id == 0 else 901].astype(np.int8)

    def _legal_value(self, action_id):
        return cards2array(COUNTS[action_id])

    def _action_id(self, raw):
        if isinstance(raw, (int, np.integer)):
            return int(raw)
        return ACTION_2_ID[raw]

    def _decode_action(self, action_id):
        """An id outside the legal set: lowest solo when leading, pass when following (include/cardsim.h cs_step;
        the reference would corrupt the hands)."""
        legal = self._legal_ids(self._last)
        if action_id in legal:
            return ID_2_ACTION[action_id]
        if PASS_ID in legal:
            return 'pass'
        return ID_2_ACTION[min(legal)]

    def get_action_feature(self, action):
        return cards2array(COUNTS[action])

    def _fields(self):
        w = self._state_words()
        hands = [_unpack(w[2 * p], w[2 * p + 1]) for p in range(3)]
        played = [_unpack(w[6 + 2 * p], w[7 + 2 * p]) for p in range(3)]
        return hands, played

    def _raw_obs(self, player_id, legal):
        """A subset of Game.get_state (games/doudizhu/game.py:110-128) decoded from the packed state; the trace is
        the host-side action record."""
        hands, played = self._fields()
        others = hands[(player_id + 1) % 3] + hands[(player_id + 2) % 3]
        return {'landlord': 0, 'self': player_id, 'current_hand': counts_str(hands[player_id]),
                'others_hand': counts_str(others), 'played_cards': [counts_str(p) for p in played],
                'num_cards_left': [int(h.sum()) for h in hands],
                'trace': [(p, a) for p, a in self.action_recorder], 'actions': [ID_2_ACTION[i] for i in legal]}

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.int64)        # judger.py judge_payoffs: landlord wins -> [1, 0, 0]

    def get_perfect_information(self):
        hands, played = self._fields()
        return {'hand_cards': [counts_str(h) for h in hands], 'played_cards': [counts_str(p) for p in played],
                'current_player': self.get_player_id() if self._last else 0,
                'legal_actions': [ID_2_ACTION[i] for i in self._legal_ids(self._last)] if self._last else []}
