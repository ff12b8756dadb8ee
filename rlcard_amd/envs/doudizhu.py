"""DouDizhu env (rlcard/envs/doudizhu.py:26-188) over the HIP engine (rlcard_amd/csrc/cs_doudizhu.hip).

The action ids and strings are the reference's action space (rlcard/games/doudizhu/jsondata.zip), compiled into the
engine from rlcard_amd/csrc/ddz_actions.bin; an action string lists its cards by rank, 3..A, 2, B(lack joker),
R(ed joker) (the joined id -> string list hashes to the reference's, tests/test_envs.py).

The engine plays on rank counts. The raw side of the API also shows suits and the public record, which this layer
keeps from the engine's dealt deck (state words 20..33, written by the deal kernel) and the actions it submits,
exactly as the reference's objects evolve:
  * suit-level hands (get_perfect_information 'hand_cards_with_suit'): the dealt slices sorted stably by rank
    (dealer.py:30-75), Player.play removing the first card of each played rank (player.py:78-108), play_back
    appending the removed cards and re-sorting (player.py:110-115);
  * seen_cards (round.py:32-35, 59-64): the landlord's three extra cards; every card rank the landlord plays is
    removed from it (all copies, str.replace), and step_back does not restore it;
  * trace (round.py:58, 89): (player, action) per step, popped by step_back.
"""
import os
import struct

import numpy as np

from .env import Env

RANKS = '3456789TJQKA2BR'
_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'csrc', 'ddz_actions.bin')
W_GREATER, W_DECK = 18, 20        # cs_doudizhu.h state words


def _load_table():
    raw = open(_TABLE, 'rb').read()
    assert raw[:4] == b'DDZT'
    na, pass_id, _ = struct.unpack('<III', raw[4:16])
    assert len(raw) == 16 + 12 * na
    packed = np.frombuffer(raw, dtype='<u8', count=na, offset=16)
    counts = ((packed[:, None] >> (4 * np.arange(15, dtype=np.uint64))) & np.uint64(15)).astype(np.int8)
    types = np.frombuffer(raw, dtype=np.uint8, count=na, offset=16 + 8 * na).astype(np.int32)
    tc_order = np.frombuffer(raw, dtype='<u2', count=na, offset=16 + 10 * na).astype(np.int32)
    names = [''.join(RANKS[r] * int(c) for r, c in enumerate(row)) for row in counts]
    names[pass_id] = 'pass'
    return counts, names, pass_id, types, tc_order


COUNTS, ID_2_ACTION, PASS_ID, TYPES, TC_ORDER = _load_table()
ACTION_2_ID = {a: i for i, a in enumerate(ID_2_ACTION)}
TYPE_BOMB, TYPE_ROCKET = 35, 36   # tools/gen_ddz_table.py TYPE_NAMES


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


def card_rank(c):
    """Sorted-deck card id (cs_doudizhu.h W_DECK) -> rank 0..14."""
    return c >> 2 if c < 52 else c - 39


def card_name(c):
    """Card.suit + Card.rank (games/base.py; init_54_deck, utils/utils.py:45-56): 'S3' .. 'C2', 'BJ', 'RJ'."""
    return 'SHDC'[c & 3] + RANKS[c >> 2] if c < 52 else ('BJ' if c == 52 else 'RJ')


def following_order(ids, target):
    """get_gt_cards' order (games/doudizhu/utils.py:225-262): 'pass', then the previous play's type by TYPE_CARD
    enumeration, then the rocket, then the bombs (a bomb on the table: bombs, then the rocket)."""
    tt = int(TYPES[target])

    def key(i):
        if i == PASS_ID:
            return (0, 0)
        t = int(TYPES[i])
        return (1 if t == tt else (2 if t == TYPE_ROCKET else 3), int(TC_ORDER[i]))
    return sorted(ids, key=key)


class DoudizhuEnv(Env):
    name = 'doudizhu'
    actions = ID_2_ACTION

    def __init__(self, config):
        self._suits = [[], [], []]   # suit-level hands: sorted-deck card ids in the reference's list order
        self._removed = []           # per step: the card ids Player.play removed (play_back restores them)
        self._trace = []
        self._seen = ''
        super().__init__(config)
        self.state_shape = [[790], [901], [901]]
        self.action_shape = [[54] for _ in range(self.num_players)]

    def _obs_of(self, obs_bytes, player_id):
        return obs_bytes[:790 if player_id == 0 else 901].astype(np.int8)

    def _legal_value(self, action_id):
        return cards2array(COUNTS[action_id])

    def _legal_order(self, out):
        ids = self._legal_ids(out)
        if PASS_ID in ids and len(ids) > 1:
            ids = following_order(ids, self._state_words()[W_GREATER] >> 16)
        return ids

    def _action_id(self, raw):
        if isinstance(raw, (int, np.integer)):
            return int(raw)
        return ACTION_2_ID[raw]

    def _decode_action(self, action_id):
        """An id outside the legal set: lowest solo when leading, pass when following (include/cardsim.h cs_step;
        the reference would corrupt the hands). A finished game has no legal ids: the engine ignores the action and
        deals the next game (lazy auto-reset)."""
        legal = self._legal_ids(self._last)
        if action_id in legal or not legal:
            return ID_2_ACTION[action_id]
        if PASS_ID in legal:
            return 'pass'
        return ID_2_ACTION[min(legal)]

    def get_action_feature(self, action):
        return cards2array(COUNTS[action])

    # -- the reference's suit-level bookkeeping (module docstring) -------------------------------------------------
    def _after_deal(self):
        w = self._state_words()
        deck = np.array(w[W_DECK:W_DECK + 14], dtype='<u4').view(np.uint8)[:54].tolist()
        key = card_rank
        self._suits = [sorted(sorted(deck[0:17], key=key) + deck[51:54], key=key),
                       sorted(deck[17:34], key=key), sorted(deck[34:51], key=key)]
        self._seen = ''.join(RANKS[card_rank(c)] for c in sorted(deck[51:54], key=key))
        self._removed, self._trace = [], []
        self._check()

    def _after_step(self, player, decoded, before):
        self._trace.append((player, decoded))
        removed = []
        if decoded != 'pass':
            hand = self._suits[player]
            for ch in decoded:
                r = RANKS.index(ch)
                k = next(j for j, c in enumerate(hand) if card_rank(c) == r)
                removed.append(hand.pop(k))
                if player == 0 and ch in self._seen:
                    self._seen = self._seen.replace(ch, '')
        self._removed.append(removed)
        self._check()

    def _after_step_back(self):
        player, _ = self._trace.pop()
        self._suits[player] = sorted(self._suits[player] + self._removed.pop(), key=card_rank)
        self._check()

    def _check(self):
        hands, _ = self._fields()
        for p in range(3):
            got = np.bincount([card_rank(c) for c in self._suits[p]], minlength=15)
            if not np.array_equal(got, hands[p]):
                raise RuntimeError('doudizhu suit bookkeeping out of step with the engine (player %d)' % p)

    def _fields(self):
        w = self._state_words()
        hands = [_unpack(w[2 * p], w[2 * p + 1]) for p in range(3)]
        played = [_unpack(w[6 + 2 * p], w[7 + 2 * p]) for p in range(3)]
        return hands, played

    def _raw_obs(self, player_id, legal, via):
        """Player.get_state (games/doudizhu/player.py:46-58) as Game.get_state fills it (game.py:110-128)."""
        hands, played = self._fields()
        others = hands[(player_id + 1) % 3] + hands[(player_id + 2) % 3]
        return {'seen_cards': self._seen, 'landlord': 0, 'trace': list(self._trace),
                'played_cards': [counts_str(p) for p in played], 'self': player_id,
                'current_hand': counts_str(hands[player_id]), 'others_hand': counts_str(others),
                'num_cards_left': [int(h.sum()) for h in hands], 'actions': [ID_2_ACTION[i] for i in legal]}

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.int64)        # judger.py judge_payoffs: landlord wins -> [1, 0, 0]

    def get_perfect_information(self):
        """envs/doudizhu.py:122-134."""
        hands, _ = self._fields()
        legal = self._legal_order(self._last) if self._last else []
        return {'hand_cards_with_suit': [' '.join(card_name(c) for c in h) for h in self._suits],
                'hand_cards': [counts_str(h) for h in hands], 'trace': list(self._trace),
                'current_player': self.get_player_id() if self._last else 0,
                'legal_actions': [ID_2_ACTION[i] for i in legal]}
