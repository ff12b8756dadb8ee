"""Limit Texas Hold'em env (rlcard/envs/limitholdem.py:40-96) over the HIP engine (rlcard_amd/csrc/cs_limit.h)."""
import numpy as np

from .env import Env


def card_str(c):   # card2index order: S A..K = 0..12, H, D, C
    return 'SHDC'[c // 13] + 'A23456789TJQK'[c % 13]


class LimitholdemEnv(Env):
    name = 'limit-holdem'
    default_game_config = {'game_num_players': 2}
    configurable = True
    actions = ['call', 'raise', 'fold', 'check']

    def __init__(self, config):
        super().__init__(config)
        self.state_shape = [[72] for _ in range(self.num_players)]
        self.action_shape = [None for _ in range(self.num_players)]

    def _decode_action(self, action_id):
        """limitholdem.py:81-96: an illegal id becomes check, else fold."""
        legal = self._legal_ids(self._last)
        if action_id not in legal:
            return 'check' if 3 in legal else 'fold'
        return self.actions[action_id]

    def _fields(self):
        if self.num_players > 2:   # cs_holdem_n.h LimitN: a word per player (c0 c1 in:8@12), board, ptr:5 rc:3@5, raises
            w = self._state_words()
            P = self.num_players
            b, s1, s2 = w[P], w[P + 1], w[P + 2]
            rc = (s1 >> 5) & 7
            nboard = 0 if rc == 0 else min(5, rc + 2)
            rn = (s2 >> 12) if (s1 >> 16) & 1 else s2
            return dict(hands=[[x & 63, (x >> 6) & 63] for x in w[:P]], board=[(b >> (6 * k)) & 63 for k in range(nboard)],
                        chips=[(x >> 12) & 255 for x in w[:P]], ptr=s1 & 31, rc=rc,
                        raise_nums=[(rn >> (3 * k)) & 7 for k in range(4)])
        w0, w1, w2, w3 = self._state_words()[:4]
        rc = (w2 >> 21) & 7
        nboard = 0 if rc == 0 else min(5, rc + 2)
        rn = (w3 >> 12) if (w2 >> 26) & 1 else w3   # a reset state shows the previous game's (game.py:98 / :101)
        return dict(hands=[[w0 & 63, (w0 >> 6) & 63], [(w0 >> 12) & 63, (w0 >> 18) & 63]],
                    board=[(w1 >> (6 * k)) & 63 for k in range(nboard)], chips=[(w0 >> 24) & 63, w2 & 63],
                    ptr=(w0 >> 30) & 1, rc=rc, raise_nums=[(rn >> (3 * k)) & 7 for k in range(4)])

    def _step_back_words(self, words, current):
        """Game.step_back assigns the saved raise history to a misspelt attribute (game.py:167-168,
        history_raises_nums), so history_raise_nums keeps what the undone steps wrote, and the restored state shows
        that list, not the previous game's one a reset state shows (use_prev cleared)."""
        if self.num_players > 2:   # cs_holdem_n.h LimitN: raises in S2 (current 0..11), use_prev S1 bit 16
            P = self.num_players
            words[P + 2] = (words[P + 2] & ~0xFFF) | (current[P + 2] & 0xFFF)
            words[P + 1] &= ~(1 << 16)
        else:                      # cs_limit.h: raises in w3 (current 0..11), use_prev w2 bit 26
            words[3] = (words[3] & ~0xFFF) | (current[3] & 0xFFF)
            words[2] &= ~(1 << 26)
        return words

    def _raw_obs(self, player_id, legal, via):
        f = self._fields()
        return {'hand': [card_str(c) for c in f['hands'][player_id]], 'public_cards': [card_str(c) for c in f['board']],
                'all_chips': f['chips'], 'my_chips': f['chips'][player_id],
                'legal_actions': [self.actions[i] for i in legal], 'raise_nums': f['raise_nums']}

    def get_perfect_information(self):
        """envs/limitholdem.py:98-109 (no current_round, unlike Leduc; no board -> None)."""
        f = self._fields()
        return {'chips': f['chips'], 'public_card': [card_str(c) for c in f['board']] or None,
                'hand_cards': [[card_str(c) for c in h] for h in f['hands']],
                'current_player': f['ptr'], 'legal_actions': [self.actions[i] for i in self._legal_ids(self._last)]}
