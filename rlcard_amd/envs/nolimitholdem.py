"""No-limit Texas Hold'em env (rlcard/envs/nolimitholdem.py:14-119) over the HIP engine (rlcard_amd/csrc/cs_nolimit.h)."""
from enum import Enum

import numpy as np

from .env import Env
from .limitholdem import card_str


class Action(Enum):          # rlcard/games/nolimitholdem/round.py:8-19
    FOLD = 0
    CHECK_CALL = 1
    RAISE_HALF_POT = 2
    RAISE_POT = 3
    ALL_IN = 4


class Stage(Enum):           # rlcard/games/nolimitholdem/game.py:14-20
    PREFLOP = 0
    FLOP = 1
    TURN = 2
    RIVER = 3
    END_HIDDEN = 4
    SHOWDOWN = 5


class NolimitholdemEnv(Env):
    name = 'no-limit-holdem'
    default_game_config = {'game_num_players': 2, 'chips_for_each': 100, 'dealer_id': None}
    configurable = True
    actions = list(Action)

    def __init__(self, config):
        super().__init__(config)
        self.state_shape = [[54] for _ in range(self.num_players)]
        self.action_shape = [None for _ in range(self.num_players)]

    def _decode_action(self, action_id):
        """envs/nolimitholdem.py:90-104. The reference's fallback for an illegal id names Action.CHECK, which does
        not exist, so it raises; the engine defines the fallback as CHECK_CALL (always legal)."""
        if action_id not in self._legal_ids(self._last):
            return Action.CHECK_CALL
        return Action(action_id)

    def _raw_action(self, action_id):
        return Action(action_id)

    def _action_id(self, raw):
        return raw.value if isinstance(raw, Action) else int(raw)

    def _fields(self):
        stack = int(self.game_config['chips_for_each'])
        if self.num_players > 2:   # cs_holdem_n.h NolimitN: a word per player (c0 c1 in:8@12), board, ptr:5 rc:3@5
            w = self._state_words()
            P = self.num_players
            b, s1 = w[P], w[P + 1]
            rc = (s1 >> 5) & 7
            nboard = 0 if rc == 0 else min(5, rc + 2)
            chips = [(x >> 12) & 255 for x in w[:P]]
            return dict(hands=[[x & 63, (x >> 6) & 63] for x in w[:P]], board=[(b >> (6 * k)) & 63 for k in range(nboard)],
                        chips=chips, stakes=[stack - c for c in chips], ptr=s1 & 31, rc=rc)
        w0, w1, w2, w3 = self._state_words()[:4]
        rc = (w0 >> 27) & 7
        nboard = 0 if rc == 0 else min(5, rc + 2)
        chips = [w2 & 255, (w2 >> 8) & 255]
        return dict(hands=[[w0 & 63, (w0 >> 6) & 63], [(w0 >> 12) & 63, (w0 >> 18) & 63]],
                    board=[(w1 >> (6 * k)) & 63 for k in range(nboard)], chips=chips,
                    stakes=[stack - c for c in chips], ptr=(w0 >> 24) & 1, rc=rc)

    def _raw_obs(self, player_id, legal, via):
        """Game.get_state (game.py:187-205): the player's view plus stakes, pot and stage."""
        f = self._fields()
        return {'hand': [card_str(c) for c in f['hands'][player_id]],
                'public_cards': [card_str(c) for c in f['board']], 'all_chips': f['chips'],
                'my_chips': f['chips'][player_id], 'legal_actions': [Action(i) for i in legal],
                'stakes': f['stakes'], 'current_player': f['ptr'], 'pot': np.int64(sum(f['chips'])),   # np.sum
                'stage': Stage(min(f['rc'], 3))}

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.int64)        # judger chips, not divided by the big blind (game.py:226-236)

    def get_perfect_information(self):
        f = self._fields()
        return {'chips': f['chips'], 'public_card': [card_str(c) for c in f['board']] or None,
                'hand_cards': [[card_str(c) for c in h] for h in f['hands']], 'current_player': f['ptr'],
                'legal_actions': [Action(i) for i in self._legal_ids(self._last)]}
