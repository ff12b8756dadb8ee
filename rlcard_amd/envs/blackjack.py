"""Blackjack env (rlcard/envs/blackjack.py:38-103) over the HIP engine (rlcard_amd/csrc/cs_blackjack.h).

step_back restores the whole game and continues the env's stream; the reference's Game.step_back (game.py:65-70,
125-135) restores a deep copy of the dealer with its RandomState, so its next hits redraw the undone cards, and puts
the acting player's snapshot into the current pointer's seat."""
import numpy as np

from .env import Env
from .limitholdem import card_str


class BlackjackEnv(Env):
    name = 'blackjack'
    default_game_config = {'game_num_players': 1, 'game_num_decks': 1}
    configurable = True
    actions = ['hit', 'stand']

    def __init__(self, config):
        super().__init__(config)
        self.state_shape = [[2] for _ in range(self.num_players)]
        self.action_shape = [None for _ in range(self.num_players)]

    def _obs_of(self, obs_bytes, player_id):
        return obs_bytes.astype(np.int64)          # (player score, dealer's visible score)

    def _hands(self):
        """The hands (players 0..P-1, then the dealer) from the packed state: cs_blackjack.h (1 deck, <= 4 players:
        sizes 4 bits each in word 30, 12-byte hands from word 15) or cs_blackjack_shoe.hip (168 words: sizes 5 bits
        each in words 1..2, 24-byte hands from word 120)."""
        w = self._state_words()
        hands = []
        if len(w) == 168:
            b = np.array(w[120:168], dtype='<u4').view(np.uint8)
            for h in range(self.num_players + 1):
                n = (w[1] >> (5 * h)) & 31 if h < 6 else (w[2] >> (5 * (h - 6))) & 31
                hands.append([card_str(int(c)) for c in b[24 * h:24 * h + n]])
            return hands
        sizes = w[30]
        for h in range(self.num_players + 1):
            n = (sizes >> (4 * h)) & 15
            hands.append([card_str((w[15 + (12 * h + k) // 4] >> (8 * ((12 * h + k) % 4))) & 255) for k in range(n)])
        return hands

    def _raw_obs(self, player_id, legal, via):
        """Game.get_state (games/blackjack/game.py:162-190) -- or, for the state Env.step returns, the dict Game.step
        builds (game.py:104-117): the same entries, 'actions' moved after the hands."""
        hands = self._hands()
        dealer = hands[-1] if self.is_over() else hands[-1][1:]
        seats = [('player%d hand' % i, hands[i]) for i in range(self.num_players)]
        if via == 'step':
            items = seats + [('dealer hand', dealer), ('actions', tuple(self.actions))]
        else:
            items = [('actions', tuple(self.actions))] + seats + [('dealer hand', dealer)]
        return dict(items + [('state', (hands[player_id], dealer))])

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.int64)        # blackjack.py get_payoffs: 1 win, 0 tie, -1 loss
