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
        self._after_deal()
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

    # -- Python int vs numpy int64 (what a use_raw agent sees in raw_obs / get_perfect_information) ----------------
    # The reference's chip counts start as Python ints and become numpy int64 once numpy values flow into them:
    # RAISE_POT bets dealer.pot (np.sum, game.py:200), a call / all-in carries the type of the amount it moves
    # (round.py:79-100, player.py bet: in_chips += quantity, remained_chips -= quantity). The engine keeps values only,
    # so the host follows the types through the same operations on the values of the step's starting state.
    def _after_deal(self):
        P = self.num_players
        self._np_in, self._np_rem, self._np_raised = [False] * P, [False] * P, [False] * P
        self._np_stack = []

    def _after_step(self, player, decoded, before):
        self._np_stack.append((list(self._np_in), list(self._np_rem), list(self._np_raised)))
        f = self._fields(before)
        p, a = player, decoded
        raised, rem = f['raised'], f['stakes']
        t_in, t_rem, t_raised = self._np_in, self._np_rem, self._np_raised
        if a == Action.CHECK_CALL:
            mx = max(raised)
            first = raised.index(mx)                      # max() returns the first maximal element
            diff_t = t_raised[first] or t_raised[p]
            q_t = diff_t if mx - raised[p] <= rem[p] else t_rem[p]
            t_raised[p] = t_raised[first]
            t_in[p] = t_in[p] or q_t
            t_rem[p] = t_rem[p] or q_t
        elif a == Action.RAISE_POT:                       # quantity = dealer.pot, a numpy int64 (legal: pot <= stack)
            t_raised[p] = t_in[p] = t_rem[p] = True
        elif a == Action.ALL_IN:                          # quantity = remained_chips, of its own type
            t_raised[p] = t_raised[p] or t_rem[p]
            t_in[p] = t_in[p] or t_rem[p]
        # RAISE_HALF_POT bets int(pot / 2), a Python int; FOLD moves nothing
        if self._fields()['rc'] != f['rc']:               # a new round: raised = [0] * N (round.py:57-63)
            self._np_raised = [False] * self.num_players

    def _after_step_back(self):
        self._np_in, self._np_rem, self._np_raised = self._np_stack.pop()

    def _step_back_words(self, words, current):
        """Game.step_back restores deep copies of the round and of the dealer made by separate deepcopy calls
        (game.py:137-143, 219): the round's dealer is detached from the game's from then on, and the round (legal
        actions, pot-sized raises, round.py:93-98, 150-159) reads the pot that detached copy holds -- the pot of the
        snapshot's state, or of the earlier snapshot it was itself restored from -- until the next init_game.
        The engine keeps that value + 1 in the round-pot field (cs_nolimit.h round_pot; 0 = live pot)."""
        P = self.num_players
        if P > 2:
            if words[P + 2] == 0:
                words[P + 2] = sum((x >> 12) & 255 for x in words[:P]) + 1
        elif (words[3] >> 12) & 0x1FFF == 0:
            words[3] |= ((words[2] & 255) + ((words[2] >> 8) & 255) + 1) << 12
        return words

    def _typed(self, values, numpy_flags):
        return [np.int64(v) if t else int(v) for v, t in zip(values, numpy_flags)]

    def _fields(self, words=None):
        stack = int(self.game_config['chips_for_each'])
        w = self._state_words() if words is None else words
        if self.num_players > 2:   # cs_holdem_n.h NolimitN: a word per player (c0 c1 in:8@12 raised:8@20), board,
            P = self.num_players   # ptr:5 rc:3@5
            b, s1 = w[P], w[P + 1]
            rc = (s1 >> 5) & 7
            nboard = 0 if rc == 0 else min(5, rc + 2)
            chips = [(x >> 12) & 255 for x in w[:P]]
            return dict(hands=[[x & 63, (x >> 6) & 63] for x in w[:P]], board=[(b >> (6 * k)) & 63 for k in range(nboard)],
                        chips=chips, stakes=[stack - c for c in chips], ptr=s1 & 31, rc=rc,
                        raised=[(x >> 20) & 255 for x in w[:P]])
        w0, w1, w2, w3 = w[:4]
        rc = (w0 >> 27) & 7
        nboard = 0 if rc == 0 else min(5, rc + 2)
        chips = [w2 & 255, (w2 >> 8) & 255]
        return dict(hands=[[w0 & 63, (w0 >> 6) & 63], [(w0 >> 12) & 63, (w0 >> 18) & 63]],
                    board=[(w1 >> (6 * k)) & 63 for k in range(nboard)], chips=chips,
                    stakes=[stack - c for c in chips], ptr=(w0 >> 24) & 1, rc=rc,
                    raised=[(w2 >> 16) & 255, (w2 >> 24) & 255])

    def _raw_obs(self, player_id, legal, via):
        """Game.get_state (game.py:187-205): the player's view plus stakes, pot and stage."""
        f = self._fields()
        chips = self._typed(f['chips'], self._np_in)
        return {'hand': [card_str(c) for c in f['hands'][player_id]],
                'public_cards': [card_str(c) for c in f['board']], 'all_chips': chips,
                'my_chips': chips[player_id], 'legal_actions': [Action(i) for i in legal],
                'stakes': self._typed(f['stakes'], self._np_rem), 'current_player': f['ptr'],
                'pot': np.int64(sum(f['chips'])), 'stage': Stage(min(f['rc'], 3))}   # pot: np.sum

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.int64)        # judger chips, not divided by the big blind (game.py:226-236)

    def get_perfect_information(self):
        f = self._fields()
        return {'chips': self._typed(f['chips'], self._np_in), 'public_card': [card_str(c) for c in f['board']] or None,
                'hand_cards': [[card_str(c) for c in h] for h in f['hands']], 'current_player': f['ptr'],
                'legal_actions': [Action(i) for i in self._legal_ids(self._last)]}
