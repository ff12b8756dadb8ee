"""Leduc Hold'em env (rlcard/envs/leducholdem.py:11-112) over the HIP engine (rlcard_amd/csrc/cs_leduc.h)."""
import numpy as np

from .env import Env

CARDS = ['SJ', 'HJ', 'SQ', 'HQ', 'SK', 'HK']   # engine card index = rlcard/games/leducholdem/dealer.py deck order


class LeducholdemEnv(Env):
    name = 'leduc-holdem'
    default_game_config = {'game_num_players': 2}
    configurable = True
    actions = ['call', 'raise', 'fold', 'check']

    def __init__(self, config):
        super().__init__(config)
        self.state_shape = [[36] for _ in range(self.num_players)]
        self.action_shape = [None for _ in range(self.num_players)]

    def _decode_action(self, action_id):
        """leducholdem.py:81-96: an illegal id becomes check, else fold."""
        legal = self._legal_ids(self._last)
        if action_id not in legal:
            return 'check' if 3 in legal else 'fold'
        return self.actions[action_id]

    def _obs_of(self, obs_bytes, player_id):
        """_extract_state (leducholdem.py:59-64) sets obs[sum(all_chips) - my_chips + 21]: with 3+ players the others'
        chips can pass 14 and the index 36, where the reference raises IndexError -- after Game.step has advanced,
        so is_over / get_payoffs / the next step see the new state. This Env raises the same error at the same point.
        (The engine's batched rows hold the other slots -- hand, public card, my chips -- and no bit for the
        out-of-range one: cs_holdem_n.h LeducN::observe.) Heads-up the index stays <= 35 (others' chips <= 14)."""
        if self.num_players > 2:
            f = self._fields()
            k = sum(f['chips']) - f['chips'][player_id] + 21
            if k >= 36:
                raise IndexError('index %d is out of bounds for axis 0 with size 36' % k)
        return obs_bytes.astype(np.float64)

    def _fields(self):
        w = self._state_words()
        if self.num_players > 2:   # cs_holdem_n.h LeducN: a word per player (hand:3 in:5), then pub:3 rc:2 ptr:3
            P, sw = self.num_players, w[self.num_players]
            return dict(h=[x & 7 for x in w[:P]], pub=sw & 7, chips=[(x >> 3) & 31 for x in w[:P]],
                        rc=(sw >> 3) & 3, ptr=(sw >> 5) & 7)
        w0, w1 = w[:2]
        return dict(h=[w0 & 7, (w0 >> 3) & 7], pub=(w0 >> 6) & 7, chips=[(w0 >> 9) & 31, (w0 >> 14) & 31],
                    rc=w1 & 3, ptr=(w1 >> 2) & 1)

    def _raw_obs(self, player_id, legal, via):
        f = self._fields()
        return {'hand': CARDS[f['h'][player_id]], 'public_card': CARDS[f['pub']] if f['rc'] >= 1 else None,
                'all_chips': f['chips'], 'my_chips': f['chips'][player_id],
                'legal_actions': [self.actions[i] for i in legal], 'current_player': f['ptr']}

    def _payoff_array(self, r):
        """Game.get_payoffs (leducholdem/game.py:170-178): judger chips / big blind in float64. Heads-up payoffs are
        multiples of 0.5, exact in the engine's f32 reward row; with 3+ players a split pot pays
        float(total) / #winners (judger.py:50-56), so the payoffs are rebuilt in float64 with the reference's
        operations: the winners are the players whose reward is not -in_chips / 2 (each_win > 0)."""
        r = np.asarray(r, dtype=np.float64)
        if self.num_players <= 2 or self._payoffs is None or self._words is None:
            return r
        chips = self._fields()['chips']
        won = [float(r[i]) != -chips[i] / 2.0 for i in range(self.num_players)]
        if not any(won):
            return r
        each_win = float(sum(chips)) / sum(won)
        return np.array([(each_win - c) if w else float(-c) for c, w in zip(chips, won)]) / 2

    def get_perfect_information(self):
        f = self._fields()
        return {'chips': f['chips'], 'public_card': CARDS[f['pub']] if f['rc'] >= 1 else None,
                'hand_cards': [CARDS[h] for h in f['h']], 'current_round': f['rc'], 'current_player': f['ptr'],
                'legal_actions': [self.actions[i] for i in self._legal_ids(self._last)]}
