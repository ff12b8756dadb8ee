"""Blackjack env (rlcard/envs/blackjack.py:38-103) over the HIP engine (rlcard_amd/csrc/cs_blackjack.h,
cs_blackjack_shoe.hip).

step_back follows the reference's Game.step / step_back (games/blackjack/game.py:66-70, 125-135) exactly:
* Game.step deep-copies the dealer -- its np_random included -- and the acting player before every step; step_back
  makes the copy the dealer, so the redraws after a step back replay the undone cards. The env's whole RNG stream is
  snapshotted with each history entry (cs_copy_env_rng, on the env's stream before the step) and loaded back
  (cs_load_env_rng).
* The game's own np_random is not the restored copy: it stays where the original dealer left it, and the next
  init_game deals from it. So at the first step back of a game the live stream is kept aside and loaded again before
  the next deal (_before_deal), discarding whatever the restored copies drew.
* The saved player goes into the seat of the *current* game_pointer, which step_back does not restore; the winner
  table comes back, the other seats stay (_step_back_words)."""
import ctypes as C

import numpy as np
import torch

from .. import _abi
from .env import Env
from .limitholdem import card_str


class BlackjackEnv(Env):
    name = 'blackjack'
    default_game_config = {'game_num_players': 1, 'game_num_decks': 1}
    configurable = True
    actions = ['hit', 'stand']

    def __init__(self, config):
        self._game_rng = None   # the game's own stream, kept aside while restored dealer copies draw (module doc)
        super().__init__(config)
        self.state_shape = [[2] for _ in range(self.num_players)]
        self.action_shape = [None for _ in range(self.num_players)]
        n = C.c_int32()
        _abi.check(_abi.lib().cs_env_rng_words(self._vec._h, C.byref(n)), 'cs_env_rng_words')
        self._rng_words = n.value

    def seed(self, seed=None):
        self._game_rng = None
        return super().seed(seed)

    # -- step_back (games/blackjack/game.py:66-70, 125-135) -----------------------------------------------------
    def _rng_copy(self):
        io = self._io
        buf = torch.empty(self._rng_words, dtype=torch.int32, device=self._vec.device)
        buf.record_stream(io.stream)
        _abi.check(_abi.lib().cs_copy_env_rng(self._vec._h, 0, C.c_void_p(buf.data_ptr()), io.st), 'cs_copy_env_rng')
        return buf

    def _rng_load(self, buf):
        io = self._io
        buf.record_stream(io.stream)
        _abi.check(_abi.lib().cs_load_env_rng(self._vec._h, 0, C.c_void_p(buf.data_ptr()), io.st), 'cs_load_env_rng')

    def _snapshot_extra(self):
        return self._rng_copy()      # deepcopy(self.dealer) holds the dealer's np_random

    def _restore_extra(self, buf):
        if self._game_rng is None:   # the game's np_random stays where the original dealer left it
            self._game_rng = self._rng_copy()
        self._rng_load(buf)

    def _before_deal(self):
        if self._game_rng is not None:   # init_game: Dealer(self.np_random), the game's own stream
            self._rng_load(self._game_rng)
            self._game_rng = None

    def _layout(self, w):
        """(sizes word / bit width per hand, hand bytes base word, hand capacity, meta word, pointer shift, over
        shift, winner word, winner shift) of the packed state: cs_blackjack.h (32 words) or the shoe (168 words)."""
        if len(w) == 168:
            return dict(hand_w=120, cap=24, meta=0, ptr=9, over=12, win_w=2, win_sh=10)
        return dict(hand_w=15, cap=12, meta=14, ptr=26, over=29, win_w=30, win_sh=20)

    def _size(self, w, h):
        if len(w) == 168:
            return (w[1] >> (5 * h)) & 31 if h < 6 else (w[2] >> (5 * (h - 6))) & 31
        return (w[30] >> (4 * h)) & 15

    def _set_size(self, w, h, n):
        if len(w) == 168:
            k, sh = (1, 5 * h) if h < 6 else (2, 5 * (h - 6))
            w[k] = (w[k] & ~(31 << sh)) | (n << sh)
        else:
            w[30] = (w[30] & ~(15 << (4 * h))) | (n << (4 * h))

    def _step_back_words(self, words, current):
        """game.py:133: self.dealer, self.players[self.game_pointer], self.winner = history.pop(). The snapshot
        `words` (before the undone step) gives the dealer (deck, removed cards, dealer hand) and the winner table;
        the seat of the current pointer gets the hand of the player who acted (the snapshot's pointer); every other
        seat and the pointer itself stay as they are now."""
        L = self._layout(words)
        cur = list(current)
        out = list(words)
        P = self.num_players
        acted = (words[L['meta']] >> L['ptr']) & 7
        ptr = (cur[L['meta']] >> L['ptr']) & 7
        out[L['meta']] = (out[L['meta']] & ~(7 << L['ptr'])) | (ptr << L['ptr'])
        hb = np.array(out[L['hand_w']:L['hand_w'] + (P + 1) * L['cap'] // 4], dtype='<u4').view(np.uint8).copy()
        cb = np.array(cur[L['hand_w']:L['hand_w'] + (P + 1) * L['cap'] // 4], dtype='<u4').view(np.uint8)
        saved = hb[acted * L['cap']:(acted + 1) * L['cap']].copy()
        saved_n = self._size(words, acted)
        for p in range(P):
            sl = slice(p * L['cap'], (p + 1) * L['cap'])
            if p == ptr:
                hb[sl] = saved
                self._set_size(out, p, saved_n)
            else:
                hb[sl] = cb[sl]
                self._set_size(out, p, self._size(cur, p))
        out[L['hand_w']:L['hand_w'] + len(hb) // 4] = hb.view('<u4').tolist()
        return out

    def _after_step_back(self):
        w = self._state_words()
        L = self._layout(w)
        self._last = dict(self._last, player=(w[L['meta']] >> L['ptr']) & 7, done=bool((w[L['meta']] >> L['over']) & 1))

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
