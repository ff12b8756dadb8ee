"""The batched reward rows are f32 (include/cardsim.h cs_step_out.reward); the reference computes payoffs in float64.
These CPU checks enumerate every payoff the f32 rows can be asked to hold and require it to be exactly representable,
so the rows equal the reference's float64 payoffs bit for bit after widening:

* Leduc, 2..5 players (reference rlcard/games/leducholdem/judger.py:22-64, game.py:170-178): the winners are the fold
  survivor, else the first seat pairing the public card, else every seat holding the highest rank -- and a rank has
  two cards in the 6-card deck, so at most two seats split; each_win = total / #winners, payoff = (each_win or 0 -
  in_chips) / big_blind (2).
* Hold'em: chips are integers (Limit divides by the big blind, 2).
"""
import itertools

import numpy as np

DECK = [0, 0, 1, 1, 2, 2]   # Leduc ranks J J Q Q K K (dealer.py:4-12)


def leduc_winners(ranks, public, folded):
    """judger.py:22-48 restated: the winner flags for hands `ranks`, public rank, folded flags"""
    n = len(ranks)
    w = [0] * n
    alive = [i for i in range(n) if not folded[i]]
    if len(alive) == 1:
        w[alive[0]] = 1
    if sum(w) < 1:
        for i in range(n):
            if ranks[i] == public:
                w[i] = 1
                break
    if sum(w) < 1:
        m = max(ranks)
        for i in range(n):
            if ranks[i] == m:
                w[i] = 1
    return w


def test_leduc_split_pots_are_dyadic_for_every_player_count():
    most = 0
    for n in range(2, 6):
        for cards in itertools.permutations(range(6), n + 1):   # n hands + the public card, distinct deck cards
            ranks = [DECK[c] for c in cards[:n]]
            public = DECK[cards[n]]
            for folded in itertools.product((0, 1), repeat=n):
                if sum(folded) == n:
                    continue
                k = sum(leduc_winners(ranks, public, folded))
                most = max(most, k)
                assert k in (1, 2), (ranks, public, folded)
    assert most == 2   # a two-way split happens (a non-dyadic share such as 7/3 never does)


def test_leduc_payoffs_exact_in_f32():
    # in_chips per player <= 1 + 2 raises in each of 2 rounds (2 + 2 + 4 + 4) = 13 (round.py allowed_raise_num 2)
    for n in range(2, 6):
        for total in range(2 * n, 14 * n + 1):
            for k in (1, 2):
                each = float(total) / k
                for inc in range(1, 15):
                    for pay in (each - inc, float(-inc)):
                        v = np.array([pay]) / 2   # game.py:177 np.array(chips_payoffs) / big_blind
                        assert float(np.float32(v[0])) == float(v[0])


def test_holdem_chip_payoffs_exact_in_f32():
    # Limit: integer chip payoffs / big blind 2; No-limit: integer chips (stacks <= 255 per player, <= 22 players)
    for chips in range(-255 * 22, 255 * 22 + 1):
        assert float(np.float32(chips / 2)) == chips / 2
        assert float(np.float32(float(chips))) == float(chips)
