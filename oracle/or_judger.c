/*
 * or_judger.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). The hold'em pot judge shared by limit and no-limit
 * (nolimitholdem/judger.py:1-5 subclasses it unchanged), restated for any number of players.
 *
 * Follows:
 *   rlcard/games/limitholdem/judger.py:11-43    judge_game: repeat { winners = compare_hands(hands); split the pots;
 *                                               winners leave (hand None, chips 0), the others keep what the split
 *                                               handed back } while chips remain
 *   rlcard/games/limitholdem/judger.py:45-88    split_pot_among_players: the smallest stake level of the players still
 *                                               in the pot; no winner in it or only winners -> everyone takes their
 *                                               chips back; else divmod(level * players, winners) each, the remainder
 *                                               to np_random.choice(winners in the pot)
 *   rlcard/games/limitholdem/judger.py:90-108   split_pots_among_players: main pot, then side pots, until no chips left
 *   rlcard/games/limitholdem/utils.py:526-614   compare_hands: the best 7-card value among the hands still in; one
 *                                               hand left -> it wins (values from or_holdem_rank7, pinned by
 *                                               tests/golden/holdem_eval.npz)
 * Where the reference fails -- compare_hands over hands that are all None, which the judge loop reaches when chips
 * handed back to a folded player remain after every player still in has won a pot (it raises from Hand(None)) -- this
 * restatement, like the ABI, stops: those chips stay with the player they were handed back to (the payoffs already
 * sum to zero at that point).
 */
#include <string.h>
#include "or_games.h"

/* judger.py:45-88 on in_chips (updated in place to in_chips_after); adds to alloc */
static void split_pot(int np, int *in_chips, const int *winners, int *alloc, or_mt *rng)
{
    int nwin = 0, nply = 0;
    for (int i = 0; i < np; i++) {
        nwin += winners[i] && in_chips[i] > 0;
        nply += in_chips[i] > 0;
    }
    if (nwin == 0 || nwin == nply) {
        for (int i = 0; i < np; i++) { alloc[i] += in_chips[i]; in_chips[i] = 0; }
        return;
    }
    int amount = 0;
    for (int i = 0; i < np; i++) if (in_chips[i] > 0 && (amount == 0 || in_chips[i] < amount)) amount = in_chips[i];
    const int one = amount * nply / nwin, rem = amount * nply % nwin;
    int cand[OR_HOLDEM_MAXP], nc = 0;
    for (int i = 0; i < np; i++) {
        if (in_chips[i] == 0) continue;
        if (winners[i]) { alloc[i] += one; cand[nc++] = i; }
    }
    if (rem > 0) alloc[cand[or_mt_interval(rng, (uint64_t)(nc - 1))]] += rem;   /* np_random.choice(cand) */
    for (int i = 0; i < np; i++) if (in_chips[i] > 0) in_chips[i] -= amount;
}

void or_holdem_judge(int np, const uint32_t *value, const int *in_chips0, or_mt *rng, int *payoffs)
{
    int in_hand[OR_HOLDEM_MAXP], in_chips[OR_HOLDEM_MAXP], remaining = 0;
    for (int i = 0; i < np; i++) {
        in_hand[i] = value[i] != 0;
        in_chips[i] = in_chips0[i];
        remaining += in_chips[i];
        payoffs[i] = 0;
    }
    while (remaining > 0) {
        int winners[OR_HOLDEM_MAXP] = {0};
        uint32_t best = 0;
        for (int i = 0; i < np; i++) if (in_hand[i] && value[i] > best) best = value[i];
        if (best == 0) break;                                  /* every hand is None: see the header */
        for (int i = 0; i < np; i++) winners[i] = in_hand[i] && value[i] == best;
        int each[OR_HOLDEM_MAXP] = {0}, left[OR_HOLDEM_MAXP];
        memcpy(left, in_chips, sizeof(int) * (size_t)np);
        for (int guard = 0; guard < 2 * OR_HOLDEM_MAXP + 2; guard++) {   /* split_pots_among_players */
            int any = 0;
            for (int i = 0; i < np; i++) any |= left[i] > 0;
            if (!any) break;
            split_pot(np, left, winners, each, rng);
        }
        for (int i = 0; i < np; i++) {
            if (winners[i]) {
                remaining -= each[i];
                payoffs[i] += each[i] - in_chips[i];
                in_hand[i] = 0;
                in_chips[i] = 0;
            } else if (in_chips[i] > 0) {
                payoffs[i] += each[i] - in_chips[i];
                in_chips[i] = each[i];
            }
        }
    }
}
