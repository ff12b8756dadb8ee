/*
 * or_nolimit.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of No-limit Texas Hold'em (2..10 players).
 *
 * Follows:
 *   rlcard/games/nolimitholdem/game.py:45-56     configure: chips_for_each, dealer_id (None = drawn once, then kept:
 *                                                the Game object outlives init_game)
 *   rlcard/games/nolimitholdem/game.py:58-110    init_game: dealer_id = randint(0, N) if still None, THEN the dealer
 *                                                shuffles (limitholdem/dealer.py:11-21); hole i -> player i % N from
 *                                                deck.pop(); SB (dealer+1) bets 1, BB (dealer+2) bets 2 (bet clamps
 *                                                to the stack, player.py:14-17); first actor (BB+1) % N
 *   rlcard/games/nolimitholdem/game.py:123-185   step: proceed_round, the bypass rule (folded / all-in players, and
 *                                                the last player if already level), round end -> pointer (dealer+1)
 *                                                skipping bypassed players, flop / turn / river, each skipped ahead
 *                                                when everyone is bypassed
 *   rlcard/games/nolimitholdem/round.py:62-130   proceed_round: CHECK_CALL / ALL_IN / RAISE_POT / RAISE_HALF_POT /
 *                                                FOLD (raised[] takes the unclamped amount), all-in status and the
 *                                                not_raise_num / not_playing_num counters (the latter never reset
 *                                                within a game, and bumped again each time an all-in player acts)
 *   rlcard/games/nolimitholdem/round.py:132-165  get_nolimit_legal_actions (pot = dealer.pot = sum of in_chips as of
 *                                                the last get_state, which is always the current sum on this path)
 *   rlcard/games/nolimitholdem/round.py:167-173  is_over: not_raise_num + not_playing_num >= N
 *   rlcard/games/limitholdem/game.py:216-231     is_over: one player alive (ALIVE or ALLIN) or round_counter >= 4
 *   rlcard/games/nolimitholdem/game.py:226-236   payoffs = judger chips (NOT divided by the big blind)
 *   rlcard/games/limitholdem/judger.py:11-108    judge_game over ALIVE / ALL-IN hands (or_judger.c): side pots, odd
 *                                                splits draw np_random.choice
 *   rlcard/envs/nolimitholdem.py:54-85           obs[54]: card one-hot (card2index), [52] my in_chips, [53] max in_chips
 * Illegal ids: the reference's fallback names Action.CHECK, which does not exist (envs/nolimitholdem.py:98-100), so it
 * raises; this ABI defines an illegal id as CHECK_CALL (always legal).
 */
#include <string.h>
#include "or_games.h"

enum { FOLD = 0, CHECK_CALL = 1, RAISE_HALF_POT = 2, RAISE_POT = 3, ALL_IN = 4 };
enum { ALIVE = 0, FOLDED = 1, ALLIN = 2 };
#define NP OR_HOLDEM_MAXP

typedef struct {
    int np;                     /* game_num_players */
    int deck[52], deck_len;
    int hand[NP][2];
    int pub[5], npub;
    int in_chips[NP], remained[NP], status[NP];
    int raised[NP], not_raise_num, not_playing_num, round_pointer;
    int game_pointer, round_counter;
    int dealer_plus1;           /* Game.dealer_id + 1 (0 = None, drawn by the next init_game) */
} nl_env;

static int n_info(const or_cfg *cfg, or_info *info)
{
    if (cfg->num_players < 2 || cfg->num_players > NP) return -1;
    if (cfg->chips_for_each < 1 || cfg->chips_for_each > 255) return -1;
    if (cfg->dealer_id < -1 || cfg->dealer_id >= cfg->num_players) return -1;
    info->obs_dim = 54; info->num_actions = 5; info->num_players = cfg->num_players; info->legal_bytes = 1;
    return 0;
}
static size_t n_size(const or_cfg *cfg) { (void)cfg; return sizeof(nl_env); }

static int max_raised(const nl_env *e)
{
    int m = e->raised[0];
    for (int i = 1; i < e->np; i++) if (e->raised[i] > m) m = e->raised[i];
    return m;
}
static int pot_of(const nl_env *e)
{
    int t = 0;
    for (int i = 0; i < e->np; i++) t += e->in_chips[i];
    return t;
}

static void bet(nl_env *e, int p, int chips)        /* nolimitholdem/player.py:14-17 */
{
    int q = chips <= e->remained[p] ? chips : e->remained[p];
    e->in_chips[p] += q;
    e->remained[p] -= q;
}

static unsigned legal_mask(const nl_env *e)
{
    unsigned m = 0x1F;
    int p = e->round_pointer, mx = max_raised(e), pot = pot_of(e);
    int diff = mx - e->raised[p];
    if (diff > 0 && diff >= e->remained[p]) {
        m &= ~((1u << RAISE_HALF_POT) | (1u << RAISE_POT) | (1u << ALL_IN));
    } else {
        if (pot > e->remained[p]) m &= ~(1u << RAISE_POT);
        if (pot / 2 > e->remained[p]) m &= ~(1u << RAISE_HALF_POT);
        if ((m >> RAISE_HALF_POT & 1) && pot / 2 + e->raised[p] <= mx) m &= ~(1u << RAISE_HALF_POT);
    }
    return m;
}

static void n_init(void *v, or_mt *rng, const or_cfg *cfg)
{
    nl_env *e = (nl_env *)v;
    int dealer_plus1 = e->dealer_plus1;
    memset(e, 0, sizeof(*e));
    const int np = e->np = cfg->num_players;
    if (cfg->dealer_id >= 0) dealer_plus1 = cfg->dealer_id + 1;
    if (dealer_plus1 == 0) dealer_plus1 = 1 + (int)or_mt_interval(rng, (uint64_t)(np - 1));   /* randint(0, N), before the deal */
    e->dealer_plus1 = dealer_plus1;
    const int dealer = dealer_plus1 - 1;
    for (int i = 0; i < 52; i++) e->deck[i] = i;
    e->deck_len = 52;
    or_shuffle_int(rng, e->deck, 52);
    for (int p = 0; p < np; p++) {
        e->remained[p] = cfg->chips_for_each;
        e->status[p] = ALIVE;
    }
    for (int i = 0; i < 2 * np; i++) e->hand[i % np][i / np] = e->deck[--e->deck_len];
    int s = (dealer + 1) % np, b = (dealer + 2) % np;
    bet(e, b, 2);
    bet(e, s, 1);
    e->game_pointer = (b + 1) % np;
    e->round_pointer = e->game_pointer;              /* start_new_round(game_pointer, raised = in_chips) */
    e->not_raise_num = 0;
    for (int p = 0; p < np; p++) e->raised[p] = e->in_chips[p];
    e->round_counter = 0;
}

static void n_step(void *v, or_mt *rng, int a)
{
    (void)rng;
    nl_env *e = (nl_env *)v;
    unsigned legal = legal_mask(e);
    if (a < 0 || a > 4 || !((legal >> a) & 1)) a = CHECK_CALL;
    /* Round.proceed_round */
    int p = e->round_pointer, mx = max_raised(e), pot = pot_of(e);
    if (a == CHECK_CALL) {
        int diff = mx - e->raised[p];
        e->raised[p] = mx;
        bet(e, p, diff);
        e->not_raise_num += 1;
    } else if (a == ALL_IN) {
        int q = e->remained[p];
        e->raised[p] += q;
        bet(e, p, q);
        e->not_raise_num = 1;
    } else if (a == RAISE_POT) {
        e->raised[p] += pot;
        bet(e, p, pot);
        e->not_raise_num = 1;
    } else if (a == RAISE_HALF_POT) {
        int q = pot / 2;
        e->raised[p] += q;
        bet(e, p, q);
        e->not_raise_num = 1;
    } else {
        e->status[p] = FOLDED;
    }
    if (e->remained[p] == 0 && e->status[p] != FOLDED) e->status[p] = ALLIN;
    const int np = e->np;
    int rp = (p + 1) % np;
    if (e->status[p] == ALLIN) {
        e->not_playing_num += 1;
        e->not_raise_num -= 1;
    }
    if (e->status[p] == FOLDED) e->not_playing_num += 1;
    while (e->status[rp] == FOLDED) rp = (rp + 1) % np;
    e->round_pointer = rp;
    e->game_pointer = rp;
    /* Game.step: bypass rule and the end of a betting round */
    int bypass[NP], nby = 0;
    for (int i = 0; i < np; i++) { bypass[i] = e->status[i] == FOLDED || e->status[i] == ALLIN; nby += bypass[i]; }
    if (np - nby == 1) {
        int last = 0;
        while (bypass[last]) last++;                 /* players_in_bypass.index(0) */
        if (e->raised[last] >= max_raised(e)) { bypass[last] = 1; nby++; }
    }
    if (e->not_raise_num + e->not_playing_num >= np) {
        int gp = (e->dealer_plus1 - 1 + 1) % np;
        if (nby < np) while (bypass[gp]) gp = (gp + 1) % np;
        if (e->round_counter == 0) {
            for (int k = 0; k < 3; k++) e->pub[e->npub++] = e->deck[--e->deck_len];
            if (nby == np) e->round_counter += 1;
        }
        if (e->round_counter == 1) {
            e->pub[e->npub++] = e->deck[--e->deck_len];
            if (nby == np) e->round_counter += 1;
        }
        if (e->round_counter == 2) {
            e->pub[e->npub++] = e->deck[--e->deck_len];
            if (nby == np) e->round_counter += 1;
        }
        e->round_counter += 1;
        e->game_pointer = gp;
        e->round_pointer = gp;                       /* start_new_round(gp): raised = 0, not_raise_num = 0 */
        e->not_raise_num = 0;
        for (int i = 0; i < np; i++) e->raised[i] = 0;
    }
}

static int n_over(const void *v)
{
    const nl_env *e = (const nl_env *)v;
    int alive = 0;
    for (int i = 0; i < e->np; i++) alive += e->status[i] == ALIVE || e->status[i] == ALLIN;
    return alive == 1 || e->round_counter >= 4;
}

static int n_cur(const void *v) { return ((const nl_env *)v)->game_pointer; }

static void n_observe(const void *v, int player, uint8_t *obs, uint8_t *legal)
{
    const nl_env *e = (const nl_env *)v;
    memset(obs, 0, 54);
    for (int k = 0; k < e->npub; k++) obs[e->pub[k]] = 1;
    obs[e->hand[player][0]] = 1;
    obs[e->hand[player][1]] = 1;
    obs[52] = (uint8_t)e->in_chips[player];
    int mx = 0;
    for (int i = 0; i < e->np; i++) if (e->in_chips[i] > mx) mx = e->in_chips[i];
    obs[53] = (uint8_t)mx;
    legal[0] = (uint8_t)legal_mask(e);
}

static void n_payoffs(void *v, or_mt *rng, float *out)
{
    /* game.py:229-236: hands of ALIVE / ALL-IN players (others None), judge_game (or_judger.c), in chips */
    nl_env *e = (nl_env *)v;
    uint32_t value[NP];
    int pay[NP], in_hand = 0;
    for (int p = 0; p < e->np; p++) {
        value[p] = 0;
        if (e->status[p] == FOLDED) continue;
        in_hand++;
        int8_t c[7];
        c[0] = (int8_t)e->hand[p][0];
        c[1] = (int8_t)e->hand[p][1];
        for (int k = 0; k < 5; k++) c[2 + k] = (int8_t)e->pub[k];
        value[p] = or_holdem_rank7(c);
    }
    if (in_hand == 1)   /* compare_hands: the one hand left wins without being evaluated (the board may be short) */
        for (int p = 0; p < e->np; p++) value[p] = e->status[p] == FOLDED ? 0u : 1u;
    or_holdem_judge(e->np, value, e->in_chips, rng, pay);
    for (int p = 0; p < e->np; p++) out[p] = (float)pay[p];
}

const or_game_vt or_nolimit_vt = {n_info, n_size, n_init, n_step, n_over, n_cur, n_observe, n_payoffs};
