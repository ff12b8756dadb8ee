/*
 * or_limit.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of Limit Texas Hold'em (2..10 players).
 *
 * Follows:
 *   rlcard/utils/utils.py:34-43                 init_standard_deck: suits S,H,D,C x ranks A,2..K (= card2index order)
 *   rlcard/games/limitholdem/dealer.py:4-21     shuffle at construction, deal_card = deck.pop()
 *   rlcard/games/limitholdem/game.py:46-103     init_game: 2N hole cards round-robin, SB = randint(0,N),
 *                                               first actor (BB+1)%N; get_state BEFORE history_raise_nums is
 *                                               re-bound (:98 vs :101) -> the reset obs shows the PREVIOUS game's
 *                                               raise counts (quirk reproduced: prev_raise_nums below)
 *   rlcard/games/limitholdem/game.py:105-158    step: history_raise_nums[round] = have_raised; flop 3 / turn / river,
 *                                               raise amount doubles after round 1
 *   rlcard/games/limitholdem/game.py:216-243    is_over (one alive or round_counter >= 4), get_payoffs (/ big_blind)
 *   rlcard/games/limitholdem/round.py:5-127     betting FSM (allowed_raise_num 4)
 *   rlcard/games/limitholdem/judger.py:11-108   judge_game / split_pot(s)_among_players
 *   rlcard/games/limitholdem/utils.py:3-614     Hand.evaluateHand / compare_hands (== standard 7-card ranking,
 *                                               pinned by tests/golden/holdem_eval.npz)
 *   rlcard/envs/limitholdem.py:40-96            obs[72] and _decode_action fallback
 */
#include <string.h>
#include "or_games.h"

enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };
#define HP OR_HOLDEM_MAXP

typedef struct {
    int np;                     /* game_num_players (envs/env.py:33-39 -> game.py:42-44) */
    int deck[52], deck_len;
    int hand[HP][2];
    int pub[5], npub;
    int in_chips[HP], folded[HP];
    int raise_amount, allowed_raise_num, have_raised, not_raise_num, raised[HP], round_pointer;
    int game_pointer, round_counter;
    int raise_nums[4];          /* self.history_raise_nums                                   */
    int prev_raise_nums[4];     /* the list object the reset state dict still references     */
    int use_prev;               /* 1 only for the obs returned by init_game                   */
} limit_env;

static int h_np(const or_cfg *cfg) { return cfg && cfg->num_players > 0 ? cfg->num_players : 2; }

static int h_info(const or_cfg *cfg, or_info *info)
{
    const int np = h_np(cfg);
    if (np < 2 || np > HP) return -1;
    info->obs_dim = 72; info->num_actions = 4; info->num_players = np; info->legal_bytes = 1;
    return 0;
}
static size_t h_size(const or_cfg *cfg) { (void)cfg; return sizeof(limit_env); }

static int max_raised(const limit_env *e)
{
    int m = e->raised[0];
    for (int i = 1; i < e->np; i++) if (e->raised[i] > m) m = e->raised[i];
    return m;
}

static unsigned legal_mask(const limit_env *e)
{
    unsigned m = 0xF;
    int p = e->round_pointer, mx = max_raised(e);
    if (e->have_raised >= e->allowed_raise_num) m &= ~(1u << RAISE);
    if (e->raised[p] < mx) m &= ~(1u << CHECK);
    if (e->raised[p] == mx) m &= ~(1u << CALL);
    return m;
}

static void start_new_round(limit_env *e, int gp, const int *raised)
{
    e->round_pointer = gp;
    e->have_raised = 0;
    e->not_raise_num = 0;
    for (int i = 0; i < e->np; i++) e->raised[i] = raised ? raised[i] : 0;
}

static void h_init(void *v, or_mt *rng, const or_cfg *cfg)
{
    limit_env *e = (limit_env *)v;
    int prev[4];
    memcpy(prev, e->raise_nums, sizeof(prev));     /* persists across games (Game object outlives init_game) */
    memset(e, 0, sizeof(*e));
    const int np = e->np = h_np(cfg);
    for (int i = 0; i < 52; i++) e->deck[i] = i;
    e->deck_len = 52;
    or_shuffle_int(rng, e->deck, 52);
    for (int i = 0; i < 2 * np; i++) e->hand[i % np][i / np] = e->deck[--e->deck_len];
    int s = (int)or_mt_interval(rng, (uint64_t)(np - 1));   /* randint(0, N) */
    int b = (s + 1) % np;
    e->in_chips[b] = 2;
    e->in_chips[s] = 1;
    e->game_pointer = (b + 1) % np;
    e->raise_amount = 2;
    e->allowed_raise_num = 4;
    start_new_round(e, e->game_pointer, e->in_chips);
    e->round_counter = 0;
    memcpy(e->prev_raise_nums, prev, sizeof(prev));
    e->use_prev = 1;
}

static void h_step(void *v, or_mt *rng, int a)
{
    (void)rng;
    limit_env *e = (limit_env *)v;
    e->use_prev = 0;
    unsigned legal = legal_mask(e);
    if (a < 0 || a > 3 || !((legal >> a) & 1)) a = ((legal >> CHECK) & 1) ? CHECK : FOLD;
    int p = e->round_pointer, mx = max_raised(e);
    if (a == CALL) {
        e->in_chips[p] += mx - e->raised[p];
        e->raised[p] = mx;
        e->not_raise_num += 1;
    } else if (a == RAISE) {
        e->in_chips[p] += mx - e->raised[p] + e->raise_amount;
        e->raised[p] = mx + e->raise_amount;
        e->have_raised += 1;
        e->not_raise_num = 1;
    } else if (a == FOLD) {
        e->folded[p] = 1;
    } else {
        e->not_raise_num += 1;
    }
    e->round_pointer = (e->round_pointer + 1) % e->np;
    while (e->folded[e->round_pointer]) e->round_pointer = (e->round_pointer + 1) % e->np;
    e->game_pointer = e->round_pointer;
    e->raise_nums[e->round_counter] = e->have_raised;
    if (e->not_raise_num >= e->np) {
        if (e->round_counter == 0) {
            for (int k = 0; k < 3; k++) e->pub[e->npub++] = e->deck[--e->deck_len];
        } else if (e->round_counter <= 2) {
            e->pub[e->npub++] = e->deck[--e->deck_len];
        }
        if (e->round_counter == 1) e->raise_amount = 2 * 2;
        e->round_counter += 1;
        start_new_round(e, e->game_pointer, NULL);
    }
}

static int h_over(const void *v)
{
    const limit_env *e = (const limit_env *)v;
    int alive = 0;
    for (int i = 0; i < e->np; i++) alive += !e->folded[i];
    return alive == 1 || e->round_counter >= 4;
}

static int h_cur(const void *v) { return ((const limit_env *)v)->game_pointer; }

static void h_observe(const void *v, int player, uint8_t *obs, uint8_t *legal)
{
    const limit_env *e = (const limit_env *)v;
    memset(obs, 0, 72);
    for (int k = 0; k < e->npub; k++) obs[e->pub[k]] = 1;
    obs[e->hand[player][0]] = 1;
    obs[e->hand[player][1]] = 1;
    const int *rn = e->use_prev ? e->prev_raise_nums : e->raise_nums;
    for (int i = 0; i < 4; i++) obs[52 + i * 5 + rn[i]] = 1;
    legal[0] = (uint8_t)legal_mask(e);
}

/* ---- 7-card ranking: category (1 high .. 9 straight flush) << 20 | five 4-bit tiebreak ranks (2=0 .. A=12) ---- */
static int top_straight(unsigned mask13)            /* bit r = rank r present (2=0..A=12); returns top rank or -1 */
{
    unsigned m = mask13 << 1 | ((mask13 >> 12) & 1);   /* bit 0 = ace-low */
    for (int top = 13; top >= 4; top--) {
        unsigned w = 0x1Fu << (top - 4);
        if ((m & w) == w) return top - 1;              /* back to 2=0 .. A=12 scale; wheel -> 3 (the five) */
    }
    return -1;
}

uint32_t or_holdem_rank7(const int8_t *cards)
{
    int cnt[13] = {0}, scnt[4] = {0};
    unsigned smask[4] = {0}, all = 0;
    for (int i = 0; i < 7; i++) {
        int c = cards[i], s = c / 13, r = (c % 13 + 12) % 13;   /* A..K -> A=12, 2=0, ... K=11 */
        cnt[r]++;
        scnt[s]++;
        smask[s] |= 1u << r;
        all |= 1u << r;
    }
    int fs = -1;
    for (int s = 0; s < 4; s++) if (scnt[s] >= 5) fs = s;
    uint32_t v[5] = {0, 0, 0, 0, 0};
    int cat;
    if (fs >= 0 && top_straight(smask[fs]) >= 0) {
        cat = 9; v[0] = (uint32_t)top_straight(smask[fs]);
    } else {
        int quad = -1, trips[2] = {-1, -1}, nt = 0, pairs[3] = {-1, -1, -1}, np = 0;
        for (int r = 12; r >= 0; r--) {
            if (cnt[r] == 4) quad = r;
            else if (cnt[r] == 3) { if (nt < 2) trips[nt++] = r; }
            else if (cnt[r] == 2) { if (np < 3) pairs[np++] = r; }
        }
        if (quad >= 0) {
            cat = 8; v[0] = (uint32_t)quad;
            for (int r = 12; r >= 0; r--) if (r != quad && cnt[r]) { v[1] = (uint32_t)r; break; }
        } else if (nt >= 1 && (nt >= 2 || np >= 1)) {
            cat = 7; v[0] = (uint32_t)trips[0];
            int pr = -1;
            if (nt >= 2) pr = trips[1];
            if (np >= 1 && pairs[0] > pr) pr = pairs[0];
            v[1] = (uint32_t)pr;
        } else if (fs >= 0) {
            cat = 6;
            int k = 0;
            for (int r = 12; r >= 0 && k < 5; r--) if (smask[fs] >> r & 1) v[k++] = (uint32_t)r;
        } else if (top_straight(all) >= 0) {
            cat = 5; v[0] = (uint32_t)top_straight(all);
        } else if (nt == 1) {
            cat = 4; v[0] = (uint32_t)trips[0];
            int k = 1;
            for (int r = 12; r >= 0 && k < 3; r--) if (cnt[r] == 1) v[k++] = (uint32_t)r;
        } else if (np >= 2) {
            cat = 3; v[0] = (uint32_t)pairs[0]; v[1] = (uint32_t)pairs[1];
            for (int r = 12; r >= 0; r--) if (cnt[r] && r != pairs[0] && r != pairs[1]) { v[2] = (uint32_t)r; break; }
        } else if (np == 1) {
            cat = 2; v[0] = (uint32_t)pairs[0];
            int k = 1;
            for (int r = 12; r >= 0 && k < 4; r--) if (cnt[r] == 1) v[k++] = (uint32_t)r;
        } else {
            cat = 1;
            int k = 0;
            for (int r = 12; r >= 0 && k < 5; r--) if (cnt[r]) v[k++] = (uint32_t)r;
        }
    }
    return (uint32_t)cat << 20 | v[0] << 16 | v[1] << 12 | v[2] << 8 | v[3] << 4 | v[4];
}

static void h_payoffs(void *v, or_mt *rng, float *out)
{
    /* game.py:233-243: hands of folded players are None, judge_game (or_judger.c), / big_blind. With 2 players the
     * bets are level at a showdown and no split leaves a remainder, so np_random is never drawn; with
     * more, an odd split of a pot among tied winners draws np_random.choice. */
    limit_env *e = (limit_env *)v;
    uint32_t value[HP];
    int pay[HP];
    for (int p = 0; p < e->np; p++) {
        value[p] = 0;
        if (e->folded[p]) continue;
        int8_t c[7];
        c[0] = (int8_t)e->hand[p][0];
        c[1] = (int8_t)e->hand[p][1];
        for (int k = 0; k < 5; k++) c[2 + k] = (int8_t)e->pub[k];
        value[p] = or_holdem_rank7(c);
    }
    int alive = 0;
    for (int p = 0; p < e->np; p++) alive += !e->folded[p];
    if (alive == 1)   /* compare_hands: the one hand left wins without being evaluated (the board may be short) */
        for (int p = 0; p < e->np; p++) value[p] = e->folded[p] ? 0u : 1u;
    or_holdem_judge(e->np, value, e->in_chips, rng, pay);
    for (int p = 0; p < e->np; p++) out[p] = (float)((double)pay[p] / 2.0);
}

const or_game_vt or_limit_vt = {h_info, h_size, h_init, h_step, h_over, h_cur, h_observe, h_payoffs};
