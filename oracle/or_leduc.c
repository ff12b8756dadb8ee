/*
 * or_leduc.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of Leduc Hold'em (2..5 players).
 *
 * Follows, line for line in behaviour:
 *   rlcard/games/leducholdem/dealer.py:4-12    6-card deck [SJ,HJ,SQ,HQ,SK,HK], shuffled at construction
 *   rlcard/games/limitholdem/dealer.py:11-21   shuffle = np_random.shuffle; deal_card = deck.pop()
 *   rlcard/games/leducholdem/game.py:46-95     init_game: hands pop p0..pN-1, SB = randint(0,N), BB=(SB+1)%N
 *   rlcard/games/leducholdem/game.py:97-133    step: proceed_round; round over -> public card, raise 2->4
 *   rlcard/games/leducholdem/game.py:148-178   is_over / get_payoffs (/ big_blind)
 *   rlcard/games/limitholdem/round.py:35-127   start_new_round / proceed_round / get_legal_actions / is_over
 *   rlcard/games/leducholdem/judger.py:11-64   judge_game
 *   rlcard/envs/leducholdem.py:41-96           _extract_state (obs[36]) and _decode_action fallback
 */
#include <string.h>
#include "or_games.h"

enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };
#define LMAXP 5                   /* 6-card deck: N hands + the public card */

typedef struct {
    int np;                       /* game_num_players (envs/env.py:33-39 -> game.py:40-44) */
    int deck[6], deck_len;
    int hand[LMAXP];              /* card id: 0 SJ, 1 HJ, 2 SQ, 3 HQ, 4 SK, 5 HK  -> rank = id / 2 */
    int public_card;              /* -1 = None */
    int in_chips[LMAXP], folded[LMAXP];
    /* LimitHoldemRound */
    int raise_amount, allowed_raise_num, have_raised, not_raise_num, raised[LMAXP], round_pointer;
    int game_pointer, round_counter;
} leduc_env;

static int l_np(const or_cfg *cfg) { return cfg && cfg->num_players > 0 ? cfg->num_players : 2; }

static int l_info(const or_cfg *cfg, or_info *info)
{
    const int np = l_np(cfg);
    if (np < 2 || np > LMAXP) return -1;
    info->obs_dim = 36; info->num_actions = 4; info->num_players = np; info->legal_bytes = 1;
    return 0;
}
static size_t l_size(const or_cfg *cfg) { (void)cfg; return sizeof(leduc_env); }

static int max_raised(const leduc_env *e)
{
    int m = e->raised[0];
    for (int i = 1; i < e->np; i++) if (e->raised[i] > m) m = e->raised[i];
    return m;
}

/* round.py:95-116 -- bitmask over {call, raise, fold, check} */
static unsigned legal_mask(const leduc_env *e)
{
    unsigned m = 0xF;
    int p = e->round_pointer, mx = max_raised(e);
    if (e->have_raised >= e->allowed_raise_num) m &= ~(1u << RAISE);
    if (e->raised[p] < mx) m &= ~(1u << CHECK);
    if (e->raised[p] == mx) m &= ~(1u << CALL);
    return m;
}

static void start_new_round(leduc_env *e, int game_pointer, const int *raised)
{
    e->round_pointer = game_pointer;
    e->have_raised = 0;
    e->not_raise_num = 0;
    for (int i = 0; i < e->np; i++) e->raised[i] = raised ? raised[i] : 0;
}

static void l_init(void *v, or_mt *rng, const or_cfg *cfg)
{
    leduc_env *e = (leduc_env *)v;
    memset(e, 0, sizeof(*e));
    const int np = e->np = l_np(cfg);
    for (int i = 0; i < 6; i++) e->deck[i] = i;
    e->deck_len = 6;
    or_shuffle_int(rng, e->deck, 6);
    for (int i = 0; i < np; i++) e->hand[i] = e->deck[--e->deck_len];
    int s = (int)or_mt_interval(rng, (uint64_t)(np - 1));   /* randint(0, N) */
    int b = (s + 1) % np;
    e->in_chips[b] = 2;   /* big_blind */
    e->in_chips[s] = 1;   /* small_blind */
    e->public_card = -1;
    e->game_pointer = s;
    e->raise_amount = 2;
    e->allowed_raise_num = 2;
    start_new_round(e, e->game_pointer, e->in_chips);
    e->round_counter = 0;
}

static int proceed_round(leduc_env *e, int action)
{
    int p = e->round_pointer, mx = max_raised(e);
    if (action == CALL) {
        int diff = mx - e->raised[p];
        e->raised[p] = mx;
        e->in_chips[p] += diff;
        e->not_raise_num += 1;
    } else if (action == RAISE) {
        int diff = mx - e->raised[p] + e->raise_amount;
        e->raised[p] = mx + e->raise_amount;
        e->in_chips[p] += diff;
        e->have_raised += 1;
        e->not_raise_num = 1;
    } else if (action == FOLD) {
        e->folded[p] = 1;
    } else {
        e->not_raise_num += 1;
    }
    e->round_pointer = (e->round_pointer + 1) % e->np;
    while (e->folded[e->round_pointer]) e->round_pointer = (e->round_pointer + 1) % e->np;
    return e->round_pointer;
}

static void l_step(void *v, or_mt *rng, int a)
{
    (void)rng;
    leduc_env *e = (leduc_env *)v;
    unsigned legal = legal_mask(e);
    if (a < 0 || a > 3 || !((legal >> a) & 1)) a = ((legal >> CHECK) & 1) ? CHECK : FOLD;  /* _decode_action */
    e->game_pointer = proceed_round(e, a);
    if (e->not_raise_num >= e->np) {                                  /* round.is_over() */
        if (e->round_counter == 0) {
            e->public_card = e->deck[--e->deck_len];
            e->raise_amount = 2 * 2;
        }
        e->round_counter += 1;
        start_new_round(e, e->game_pointer, NULL);
    }
}

static int l_over(const void *v)
{
    const leduc_env *e = (const leduc_env *)v;
    int alive = 0;
    for (int i = 0; i < e->np; i++) alive += !e->folded[i];
    return alive == 1 || e->round_counter >= 2;
}

static int l_cur(const void *v) { return ((const leduc_env *)v)->game_pointer; }

static void l_observe(const void *v, int player, uint8_t *obs, uint8_t *legal)
{
    const leduc_env *e = (const leduc_env *)v;
    memset(obs, 0, 36);
    obs[e->hand[player] / 2] = 1;
    if (e->public_card >= 0) obs[e->public_card / 2 + 3] = 1;
    int total = 0;
    for (int i = 0; i < e->np; i++) total += e->in_chips[i];
    obs[e->in_chips[player] + 6] = 1;
    /* others' chips past the 36-slot obs (3+ players): the reference raises IndexError; this ABI sets no bit */
    if (total - e->in_chips[player] + 21 < 36) obs[total - e->in_chips[player] + 21] = 1;
    legal[0] = (uint8_t)legal_mask(e);
}

static void l_payoffs(void *v, or_mt *rng, float *out)
{
    (void)rng;
    leduc_env *e = (leduc_env *)v;
    const int np = e->np;
    int winners[LMAXP] = {0}, fold_count = 0, alive_idx = -1, nwin = 0, total = 0;
    for (int i = 0; i < np; i++) {
        if (e->folded[i]) fold_count++;
        else alive_idx = i;
    }
    if (fold_count == np - 1) winners[alive_idx] = 1;
    for (int i = 0; i < np; i++) nwin += winners[i];
    if (nwin < 1) {   /* the first player (folded or not) whose rank matches the public card */
        for (int i = 0; i < np; i++)
            if (e->hand[i] / 2 == e->public_card / 2) { winners[i] = 1; break; }
    }
    nwin = 0;
    for (int i = 0; i < np; i++) nwin += winners[i];
    if (nwin < 1) {   /* highest rank over all players, folded ones included (judger.py:46-51) */
        int mx = -1;
        for (int i = 0; i < np; i++) if (e->hand[i] / 2 > mx) mx = e->hand[i] / 2;
        for (int i = 0; i < np; i++) if (e->hand[i] / 2 == mx) winners[i] = 1;
    }
    nwin = 0;
    for (int i = 0; i < np; i++) { nwin += winners[i]; total += e->in_chips[i]; }
    double each_win = (double)total / nwin;
    for (int i = 0; i < np; i++) {
        double p = winners[i] ? each_win - e->in_chips[i] : -(double)e->in_chips[i];
        out[i] = (float)(p / 2.0);
    }
}

const or_game_vt or_leduc_vt = {l_info, l_size, l_init, l_step, l_over, l_cur, l_observe, l_payoffs};
