/*
 * or_doudizhu.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of DouDizhu.
 *
 * Follows:
 *   rlcard/games/doudizhu/dealer.py:12-76   init_54_deck sorted by doudizhu_sort_card (stable: S,H,D,C within a rank),
 *                                           one 54-card shuffle, hands deck[0:17],[17:34],[34:51], player 0 is the
 *                                           landlord and takes deck[-3:]
 *   rlcard/games/doudizhu/game.py:23-81     init_game / step (proceed_round, winner when a hand empties, next=(p+1)%3)
 *   rlcard/games/doudizhu/game.py:110-128   get_state: no legal actions once the game is over
 *   rlcard/games/doudizhu/round.py:67-79    update_public (trace, played cards) + Player.play
 *   rlcard/games/doudizhu/player.py:60-108  available_actions: leading (greater_player None or self) -> the judger's
 *                                           playable set; following -> get_gt_cards
 *   rlcard/games/doudizhu/judger.py:124-331 playable_cards_from_hand / calc_playable_cards. The playable set of a hand
 *                                           equals {combo in the 27 471-entry table : contains_cards(hand, combo)}
 *                                           (SURVEY 0.4); restated that way here and pinned by ddz_judger.npz, which
 *                                           holds the reference judger's own sets for thousands of hands
 *   rlcard/games/doudizhu/utils.py:517-621  contains_cards / get_gt_cards (pass + same type with greater weight +
 *                                           bombs unless the target is a bomb + rocket; only pass after a rocket)
 *   rlcard/envs/doudizhu.py:26-188          obs (landlord 790, peasants 901), _cards2array, _get_one_hot_array
 *                                           (0 cards -> index -1 = last slot), _process_action_seq (last 9, '' padded)
 *   rlcard/games/doudizhu/judger.py:350-359 judge_payoffs: landlord wins -> [1,0,0] else [0,1,1]
 * The action table (id -> rank counts, type, weight) is data from the reference's jsondata.zip, handed in by the
 * test harness through or_ddz_set_table().
 */
#include <stdlib.h>
#include <string.h>
#include "or_games.h"

#define NA 27472
#define PASS 27471
#define MAXTRACE 1024

static uint8_t T_cnt[NA][15];
static int16_t T_type[NA];
static int16_t T_weight[NA];
static int T_loaded = 0;

/* counts: [NA][15] u8; type: type index (bomb/rocket identified by name index below); weight: int */
static int T_bomb = -1, T_rocket = -1;
void or_ddz_set_table(const uint8_t *counts, const int16_t *type, const int16_t *weight, int bomb_type,
                      int rocket_type)
{
    memcpy(T_cnt, counts, sizeof(T_cnt));
    memcpy(T_type, type, sizeof(T_type));
    memcpy(T_weight, weight, sizeof(T_weight));
    T_bomb = bomb_type;
    T_rocket = rocket_type;
    T_loaded = 1;
}

typedef struct {
    uint8_t hand[3][15];
    uint8_t played[3][15];
    int16_t trace_p[MAXTRACE];
    int16_t trace_a[MAXTRACE];
    int ntrace;
    int greater;        /* greater_player id or -1 */
    int greater_play;   /* greater_player.played_cards (its last non-pass action id) */
    int winner;         /* -1 = None */
    int current;
} ddz_env;

static int d_info(const or_cfg *cfg, or_info *info)
{
    (void)cfg;
    info->obs_dim = 901; info->num_actions = NA; info->num_players = 3; info->legal_bytes = (NA + 7) / 8;
    return T_loaded ? 0 : -1;
}
static size_t d_size(const or_cfg *cfg) { (void)cfg; return sizeof(ddz_env); }

static void d_init(void *v, or_mt *rng, const or_cfg *cfg)
{
    (void)cfg;
    ddz_env *e = (ddz_env *)v;
    memset(e, 0, sizeof(*e));
    int deck[54];
    for (int i = 0; i < 54; i++) deck[i] = i;      /* sorted deck: index k -> rank k/4 (k<52), 52 = B, 53 = R */
    or_shuffle_int(rng, deck, 54);
    for (int p = 0; p < 3; p++)
        for (int k = 17 * p; k < 17 * p + 17; k++) {
            int c = deck[k];
            e->hand[p][c < 52 ? c / 4 : c - 39]++;
        }
    for (int k = 51; k < 54; k++) {
        int c = deck[k];
        e->hand[0][c < 52 ? c / 4 : c - 39]++;
    }
    e->greater = -1;
    e->greater_play = -1;
    e->winner = -1;
    e->current = 0;
}

static int contains(const uint8_t *hand, int id)
{
    for (int r = 0; r < 15; r++) if (T_cnt[id][r] > hand[r]) return 0;
    return 1;
}

static void legal_bits(const ddz_env *e, uint8_t *bits)
{
    if (e->winner >= 0) return;                                  /* game over -> actions = [] */
    const uint8_t *h = e->hand[e->current];
    if (e->greater < 0 || e->greater == e->current) {
        for (int id = 0; id < PASS; id++) if (contains(h, id)) or_set_bit(bits, id);
        return;
    }
    or_set_bit(bits, PASS);
    int tt = T_type[e->greater_play], tw = T_weight[e->greater_play];
    if (tt == T_rocket) return;
    for (int id = 0; id < PASS; id++) {
        int ty = T_type[id], ok = 0;
        if (ty == tt && T_weight[id] > tw) ok = 1;
        else if (ty == T_rocket) ok = 1;
        else if (ty == T_bomb && tt != T_bomb) ok = 1;
        if (ok && contains(h, id)) or_set_bit(bits, id);
    }
}

/* One id against the rules of legal_bits (no table scan). */
static int is_legal(const ddz_env *e, int a)
{
    if (a < 0 || a >= NA) return 0;
    const int leading = e->greater < 0 || e->greater == e->current;
    if (a == PASS) return !leading;
    if (!contains(e->hand[e->current], a)) return 0;
    if (leading) return 1;
    const int tt = T_type[e->greater_play], tw = T_weight[e->greater_play], ty = T_type[a];
    if (tt == T_rocket) return 0;
    return (ty == tt && T_weight[a] > tw) || ty == T_rocket || (ty == T_bomb && tt != T_bomb);
}

/* The reference applies any id (an illegal one corrupts the hands, player.py:88-108); the engine's ABI replaces an
 * id outside the legal set by the lowest solo when leading and by pass when following (include/cardsim.h cs_step). */
static int decode(const ddz_env *e, int a)
{
    if (is_legal(e, a)) return a;
    if (!(e->greater < 0 || e->greater == e->current)) return PASS;
    for (int r = 0; r < 15; r++)
        if (e->hand[e->current][r]) return r;          /* solo ids 0..14 = ranks (tests/golden/ddz_actions.npz) */
    return PASS;
}

static void d_step(void *v, or_mt *rng, int a)
{
    (void)rng;
    ddz_env *e = (ddz_env *)v;
    a = decode(e, a);
    const int p = e->current;
    if (e->ntrace < MAXTRACE) {
        e->trace_p[e->ntrace] = (int16_t)p;
        e->trace_a[e->ntrace] = (int16_t)a;
        e->ntrace++;
    }
    if (a != PASS) {
        int empty = 1;
        for (int r = 0; r < 15; r++) {
            e->played[p][r] += T_cnt[a][r];
            e->hand[p][r] -= T_cnt[a][r];
            if (e->hand[p][r]) empty = 0;
        }
        e->greater = p;
        e->greater_play = a;
        if (empty) e->winner = p;
    }
    e->current = (p + 1) % 3;
}

static int d_over(const void *v) { return ((const ddz_env *)v)->winner >= 0; }
static int d_cur(const void *v) { return ((const ddz_env *)v)->current; }

static void cards2array(const uint8_t *cnt, uint8_t *out)       /* 54: 4 x 13 column-major + B, R */
{
    memset(out, 0, 54);
    if (!cnt) return;
    for (int r = 0; r < 13; r++)
        for (int k = 0; k < 4 && k < cnt[r]; k++) out[r * 4 + k] = 1;
    out[52] = cnt[13] ? 1 : 0;
    out[53] = cnt[14] ? 1 : 0;
}

static const uint8_t *action_cnt(int a)                          /* 'pass' and '' both encode as zeros */
{
    if (a < 0 || a == PASS) return NULL;
    return T_cnt[a];
}

static void one_hot(int n, int m, uint8_t *out)
{
    memset(out, 0, (size_t)m);
    out[n >= 1 ? n - 1 : m - 1] = 1;
}

static int nleft(const ddz_env *e, int p)
{
    int s = 0;
    for (int r = 0; r < 15; r++) s += e->hand[p][r];
    return s;
}

static void d_observe(const void *v, int self, uint8_t *obs, uint8_t *legal)
{
    const ddz_env *e = (const ddz_env *)v;
    memset(obs, 0, 901);
    uint8_t others[15];
    for (int r = 0; r < 15; r++) others[r] = e->hand[(self + 1) % 3][r] + e->hand[(self + 2) % 3][r];
    cards2array(e->hand[self], obs);
    cards2array(others, obs + 54);
    int last = -1;
    if (e->ntrace > 0) {
        last = e->trace_a[e->ntrace - 1];
        if (last == PASS) last = e->ntrace >= 2 ? e->trace_a[e->ntrace - 2] : -1;
    }
    cards2array(action_cnt(last), obs + 108);
    for (int k = 0; k < 9; k++) {                                /* row k = trace[-9 + k], '' padded in front */
        int idx = e->ntrace - 9 + k;
        cards2array(idx >= 0 ? action_cnt(e->trace_a[idx]) : NULL, obs + 162 + 54 * k);
    }
    if (self == 0) {
        cards2array(e->played[2], obs + 648);
        cards2array(e->played[1], obs + 702);
        one_hot(nleft(e, 2), 17, obs + 756);
        one_hot(nleft(e, 1), 17, obs + 773);
    } else {
        int mate = 3 - self;
        cards2array(e->played[0], obs + 648);
        cards2array(e->played[mate], obs + 702);
        int ll = -1, lt = PASS;
        for (int i = e->ntrace - 1; i >= 0; i--) if (e->trace_p[i] == 0) { ll = e->trace_a[i]; break; }
        for (int i = e->ntrace - 1; i >= 0; i--) if (e->trace_p[i] == mate) { lt = e->trace_a[i]; break; }
        cards2array(action_cnt(ll), obs + 756);
        cards2array(action_cnt(lt), obs + 810);
        one_hot(nleft(e, 0), 20, obs + 864);
        one_hot(nleft(e, mate), 17, obs + 884);
    }
    if (self == e->current) legal_bits(e, legal);
    else legal_bits(e, legal);   /* the reference's legal set always belongs to the current player's state */
}

static void d_payoffs(void *v, or_mt *rng, float *out)
{
    (void)rng;
    const ddz_env *e = (const ddz_env *)v;
    out[0] = e->winner == 0 ? 1.0f : 0.0f;
    out[1] = e->winner == 0 ? 0.0f : 1.0f;
    out[2] = out[1];
}

/* oracle-only helper for the judger KATs: legal set for an arbitrary (hand, previous play) */
void or_ddz_legal_kat(const uint8_t *hand15, int greater_play /* -1 = leading */, uint8_t *bits)
{
    ddz_env e;
    memset(&e, 0, sizeof(e));
    memcpy(e.hand[0], hand15, 15);
    e.winner = -1;
    e.current = 0;
    e.greater = greater_play < 0 ? -1 : 1;
    e.greater_play = greater_play;
    legal_bits(&e, bits);
}

const or_game_vt or_doudizhu_vt = {d_info, d_size, d_init, d_step, d_over, d_cur, d_observe, d_payoffs};
