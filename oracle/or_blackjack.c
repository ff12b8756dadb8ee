/*
 * or_blackjack.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of Blackjack.
 *
 * Follows:
 *   rlcard/games/blackjack/dealer.py:4-37   deck = standard deck (x num_decks unless 0/1), shuffle(np.array(deck)),
 *                                           deal_card: idx = np_random.choice(len(deck)); deck.pop(idx) unless
 *                                           num_decks == 0 (infinite deck)
 *   rlcard/games/blackjack/game.py:22-123   init_game: two rounds of (each player, dealer); step hit/stand; the dealer
 *                                           draws while score < 17 once the last player busts or stands
 *   rlcard/games/blackjack/game.py:160-205  get_state: dealer shows hand[1:] until the game is over; is_over
 *   rlcard/games/blackjack/judger.py:2-73   judge_round / judge_game (2 win, 1 tie, -1 loss) / judge_score
 *   rlcard/envs/blackjack.py:38-103         obs = [score(my hand), score(dealer visible)], payoffs +1/0/-1
 */
#include <string.h>
#include "or_games.h"

#define BJ_MAXP 8
#define BJ_MAXDECK (52 * 8)
#define BJ_MAXHAND 24

typedef struct {
    int num_players, num_decks;
    int deck[BJ_MAXDECK], deck_len;
    int hand[BJ_MAXP + 1][BJ_MAXHAND], nhand[BJ_MAXP + 1];   /* index num_players = dealer */
    int bust[BJ_MAXP + 1], score[BJ_MAXP + 1];
    int winner[BJ_MAXP];
    int game_pointer;
} bj_env;

static int bj_info(const or_cfg *cfg, or_info *info)
{
    info->obs_dim = 2; info->num_actions = 2; info->num_players = cfg->num_players; info->legal_bytes = 1;
    return (cfg->num_players >= 1 && cfg->num_players <= BJ_MAXP && cfg->num_decks >= 0 && cfg->num_decks <= 8)
               ? 0 : -1;
}
static size_t bj_size(const or_cfg *cfg) { (void)cfg; return sizeof(bj_env); }

static int card_score(int c)                    /* rank2score: A 11, 2..9, T/J/Q/K 10; c % 13: A=0, 2=1 .. K=12 */
{
    int r = c % 13;
    if (r == 0) return 11;
    if (r >= 9) return 10;
    return r + 1;
}

static int judge_score(const int *cards, int n)
{
    int score = 0, aces = 0;
    for (int i = 0; i < n; i++) {
        score += card_score(cards[i]);
        if (cards[i] % 13 == 0) aces++;
    }
    while (score > 21 && aces > 0) { aces--; score -= 10; }
    return score;
}

static void deal_card(bj_env *e, or_mt *rng, int who)
{
    int idx = (int)or_mt_interval(rng, (uint64_t)(e->deck_len - 1));
    int c = e->deck[idx];
    if (e->num_decks != 0) {
        for (int k = idx; k < e->deck_len - 1; k++) e->deck[k] = e->deck[k + 1];
        e->deck_len--;
    }
    e->hand[who][e->nhand[who]++] = c;
}

static void judge_round(bj_env *e, int who)
{
    e->score[who] = judge_score(e->hand[who], e->nhand[who]);
    e->bust[who] = e->score[who] > 21;
}

static void bj_init(void *v, or_mt *rng, const or_cfg *cfg)
{
    bj_env *e = (bj_env *)v;
    memset(e, 0, sizeof(*e));
    e->num_players = cfg->num_players;
    e->num_decks = cfg->num_decks;
    int copies = (e->num_decks == 0 || e->num_decks == 1) ? 1 : e->num_decks;
    e->deck_len = 52 * copies;
    for (int i = 0; i < e->deck_len; i++) e->deck[i] = i % 52;
    or_shuffle_int(rng, e->deck, e->deck_len);
    const int P = e->num_players, D = P;
    for (int r = 0; r < 2; r++) {
        for (int j = 0; j < P; j++) deal_card(e, rng, j);
        deal_card(e, rng, D);
    }
    for (int i = 0; i < P; i++) judge_round(e, i);
    judge_round(e, D);
    e->game_pointer = 0;
}

static void finish(bj_env *e, or_mt *rng)
{
    const int P = e->num_players, D = P;
    while (judge_score(e->hand[D], e->nhand[D]) < 17) deal_card(e, rng, D);
    judge_round(e, D);
    for (int i = 0; i < P; i++) {
        if (e->bust[i]) e->winner[i] = -1;
        else if (e->bust[D]) e->winner[i] = 2;
        else if (e->score[i] > e->score[D]) e->winner[i] = 2;
        else if (e->score[i] < e->score[D]) e->winner[i] = -1;
        else e->winner[i] = 1;
    }
    e->game_pointer = 0;
}

static void bj_step(void *v, or_mt *rng, int a)
{
    bj_env *e = (bj_env *)v;
    const int gp = e->game_pointer;
    if (a != 1) {                                   /* actions = ['hit', 'stand']; anything but 'stand' hits */
        deal_card(e, rng, gp);
        judge_round(e, gp);
        if (e->bust[gp]) {
            if (gp >= e->num_players - 1) finish(e, rng);
            else e->game_pointer++;
        }
    } else {
        judge_round(e, gp);
        if (gp >= e->num_players - 1) finish(e, rng);
        else e->game_pointer++;
    }
}

static int bj_over(const void *v)
{
    const bj_env *e = (const bj_env *)v;
    for (int i = 0; i < e->num_players; i++) if (e->winner[i] == 0) return 0;
    return 1;
}

static int bj_cur(const void *v) { return ((const bj_env *)v)->game_pointer; }

static void bj_observe(const void *v, int player, uint8_t *obs, uint8_t *legal)
{
    const bj_env *e = (const bj_env *)v;
    const int D = e->num_players;
    obs[0] = (uint8_t)judge_score(e->hand[player], e->nhand[player]);
    if (bj_over(v)) obs[1] = (uint8_t)judge_score(e->hand[D], e->nhand[D]);
    else obs[1] = (uint8_t)judge_score(e->hand[D] + 1, e->nhand[D] - 1);
    legal[0] = 0x3;
}

static void bj_payoffs(void *v, or_mt *rng, float *out)
{
    (void)rng;
    const bj_env *e = (const bj_env *)v;
    for (int i = 0; i < e->num_players; i++)
        out[i] = e->winner[i] == 2 ? 1.0f : (e->winner[i] == 1 ? 0.0f : -1.0f);
}

const or_game_vt or_blackjack_vt = {bj_info, bj_size, bj_init, bj_step, bj_over, bj_cur, bj_observe, bj_payoffs};
