/* or_games.h -- TEST INFRASTRUCTURE ONLY (see oracle.h). Internal per-game vtable of the oracle. */
#ifndef RLCARD_AMD_OR_GAMES_H
#define RLCARD_AMD_OR_GAMES_H
#include <stddef.h>
#include "oracle.h"

typedef struct {
    int (*info)(const or_cfg *cfg, or_info *info);
    size_t (*env_size)(const or_cfg *cfg);
    void (*init_game)(void *env, or_mt *rng, const or_cfg *cfg);           /* Game.init_game               */
    void (*step)(void *env, or_mt *rng, int action_id);                    /* Env._decode_action + Game.step */
    int (*is_over)(const void *env);
    int (*current_player)(const void *env);
    void (*observe)(const void *env, int player, uint8_t *obs, uint8_t *legal_bits); /* Env.get_state(player) */
    void (*payoffs)(void *env, or_mt *rng, float *out);                    /* Env.get_payoffs              */
} or_game_vt;

extern const or_game_vt or_leduc_vt;
extern const or_game_vt or_limit_vt;
extern const or_game_vt or_blackjack_vt;
extern const or_game_vt or_doudizhu_vt;
extern const or_game_vt or_nolimit_vt;

/* numpy RandomState.shuffle of an int array (Fisher-Yates, i = n-1..1, j = random_interval(i)) */
static inline void or_shuffle_int(or_mt *rng, int *x, int n)
{
    for (int i = n - 1; i >= 1; i--) {
        int j = (int)or_mt_interval(rng, (uint64_t)i);
        int t = x[i]; x[i] = x[j]; x[j] = t;
    }
}

/* limitholdem/judger.py:11-108 for np players (or_judger.c): value[i] = or_holdem_rank7 of player i's seven cards, 0 =
 * hand None (folded); in_chips = chips bet; payoffs = chips won (may draw np_random.choice for odd split remainders) */
#define OR_HOLDEM_MAXP 23   /* 2P + 5 <= 52 dealt cards */
void or_holdem_judge(int np, const uint32_t *value, const int *in_chips, or_mt *rng, int *payoffs);

static inline void or_set_bit(uint8_t *bits, int a) { bits[a >> 3] |= (uint8_t)(1u << (a & 7)); }

#endif
