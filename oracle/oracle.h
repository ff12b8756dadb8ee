/*
 * oracle.h -- CPU restatement of the reference (pmcgannon22/rlcard) env.reset/env.step path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the HIP engine: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker / the CPU baseline,
 * never as the thing measured or shipped. The product (rlcard_amd/) never links or calls it.
 *
 * Pinned against the reference: tests/golden/ fixtures (.npz files) were produced by running the reference Python classes
 * (tests/golden/gen_golden.py); tests/test_oracle_*.py replay every fixture through this library and require
 * bit-exact obs / legal sets / players / done flags / payoffs.
 *
 * It is deliberately written as a scalar, one-env-at-a-time restatement that mirrors the reference's class logic
 * (players, rounds, judgers) rather than the device engine's packed layout, so that a bug in one is not silently
 * shared by the other.
 */
#ifndef RLCARD_AMD_ORACLE_H
#define RLCARD_AMD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- numpy legacy RandomState (MT19937) ------------------------------------------------------------------------ */
typedef struct {
    uint32_t key[624];
    int32_t pos;
    uint64_t ndraw;   /* tempered u32 outputs consumed so far */
    int32_t philox;   /* 1: the engine's CS_RNG_PHILOX byte stream (or_mt_seed_philox) instead of MT19937 */
    uint32_t pkey[2];
} or_mt;

void or_mt_seed_int(or_mt *s, uint32_t seed);                                  /* np.random.seed(int)         */
void or_mt_seed_by_array(or_mt *s, const uint32_t *key, int key_len);          /* RandomState().seed([...])   */
uint32_t or_mt_next(or_mt *s);                                                 /* next tempered u32           */
void or_mt_seed_philox(or_mt *s, const uint32_t *key, int key_len);            /* CS_RNG_PHILOX stream        */
uint64_t or_mt_interval(or_mt *s, uint64_t max);                               /* random_interval(max)        */
void or_mt_fill(const uint32_t *key, int key_len, uint32_t *out, int n);       /* KAT helper                  */
void or_mt_shuffle_kat(const uint32_t *key, int key_len, const int *ns, int count, int16_t *out, int stride);

/* ---- counter-based policy RNG (Philox4x32-10) and the uniform-legal policy of cs_rollout ------------------------ */
void or_philox4(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* policy u32 of (env, step t): word t % 4 of Philox4x32-10(key = seed, counter = (env, t / 4)) */
uint32_t or_philox_u32(uint64_t seed, uint64_t env, uint64_t t);
int or_policy_pick(uint64_t seed, uint64_t env, uint64_t t, const uint8_t *legal_bits, int num_actions);

/* ---- games ------------------------------------------------------------------------------------------------------ */
enum { OR_BLACKJACK = 0, OR_LEDUC = 1, OR_LIMIT = 2, OR_DOUDIZHU = 3, OR_NOLIMIT = 4 };

typedef struct {
    int32_t num_players;  /* blackjack: game_num_players; leduc/limit: 2; doudizhu: 3 */
    int32_t num_decks;    /* blackjack only (0 = infinite) */
    int32_t chips_for_each; /* no-limit only: stack per player (1..255) */
    int32_t dealer_id;      /* no-limit only: -1 = drawn by the first init_game, else fixed */
    int32_t rng_mode;       /* 0 = numpy's MT19937 (the reference), 1 = the engine's CS_RNG_PHILOX stream */
} or_cfg;

typedef struct {
    int32_t obs_dim;      /* max over players (doudizhu: 901) */
    int32_t num_actions;
    int32_t num_players;
    int32_t legal_bytes;  /* ceil(num_actions / 8) */
} or_info;

int or_game_info(int game, const or_cfg *cfg, or_info *info);

/* A batch of independent envs with the exact semantics of the C-ABI (include/cardsim.h):
 *   reset:   init_game on every env; outputs describe the current player's view.
 *   step:    envs whose game is over are re-initialised (action ignored, done=0, reward=0) -- lazy auto-reset;
 *            the others decode the action (illegal id -> reference fallback) and advance one Env.step.
 *   rollout: T lockstep steps with the uniform-legal Philox policy; records the acting player's pre-step view,
 *            the action, the transition's payoffs and done; a finished game is re-initialised immediately.
 * Output layouts (row-major): obs u8 [n][obs_dim], legal u8 [n][legal_bytes] (bit a of byte a/8, LSB first),
 * player u8 [n], reward f32 [n][num_players], done u8 [n]; rollout arrays carry a leading [T].  */
typedef struct or_batch or_batch;

or_batch *or_batch_create(int game, int64_t n, const or_cfg *cfg);
void or_batch_destroy(or_batch *b);
void or_batch_seed(or_batch *b, const uint32_t *keys /* [n][2] */, const int32_t *key_len /* [n] */);
void or_batch_reset(or_batch *b, uint8_t *obs, uint8_t *legal, uint8_t *player, float *reward, uint8_t *done);
void or_batch_step(or_batch *b, const int32_t *actions, uint8_t *obs, uint8_t *legal, uint8_t *player,
                   float *reward, uint8_t *done);
void or_batch_observe(or_batch *b, int64_t env, int player, uint8_t *obs, uint8_t *legal);
void or_batch_rollout(or_batch *b, int32_t T, uint64_t policy_seed, uint64_t t0, uint64_t env_base,
                      uint8_t *obs, uint8_t *legal, uint8_t *player, int32_t *action, float *reward, uint8_t *done,
                      uint8_t *final_obs /* [T][n][P][obs_dim] at done rows, or NULL */);
/* total u32 draws consumed so far by env i (for RNG-position parity checks) */
uint64_t or_batch_draws(or_batch *b, int64_t env);

/* ---- chance-sampling CFR on Leduc Hold'em (agents/cfr_agent.py), or_cfr.c ----------------------------------- */
#define OR_CFR_INFOSETS 2700   /* dense infoset table: ((hand * 4 + public + 1) * 15 + my chips) * 15 + others' */
typedef struct or_cfr or_cfr;
int or_cfr_infoset(const uint8_t *obs /* Leduc obs[36] */);
or_cfr *or_cfr_create(int64_t n, const uint32_t *keys /* [n][2] */, const int32_t *key_len);
void or_cfr_destroy(or_cfr *c);
void or_cfr_train(or_cfr *c, int32_t iterations);           /* `iterations` x CFRAgent.train()              */
void or_cfr_tables(const or_cfr *c, double *policy, double *avg, double *regrets, uint8_t *flags); /* [2700][4] */
uint64_t or_cfr_draws(const or_cfr *c, int64_t env);

/* ---- hold'em evaluator (limitholdem/utils.py compare_hands) ---------------------------------------------------- */
/* cards: 7 card indices (card2index order: suit-major S,H,D,C; rank A..K). Returns a value whose order is
 * the reference's hand order (equal values = split). */
uint32_t or_holdem_rank7(const int8_t *cards);

#ifdef __cplusplus
}
#endif
#endif
