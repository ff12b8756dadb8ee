/*
 * or_batch.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Batch driver with the C-ABI's semantics (include/cardsim.h), built on the scalar per-game restatements.
 * Env orchestration follows rlcard/envs/env.py:52-86 (reset -> init_game + _extract_state; step -> _decode_action,
 * Game.step, _extract_state); one numpy-legacy MT19937 per env, seeded once (env.py:228-231) and never re-seeded
 * across resets.
 */
#include <stdlib.h>
#include <string.h>
#include "or_games.h"

struct or_batch {
    int game;
    or_cfg cfg;
    or_info info;
    const or_game_vt *vt;
    int64_t n;
    size_t esz;
    uint8_t *envs;
    or_mt *rng;
};

static const or_game_vt *vt_of(int game)
{
    switch (game) {
    case OR_BLACKJACK: return &or_blackjack_vt;
    case OR_LEDUC: return &or_leduc_vt;
    case OR_LIMIT: return &or_limit_vt;
    case OR_DOUDIZHU: return &or_doudizhu_vt;
    case OR_NOLIMIT: return &or_nolimit_vt;
    default: return NULL;
    }
}

int or_game_info(int game, const or_cfg *cfg, or_info *info)
{
    const or_game_vt *vt = vt_of(game);
    if (!vt) return -1;
    return vt->info(cfg, info);
}

or_batch *or_batch_create(int game, int64_t n, const or_cfg *cfg)
{
    const or_game_vt *vt = vt_of(game);
    if (!vt || n <= 0) return NULL;
    or_batch *b = (or_batch *)calloc(1, sizeof(or_batch));
    b->game = game;
    b->cfg = *cfg;
    b->vt = vt;
    vt->info(cfg, &b->info);
    b->n = n;
    b->esz = (vt->env_size(cfg) + 15) & ~(size_t)15;
    b->envs = (uint8_t *)calloc((size_t)n, b->esz);
    b->rng = (or_mt *)calloc((size_t)n, sizeof(or_mt));
    return b;
}

void or_batch_destroy(or_batch *b)
{
    if (!b) return;
    free(b->envs);
    free(b->rng);
    free(b);
}

void or_batch_seed(or_batch *b, const uint32_t *keys, const int32_t *key_len)
{
    for (int64_t i = 0; i < b->n; i++) {
        if (b->cfg.rng_mode == 1) or_mt_seed_philox(&b->rng[i], keys + 2 * i, key_len[i]);
        else or_mt_seed_by_array(&b->rng[i], keys + 2 * i, key_len[i]);
    }
}

static void *env_at(or_batch *b, int64_t i) { return b->envs + (size_t)i * b->esz; }

static void emit(or_batch *b, int64_t i, uint8_t *obs, uint8_t *legal, uint8_t *player)
{
    void *e = env_at(b, i);
    int p = b->vt->current_player(e);
    memset(legal + i * b->info.legal_bytes, 0, (size_t)b->info.legal_bytes);
    b->vt->observe(e, p, obs + i * b->info.obs_dim, legal + i * b->info.legal_bytes);
    player[i] = (uint8_t)p;
}

void or_batch_reset(or_batch *b, uint8_t *obs, uint8_t *legal, uint8_t *player, float *reward, uint8_t *done)
{
    for (int64_t i = 0; i < b->n; i++) {
        b->vt->init_game(env_at(b, i), &b->rng[i], &b->cfg);
        emit(b, i, obs, legal, player);
        memset(reward + i * b->info.num_players, 0, sizeof(float) * b->info.num_players);
        done[i] = (uint8_t)b->vt->is_over(env_at(b, i));
    }
}

void or_batch_step(or_batch *b, const int32_t *actions, uint8_t *obs, uint8_t *legal, uint8_t *player,
                   float *reward, uint8_t *done)
{
    for (int64_t i = 0; i < b->n; i++) {
        void *e = env_at(b, i);
        float *r = reward + i * b->info.num_players;
        memset(r, 0, sizeof(float) * b->info.num_players);
        if (b->vt->is_over(e)) {
            b->vt->init_game(e, &b->rng[i], &b->cfg);
            done[i] = 0;
        } else {
            b->vt->step(e, &b->rng[i], actions[i]);
            done[i] = (uint8_t)b->vt->is_over(e);
            if (done[i]) b->vt->payoffs(e, &b->rng[i], r);
        }
        emit(b, i, obs, legal, player);
    }
}

void or_batch_observe(or_batch *b, int64_t env, int player, uint8_t *obs, uint8_t *legal)
{
    memset(legal, 0, (size_t)b->info.legal_bytes);
    b->vt->observe(env_at(b, env), player, obs, legal);
}

void or_batch_rollout(or_batch *b, int32_t T, uint64_t policy_seed, uint64_t t0, uint64_t env_base,
                      uint8_t *obs, uint8_t *legal, uint8_t *player, int32_t *action, float *reward,
                      uint8_t *done, uint8_t *final_obs)
{
    const int64_t n = b->n;
    const int O = b->info.obs_dim, LB = b->info.legal_bytes, P = b->info.num_players;
    for (int64_t i = 0; i < n; i++) {
        void *e = env_at(b, i);
        if (b->vt->is_over(e)) b->vt->init_game(e, &b->rng[i], &b->cfg);   /* left over by a previous step() */
        for (int32_t t = 0; t < T; t++) {
            const int64_t row = (int64_t)t * n + i;
            uint8_t *lg = legal + row * LB;
            int p = b->vt->current_player(e);
            memset(lg, 0, (size_t)LB);
            b->vt->observe(e, p, obs + row * O, lg);
            player[row] = (uint8_t)p;
            int a = or_policy_pick(policy_seed, env_base + (uint64_t)i, t0 + (uint64_t)t, lg, b->info.num_actions);
            action[row] = a;
            b->vt->step(e, &b->rng[i], a);
            float *r = reward + row * P;
            memset(r, 0, sizeof(float) * P);
            done[row] = (uint8_t)b->vt->is_over(e);
            if (done[row]) {
                b->vt->payoffs(e, &b->rng[i], r);
                if (final_obs) {   /* Env.run's final state of every player (envs/env.py:161-164) */
                    uint8_t scratch[4096];
                    for (int p = 0; p < P; p++) {
                        memset(scratch, 0, (size_t)LB);
                        b->vt->observe(e, p, final_obs + (row * P + p) * O, scratch);
                    }
                }
                b->vt->init_game(e, &b->rng[i], &b->cfg);
            }
        }
    }
}

uint64_t or_batch_draws(or_batch *b, int64_t env) { return b->rng[env].ndraw; }
