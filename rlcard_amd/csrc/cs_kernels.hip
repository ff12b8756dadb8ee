// cs_kernels.hip -- lockstep env kernels for gfx950 (one lane = one env, one wave = 64 consecutive envs).
//
// The kernel skeleton (cs_skeleton.h) instantiated for the heads-up hold'em games, Blackjack and DouDizhu's seeding;
// 3..6-player hold'em is instantiated in cs_holdem_n.hip. game_info / dispatch for the C ABI (cs_abi.cpp).
#include "cs_skeleton.h"
#include "cs_leduc.h"
#include "cs_limit.h"
#include "cs_blackjack.h"
#include "cs_doudizhu.h"
#include "cs_nolimit.h"

namespace cs {

int64_t stage_bytes_per_env(int32_t game, int32_t num_players, int32_t num_decks)
{
    if (game == CS_GAME_BLACKJACK && (num_decks >= 2 || num_players > 4)) return 0;   // cs_blackjack_shoe.hip
    switch (game) {
    case CS_GAME_LEDUC: return num_players > 2 ? np_stage_bytes(game, num_players) : stage_bytes_of<Leduc>();
    case CS_GAME_LIMIT: return num_players > 2 ? np_stage_bytes(game, num_players) : stage_bytes_of<Limit>();
    case CS_GAME_BLACKJACK: return num_players <= 1 ? stage_bytes_of<Blackjack<1>>() : stage_bytes_of<Blackjack<4>>();
    case CS_GAME_NOLIMIT: return num_players > 2 ? np_stage_bytes(game, num_players) : stage_bytes_of<Nolimit>();
    default: return 0;
    }
}

int game_info(int32_t game, const cs_config* cfg, cs_game_info* info)
{
    switch (game) {
    case CS_GAME_LEDUC:
        if (cfg && cfg->num_players > 2) return np_game_info(game, cfg->num_players, info);
        if (cfg && cfg->num_players != 0 && cfg->num_players != 2) return CS_E_UNSUPPORTED;
        fill_info<Leduc>(info);
        return CS_OK;
    case CS_GAME_LIMIT:
        if (cfg && cfg->num_players > 2) return np_game_info(game, cfg->num_players, info);
        if (cfg && cfg->num_players != 0 && cfg->num_players != 2) return CS_E_UNSUPPORTED;
        fill_info<Limit>(info);
        return CS_OK;
    case CS_GAME_BLACKJACK: {
        const int np = (cfg && cfg->num_players > 0) ? cfg->num_players : 1;
        const int nd = (cfg && cfg->num_decks >= 0) ? cfg->num_decks : 1;
        if (np > 4 || nd > 1) return bjs_game_info(cfg, info);   // shoes and big tables: cs_blackjack_shoe.hip
        if (np == 1) fill_info<Blackjack<1>>(info);
        else if (np == 2) fill_info<Blackjack<2>>(info);
        else if (np == 3) fill_info<Blackjack<3>>(info);
        else fill_info<Blackjack<4>>(info);
        return CS_OK;
    }
    case CS_GAME_NOLIMIT: {
        const int np = (cfg && cfg->num_players > 0) ? cfg->num_players : 2;
        if (cfg && (cfg->chips_for_each < 0 || cfg->chips_for_each > 255 || cfg->dealer_plus1 < 0 ||
                    cfg->dealer_plus1 > np))
            return CS_E_UNSUPPORTED;
        if (np > 2) return np_game_info(game, np, info);
        if (np != 2) return CS_E_UNSUPPORTED;
        fill_info<Nolimit>(info);
        return CS_OK;
    }
    case CS_GAME_DOUDIZHU:
        if (cfg && cfg->num_players != 0 && cfg->num_players != ddz::P) return CS_E_UNSUPPORTED;
        info->obs_dim = ddz::OBS;
        info->num_actions = ddz::NA;
        info->num_players = ddz::P;
        info->legal_bytes = ddz::LB;
        info->action_bytes = 2;
        info->state_words = ddz::WORDS;
        info->action_feature_dim = 54;
        info->rng_period = 2 * 624;
        info->game_words = ddz::WORDS;
        info->envs_per_wave = 2;   // k_rollout2: one env per half-wave
        return CS_OK;
    default:
        return CS_E_UNSUPPORTED;
    }
}

#define CS_DISPATCH(game, CALL)                                  \
    switch (game) {                                              \
    case CS_GAME_LEDUC: return CALL(Leduc);                      \
    case CS_GAME_LIMIT: return CALL(Limit);                      \
    case CS_GAME_NOLIMIT: return CALL(Nolimit);                  \
    case CS_GAME_BLACKJACK:                                      \
        switch (b.num_players) {                                 \
        case 1: return CALL(Blackjack<1>);                       \
        case 2: return CALL(Blackjack<2>);                       \
        case 3: return CALL(Blackjack<3>);                       \
        default: return CALL(Blackjack<4>);                      \
        }                                                        \
    default: return hipErrorInvalidValue;                        \
    }

// Test hook (cs_debug_holdem_rank7): the showdown evaluator of the hold'em kernels (tally_card + holdem_rank7, the
// functions holdem_showdown and Limit's game end call) on arbitrary 7-card hands, one thread per hand
__global__ __launch_bounds__(BLOCK) void k_debug_rank7(const int8_t* __restrict__ cards, int64_t n, uint32_t* values)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint64_t cnt = 0, sm = 0;
#pragma unroll
    for (int k = 0; k < 7; k++) tally_card((int)cards[i * 7 + k], cnt, sm);
    values[i] = holdem_rank7(cnt, sm);
}

hipError_t launch_debug_rank7(const int8_t* cards, int64_t n, uint32_t* values, hipStream_t s)
{
    hipLaunchKernelGGL(k_debug_rank7, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, cards, n, values);
    return hipGetLastError();
}

hipError_t launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                       hipStream_t s)
{
#define C_(G) seed_g<G>(b, keys, klen, first, count, s)
    if (b.game == CS_GAME_DOUDIZHU) return C_(ddz::SeedView);
    if (is_blackjack_shoe(b)) return bjs_launch_seed(b, keys, klen, first, count, s);
    if (is_holdem_n(b)) return np_launch_seed(b, keys, klen, first, count, s);
    CS_DISPATCH(b.game, C_)
#undef C_
}
hipError_t launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
#define C_(G) reset_g<G>(b, o, s)
    if (b.game == CS_GAME_DOUDIZHU) return ddz::launch_reset(b, o, s);
    if (is_blackjack_shoe(b)) return bjs_launch_reset(b, o, s);
    if (is_holdem_n(b)) return np_launch_reset(b, o, s);
    CS_DISPATCH(b.game, C_)
#undef C_
}
hipError_t launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
#define C_(G) step_g<G>(b, a, o, s)
    if (b.game == CS_GAME_DOUDIZHU) return ddz::launch_step(b, a, o, s);
    if (is_blackjack_shoe(b)) return bjs_launch_step(b, a, o, s);
    if (is_holdem_n(b)) return np_launch_step(b, a, o, s);
    CS_DISPATCH(b.game, C_)
#undef C_
}
hipError_t launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
#define C_(G) observe_g<G>(b, p, o, s)
    if (b.game == CS_GAME_DOUDIZHU) return ddz::launch_observe(b, p, o, s);
    if (is_blackjack_shoe(b)) return bjs_launch_observe(b, p, o, s);
    if (is_holdem_n(b)) return np_launch_observe(b, p, o, s);
    CS_DISPATCH(b.game, C_)
#undef C_
}
hipError_t launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                          const cs_traj_out& o, hipStream_t s)
{
#define C_(G) rollout_g<G>(b, T, seed, t0, env_base, o, s)
    if (b.game == CS_GAME_DOUDIZHU) return ddz::launch_rollout(b, T, seed, t0, env_base, o, s);
    if (is_blackjack_shoe(b)) return bjs_launch_rollout(b, T, seed, t0, env_base, o, s);
    if (is_holdem_n(b)) return np_launch_rollout(b, T, seed, t0, env_base, o, s);
    CS_DISPATCH(b.game, C_)
#undef C_
}

}  // namespace cs
