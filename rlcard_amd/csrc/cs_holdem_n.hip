// cs_holdem_n.hip -- the lockstep skeleton (cs_skeleton.h) instantiated for 3..22-player hold'em (cs_holdem_n.h):
// Leduc 3..5, Limit and No-limit 3..6 here; 7..10, 11..16 and 17..22 in cs_holdem_n10.hip / n16.hip / n22.hip (their
// own translation units: they compile in parallel). Reached from the dispatch in cs_kernels.hip when cs_config.num_players > 2.
#include "cs_skeleton.h"
#include "cs_holdem_n.h"

namespace cs {

#define CS_NP_DISPATCH(game, np, CALL)                                            \
    switch (game) {                                                               \
    case CS_GAME_LEDUC:                                                           \
        switch (np) {                                                             \
        case 3: return CALL(LeducN<3>);                                           \
        case 4: return CALL(LeducN<4>);                                           \
        case 5: return CALL(LeducN<5>);                                           \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    case CS_GAME_LIMIT:                                                           \
        switch (np) {                                                             \
        case 3: return CALL(LimitN<3>);                                           \
        case 4: return CALL(LimitN<4>);                                           \
        case 5: return CALL(LimitN<5>);                                           \
        case 6: return CALL(LimitN<6>);                                           \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    case CS_GAME_NOLIMIT:                                                         \
        switch (np) {                                                             \
        case 3: return CALL(NolimitN<3>);                                         \
        case 4: return CALL(NolimitN<4>);                                         \
        case 5: return CALL(NolimitN<5>);                                         \
        case 6: return CALL(NolimitN<6>);                                         \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    default: break;                                                               \
    }

bool np_supported(int32_t game, int32_t np)
{
    switch (game) {
    case CS_GAME_LEDUC: return np >= 3 && np <= 5;
    case CS_GAME_LIMIT:
    case CS_GAME_NOLIMIT: return np >= 3 && np <= 22;
    default: return false;
    }
}

int np_game_info(int32_t game, int32_t np, cs_game_info* info)
{
    if (np > 16) return np22_game_info(game, np, info);
    if (np > 10) return np16_game_info(game, np, info);
    if (np > 6) return np10_game_info(game, np, info);
#define C_(G) (fill_info<G>(info), CS_OK)
    CS_NP_DISPATCH(game, np, C_)
#undef C_
    return CS_E_UNSUPPORTED;
}

int64_t np_stage_bytes(int32_t game, int32_t np)
{
    if (np > 16) return np22_stage_bytes(game, np);
    if (np > 10) return np16_stage_bytes(game, np);
    if (np > 6) return np10_stage_bytes(game, np);
#define C_(G) stage_bytes_of<G>()
    CS_NP_DISPATCH(game, np, C_)
#undef C_
    return 0;
}

hipError_t np_launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                          hipStream_t s)
{
    if (b.num_players > 16) return np22_launch_seed(b, keys, klen, first, count, s);
    if (b.num_players > 10) return np16_launch_seed(b, keys, klen, first, count, s);
    if (b.num_players > 6) return np10_launch_seed(b, keys, klen, first, count, s);
#define C_(G) seed_g<G>(b, keys, klen, first, count, s)
    CS_NP_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
    if (b.num_players > 16) return np22_launch_reset(b, o, s);
    if (b.num_players > 10) return np16_launch_reset(b, o, s);
    if (b.num_players > 6) return np10_launch_reset(b, o, s);
#define C_(G) reset_g<G>(b, o, s)
    CS_NP_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np_launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
    if (b.num_players > 16) return np22_launch_step(b, a, o, s);
    if (b.num_players > 10) return np16_launch_step(b, a, o, s);
    if (b.num_players > 6) return np10_launch_step(b, a, o, s);
#define C_(G) step_g<G>(b, a, o, s)
    CS_NP_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np_launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
    if (b.num_players > 16) return np22_launch_observe(b, p, o, s);
    if (b.num_players > 10) return np16_launch_observe(b, p, o, s);
    if (b.num_players > 6) return np10_launch_observe(b, p, o, s);
#define C_(G) observe_g<G>(b, p, o, s)
    CS_NP_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                             const cs_traj_out& o, hipStream_t s)
{
    if (b.num_players > 16) return np22_launch_rollout(b, T, seed, t0, env_base, o, s);
    if (b.num_players > 10) return np16_launch_rollout(b, T, seed, t0, env_base, o, s);
    if (b.num_players > 6) return np10_launch_rollout(b, T, seed, t0, env_base, o, s);
#define C_(G) rollout_g<G>(b, T, seed, t0, env_base, o, s)
    CS_NP_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace cs
