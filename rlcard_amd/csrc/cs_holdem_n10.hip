// cs_holdem_n10.hip -- the lockstep skeleton instantiated for 7..10-player Limit / No-limit hold'em (cs_holdem_n.h);
// reached through cs_holdem_n.hip's launchers when cs_config.num_players > 6.
#include "cs_skeleton.h"
#include "cs_holdem_n.h"

namespace cs {

#define CS_NP10_DISPATCH(game, np, CALL)                                            \
    switch (game) {                                                               \
    case CS_GAME_LIMIT:                                                           \
        switch (np) {                                                             \
        case 7: return CALL(LimitN<7>);                                           \
        case 8: return CALL(LimitN<8>);                                           \
        case 9: return CALL(LimitN<9>);                                           \
        case 10: return CALL(LimitN<10>);                                         \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    case CS_GAME_NOLIMIT:                                                         \
        switch (np) {                                                             \
        case 7: return CALL(NolimitN<7>);                                         \
        case 8: return CALL(NolimitN<8>);                                         \
        case 9: return CALL(NolimitN<9>);                                         \
        case 10: return CALL(NolimitN<10>);                                       \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    default: break;                                                               \
    }

int np10_game_info(int32_t game, int32_t np, cs_game_info* info)
{
#define C_(G) (fill_info<G>(info), CS_OK)
    CS_NP10_DISPATCH(game, np, C_)
#undef C_
    return CS_E_UNSUPPORTED;
}

int64_t np10_stage_bytes(int32_t game, int32_t np)
{
#define C_(G) stage_bytes_of<G>()
    CS_NP10_DISPATCH(game, np, C_)
#undef C_
    return 0;
}

hipError_t np10_launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                          hipStream_t s)
{
#define C_(G) seed_g<G>(b, keys, klen, first, count, s)
    CS_NP10_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np10_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
#define C_(G) reset_g<G>(b, o, s)
    CS_NP10_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np10_launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
#define C_(G) step_g<G>(b, a, o, s)
    CS_NP10_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np10_launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
#define C_(G) observe_g<G>(b, p, o, s)
    CS_NP10_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np10_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                             const cs_traj_out& o, hipStream_t s)
{
#define C_(G) rollout_g<G>(b, T, seed, t0, env_base, o, s)
    CS_NP10_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace cs
