// cs_holdem_n22.hip -- the lockstep skeleton instantiated for 17..22-player Limit / No-limit hold'em (cs_holdem_n.h);
// reached through cs_holdem_n.hip's launchers when cs_config.num_players is 17..22 (2P + 5 <= 52 dealt cards).
#include "cs_skeleton.h"
#include "cs_holdem_n.h"

namespace cs {

#define CS_NP22_DISPATCH(game, np, CALL)                                            \
    switch (game) {                                                               \
    case CS_GAME_LIMIT:                                                           \
        switch (np) {                                                             \
        case 17: return CALL(LimitN<17>);                                     \
        case 18: return CALL(LimitN<18>);                                     \
        case 19: return CALL(LimitN<19>);                                     \
        case 20: return CALL(LimitN<20>);                                     \
        case 21: return CALL(LimitN<21>);                                     \
        case 22: return CALL(LimitN<22>);                                     \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    case CS_GAME_NOLIMIT:                                                         \
        switch (np) {                                                             \
        case 17: return CALL(NolimitN<17>);                                   \
        case 18: return CALL(NolimitN<18>);                                   \
        case 19: return CALL(NolimitN<19>);                                   \
        case 20: return CALL(NolimitN<20>);                                   \
        case 21: return CALL(NolimitN<21>);                                   \
        case 22: return CALL(NolimitN<22>);                                   \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    default: break;                                                               \
    }

int np22_game_info(int32_t game, int32_t np, cs_game_info* info)
{
#define C_(G) (fill_info<G>(info), CS_OK)
    CS_NP22_DISPATCH(game, np, C_)
#undef C_
    return CS_E_UNSUPPORTED;
}

int64_t np22_stage_bytes(int32_t game, int32_t np)
{
#define C_(G) stage_bytes_of<G>()
    CS_NP22_DISPATCH(game, np, C_)
#undef C_
    return 0;
}

hipError_t np22_launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                          hipStream_t s)
{
#define C_(G) seed_g<G>(b, keys, klen, first, count, s)
    CS_NP22_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np22_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
#define C_(G) reset_g<G>(b, o, s)
    CS_NP22_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np22_launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
#define C_(G) step_g<G>(b, a, o, s)
    CS_NP22_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np22_launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
#define C_(G) observe_g<G>(b, p, o, s)
    CS_NP22_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np22_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                             const cs_traj_out& o, hipStream_t s)
{
#define C_(G) rollout_g<G>(b, T, seed, t0, env_base, o, s)
    CS_NP22_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace cs
