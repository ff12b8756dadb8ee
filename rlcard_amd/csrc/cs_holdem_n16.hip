// cs_holdem_n16.hip -- the lockstep skeleton instantiated for 11..16-player Limit / No-limit hold'em (cs_holdem_n.h);
// reached through cs_holdem_n.hip's launchers when cs_config.num_players is 11..16 (its own translation unit: the
// units compile in parallel).
#include "cs_skeleton.h"
#include "cs_holdem_n.h"

namespace cs {

#define CS_NP16_DISPATCH(game, np, CALL)                                            \
    switch (game) {                                                               \
    case CS_GAME_LIMIT:                                                           \
        switch (np) {                                                             \
        case 11: return CALL(LimitN<11>);                                     \
        case 12: return CALL(LimitN<12>);                                     \
        case 13: return CALL(LimitN<13>);                                     \
        case 14: return CALL(LimitN<14>);                                     \
        case 15: return CALL(LimitN<15>);                                     \
        case 16: return CALL(LimitN<16>);                                     \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    case CS_GAME_NOLIMIT:                                                         \
        switch (np) {                                                             \
        case 11: return CALL(NolimitN<11>);                                   \
        case 12: return CALL(NolimitN<12>);                                   \
        case 13: return CALL(NolimitN<13>);                                   \
        case 14: return CALL(NolimitN<14>);                                   \
        case 15: return CALL(NolimitN<15>);                                   \
        case 16: return CALL(NolimitN<16>);                                   \
        default: break;                                                           \
        }                                                                         \
        break;                                                                    \
    default: break;                                                               \
    }

int np16_game_info(int32_t game, int32_t np, cs_game_info* info)
{
#define C_(G) (fill_info<G>(info), CS_OK)
    CS_NP16_DISPATCH(game, np, C_)
#undef C_
    return CS_E_UNSUPPORTED;
}

int64_t np16_stage_bytes(int32_t game, int32_t np)
{
#define C_(G) stage_bytes_of<G>()
    CS_NP16_DISPATCH(game, np, C_)
#undef C_
    return 0;
}

hipError_t np16_launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                          hipStream_t s)
{
#define C_(G) seed_g<G>(b, keys, klen, first, count, s)
    CS_NP16_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np16_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
#define C_(G) reset_g<G>(b, o, s)
    CS_NP16_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np16_launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
#define C_(G) step_g<G>(b, a, o, s)
    CS_NP16_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np16_launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
#define C_(G) observe_g<G>(b, p, o, s)
    CS_NP16_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}
hipError_t np16_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                             const cs_traj_out& o, hipStream_t s)
{
#define C_(G) rollout_g<G>(b, T, seed, t0, env_base, o, s)
    CS_NP16_DISPATCH(b.game, b.num_players, C_)
#undef C_
    return hipErrorInvalidValue;
}

}  // namespace cs
