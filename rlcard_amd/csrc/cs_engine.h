// cs_engine.h -- internal interface between the C ABI (cs_abi.cpp) and the kernels (cs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/cardsim.h"

namespace cs {

// Byte-ring slots of the lane-per-env games' MT19937 streams (cs_ring.h): 16 = 15 blocks twisted per refill from one
// read and one write of the block words (8: seven, 4: three)
constexpr int RING_SLOTS_HOST = 16;
constexpr int RING_ENV_WORDS_HOST = 624 + RING_SLOTS_HOST * 624 / 4;   // u32 per env: block words + the ring bytes

// cs_set_step_record: the single-step kernels also write env `env`'s packed state words to `words`, then -- after a
// system-scope fence that orders every output store of that env's wave -- `seqv` to *seq (both typically in mapped
// host memory), so a single-env host can spin on *seq instead of synchronising the stream
struct StepRecord {
    uint32_t* words;
    uint32_t* seq;
    uint32_t seqv;
    int64_t env;
};

struct Buffers {
    int32_t game;
    int64_t n;
    uint32_t* mt;     // [n][1248]
    uint32_t* ctl;    // [n]
    uint32_t* state;  // [state_words][n] (lane-per-env games) or [n][state_words] (doudizhu, wave per env)
    uint32_t* sctl;   // [n] rollout MT staging: staged stream position | staged count << 16
    uint8_t* sbuf;    // [n][stage bytes] rollout MT staging rows persisted between launches
    const void* table;  // game-specific read-only table (doudizhu action table), or null
    int32_t num_players, num_decks;
    int32_t chips_for_each, dealer_id;   // no-limit hold'em (cs_config; dealer_id -1 = drawn)
    int32_t serial_refill;  // testing hook
    int32_t rng_mode;       // cs_config.rng_mode
    StepRecord rec;         // seq == nullptr: off
    int32_t obs_dim, num_actions, action_bytes;   // cs_game_info of the handle
};

// DMC actor-buffer ring of a handle (cs_dmc.hip): per (env, player) stream, `slots` chunks of T rows
struct DmcRing {
    int32_t T, slots, F;          // rows per chunk, chunks per stream, action feature bytes
    int8_t* st;                   // [streams][slots][T][obs_dim]
    int8_t* act;                  // [streams][slots][T][F]
    float* tgt;                   // [streams][slots][T]
    float* ret;
    uint8_t* dne;
    int64_t* ctr;                 // [streams] rows appended
    int64_t* gstart;              // [streams] first row of the game in progress
    int64_t* emitted;             // [streams] chunks handed out
    int32_t* counts;              // [streams + 1] chunks ready in the last fill (last entry 0)
    int64_t* offsets;             // [streams + 1]
    uint32_t* flag;               // bit 0: rows dropped (ring full)
};

int game_info(int32_t game, const cs_config* cfg, cs_game_info* info);
int64_t stage_bytes_per_env(int32_t game, int32_t num_players, int32_t num_decks);
inline bool state_env_major(int32_t game) { return game == CS_GAME_DOUDIZHU; }

hipError_t launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                       int64_t count, hipStream_t s);
hipError_t launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                          const cs_traj_out& o, hipStream_t s);

// cs_holdem_n.hip: 3..6-player hold'em (Leduc 3..5), used when Buffers::num_players > 2
bool np_supported(int32_t game, int32_t num_players);
int np_game_info(int32_t game, int32_t num_players, cs_game_info* info);
int64_t np_stage_bytes(int32_t game, int32_t num_players);
hipError_t np_launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                          int64_t count, hipStream_t s);
hipError_t np_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t np_launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t np_launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t np_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                             const cs_traj_out& o, hipStream_t s);
// cs_holdem_n10.hip: the same for 7..10 players (Limit / No-limit)
int np10_game_info(int32_t game, int32_t num_players, cs_game_info* info);
int64_t np10_stage_bytes(int32_t game, int32_t num_players);
hipError_t np10_launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                            int64_t count, hipStream_t s);
hipError_t np10_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t np10_launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t np10_launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t np10_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                               const cs_traj_out& o, hipStream_t s);
// cs_holdem_n16.hip: the same for 11..16 players
int np16_game_info(int32_t game, int32_t num_players, cs_game_info* info);
int64_t np16_stage_bytes(int32_t game, int32_t num_players);
hipError_t np16_launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                            int64_t count, hipStream_t s);
hipError_t np16_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t np16_launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t np16_launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t np16_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                               const cs_traj_out& o, hipStream_t s);
// cs_holdem_n22.hip: the same for 17..22 players
int np22_game_info(int32_t game, int32_t num_players, cs_game_info* info);
int64_t np22_stage_bytes(int32_t game, int32_t num_players);
hipError_t np22_launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                            int64_t count, hipStream_t s);
hipError_t np22_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t np22_launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t np22_launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t np22_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                               const cs_traj_out& o, hipStream_t s);
// cs_blackjack_shoe.hip: Blackjack with 2..8-deck shoes or 5..7 players (word-stream RNG, materialised shoe)
bool is_blackjack_shoe(const Buffers& b);
int bjs_game_info(const cs_config* cfg, cs_game_info* info);
hipError_t bjs_launch_seed(const Buffers& b, const uint32_t* keys_dev, const int32_t* klen_dev, int64_t first,
                           int64_t count, hipStream_t s);
hipError_t bjs_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t bjs_launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t bjs_launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t bjs_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                              const cs_traj_out& o, hipStream_t s);

inline bool is_holdem_n(const Buffers& b)
{
    return (b.game == CS_GAME_LEDUC || b.game == CS_GAME_LIMIT || b.game == CS_GAME_NOLIMIT) && b.num_players > 2;
}

// cs_dmc.hip
hipError_t launch_dmc_fill(const Buffers& b, const DmcRing& d, int32_t T, const cs_traj_out& tr, int64_t* ready,
                           int64_t cap, int64_t* nready, int64_t* dst, void** tmp, size_t* tmp_bytes, hipStream_t s);
hipError_t launch_dmc_gather(const DmcRing& d, int32_t state_dim, int32_t obs_dim, const int64_t* chunks,
                             int64_t count, const cs_dmc_batch& o, hipStream_t s);
hipError_t launch_dmc_layer1(const float* X, const int32_t* state_of, const int32_t* ids, int64_t E, int32_t H,
                             const float* Wa, const float* b1, int32_t F, const Buffers& b, float* h1, hipStream_t s);
hipError_t launch_dmc_select(const float* values, const int32_t* counts, const int64_t* offsets, const int32_t* ids,
                             int64_t S, float eps, uint64_t seed, uint64_t t, uint64_t base, int32_t* actions,
                             hipStream_t s);

// cs_cfr.hip: chance-sampling CFR tables on Leduc (device pointers, [CFR_NI][4] fp64 + [CFR_NI] u32 flags)
constexpr int CFR_NI = 2700;
struct CfrTables {
    double* policy;
    double* avg;
    double* regrets;
    uint32_t* flags;
};
// batched mode (n > 1): the deals' table contributions, reduced in a fixed order (cs_cfr.hip); handle-owned
struct CfrScratch {
    void* mem;      // one allocation, grown on demand
    size_t bytes;
};
hipError_t launch_cfr(const Buffers& b, int32_t iterations, int64_t iteration0, const CfrTables& t, CfrScratch* sc,
                      hipStream_t s);

// cs_traj.hip
hipError_t launch_traj_probe(const Buffers& b, int32_t T, const cs_traj_out& tr, int32_t obs_dim, int32_t legal_bytes,
                             int32_t action_bytes, int32_t epw, hipStream_t s);
hipError_t launch_transitions(const Buffers& b, int32_t T, const cs_traj_out& tr, const cs_trans_out& o,
                              hipStream_t s);
hipError_t launch_legal_lists(const Buffers& b, int32_t lb, const uint8_t* legal, int64_t rows, int32_t* counts,
                              int64_t* offsets, int32_t* ids, void** tmp, size_t* tmp_bytes, hipStream_t s);
hipError_t launch_onehot(const int32_t* ids, int64_t count, int32_t na, uint8_t* out, hipStream_t s);
hipError_t launch_copy_state(const Buffers& b, int64_t env, int32_t sw, uint32_t* dst, hipStream_t s);
hipError_t launch_rng_copy(const Buffers& b, int64_t env, int32_t mtw, int32_t column, uint32_t clear_mask,
                           uint32_t* buf, int32_t load, hipStream_t s);   // cs_traj.hip
hipError_t launch_debug_rank7(const int8_t* cards, int64_t n, uint32_t* values, hipStream_t s);   // cs_kernels.hip

namespace ddz {   // cs_doudizhu.hip (seeding goes through the shared k_seed)
hipError_t launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s);
hipError_t launch_step(const Buffers& b, const int32_t* actions, const cs_step_out& o, hipStream_t s);
hipError_t launch_observe(const Buffers& b, int32_t player, const cs_step_out& o, hipStream_t s);
hipError_t launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                          const cs_traj_out& o, hipStream_t s);
hipError_t launch_features(const Buffers& b, const int32_t* ids, int64_t count, uint8_t* out, hipStream_t s);
hipError_t launch_debug_legal(const Buffers& b, const uint8_t* counts, const int32_t* prev, int64_t n,
                              uint8_t* legal, hipStream_t s);
}  // namespace ddz

}  // namespace cs
