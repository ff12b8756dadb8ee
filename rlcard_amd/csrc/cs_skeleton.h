// cs_skeleton.h -- the lockstep kernel skeleton shared by every lane-per-env game (one lane = one env, one wave = EPW
// consecutive envs): k_seed / k_reset / k_step / k_observe / k_rollout over a Game type (cs_leduc.h, cs_limit.h,
// cs_nolimit.h, cs_blackjack.h, cs_holdem_n.h) and their host launchers. Included by the translation units that
// instantiate games (cs_kernels.hip: the heads-up / single-table games; cs_holdem_n.hip: 3..6-player hold'em).
// Integer/branchy work: no MFMA. The bound is HBM (obs/legal/reward rows out, packed state + RNG words in/out).
#pragma once
#include <cstddef>
#include <type_traits>

#include "cs_device.h"
#include "cs_ring.h"
#include "cs_engine.h"
#include "cs_dq.h"

namespace cs {

constexpr int BLOCK = 256;
constexpr int WAVES_PER_BLOCK = BLOCK / WAVE;

__device__ inline void mt_init_by_array(uint32_t* mt, const uint32_t* key, int klen)
{
    uint32_t prev = 19650218u;
    mt[0] = prev;
    for (int i = 1; i < MT_N; i++) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        mt[i] = prev;
    }
    int i = 1, j = 0;
    prev = mt[0];
    for (int k = MT_N; k; k--) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        mt[i] = v;
        prev = v;
        i++;
        j++;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; prev = mt[0]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        const uint32_t v = (mt[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        mt[i] = v;
        prev = v;
        i++;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; prev = mt[0]; i = 1; }
    }
    mt[0] = 0x80000000u;
}

// k_rollout: the lane id made opaque at every step (per game, G::LANE_OPAQUE, default on). Round 5, same box: Limit
// 8.18 -> 8.07 ms and No-limit 9.33 -> 9.10 without it, Blackjack 20.62 -> 20.89 and Leduc even
template <class G, class = void>
struct LaneOpaque {
    static constexpr bool value = true;
};
template <class G>
struct LaneOpaque<G, std::void_t<decltype(G::LANE_OPAQUE)>> {
    static constexpr bool value = G::LANE_OPAQUE;
};
struct LaneCtx {
    int lane, wid;
    int64_t env, wave_first;
    int nvalid;
    bool valid;
};

// EPW envs per wave (lanes >= EPW idle): 64 everywhere but the rollouts of games with too few envs to fill the chip
// (Limit's 262 144 envs are 4 waves per SIMD at 64 per wave; half-full waves double that -- the step is latency-bound)
template <int EPW = WAVE>
__device__ __forceinline__ LaneCtx lane_ctx(int64_t n)
{
    LaneCtx c;
    c.lane = threadIdx.x & (WAVE - 1);
    c.wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);   // wave-uniform: wave_first lives in SGPRs
    const int64_t bx = (int64_t)blockIdx.x;   // (XCD-aware block order, cs_device.h xcd_block: +2 % for Leduc)
    c.wave_first = (bx * WAVES_PER_BLOCK + c.wid) * EPW;
    c.env = c.wave_first + c.lane;
    const int64_t left = n - c.wave_first;
    c.nvalid = left >= EPW ? EPW : (left > 0 ? (int)left : 0);
    c.valid = c.lane < EPW && c.env < n;
    return c;
}

// the lane-per-env games draw from the byte ring (cs_ring.h); invalid lanes get a ring that never needs a refill
template <int MODE = STAGE_NONE>
__device__ __forceinline__ RingLane<MODE> ring_lane(uint32_t* mt, const uint32_t* ctl, const LaneCtx& c)
{
    RingLane<MODE> m;
    if (c.valid) m.init(mt + c.env * RING_ENV_WORDS, ctl[c.env]);
    else m.init(mt, CTL_IDLE);
    return m;
}

// end-of-step refill (flag bit 0: skipped, every block crossing takes the in-lane serial path -- a test variant)
template <class G, class M>
__device__ __forceinline__ void refill(M& m, int lane, int flags)
{
    if (!(flags & 1)) ring_refill_wave(m, lane);
}

// obs rows: staged + coalesced when the row is a dword multiple, per-lane bytes otherwise
template <class G, int ROWS = WAVE>
__device__ __forceinline__ void emit_obs(uint32_t* lds, const uint32_t (&bits)[G::NB], uint8_t* obs, int64_t row0, int flags,
                                         const LaneCtx& c)
{
    if constexpr (G::RAW_OBS && G::OBS % 2 == 0) {
        RowWriterRaw<G::OBS, ROWS>::write(lds, bits, obs + row0 * G::OBS, c.lane, c.nvalid, !(flags & 4));
    } else if constexpr (G::RAW_OBS) {
        if (c.valid) {
            uint8_t* o = obs + (row0 + c.lane) * G::OBS;
#pragma unroll
            for (int k = 0; k < G::OBS; k++) o[k] = (uint8_t)(bits[k >> 2] >> (8 * (k & 3)));
        }
    } else if constexpr (G::OBS % 4 == 0) {
        RowWriter<G::OBS, ROWS>::write(lds, bits, obs + row0 * G::OBS, c.lane, c.nvalid, !(flags & 4));
    } else {
        if (c.valid) {
            uint8_t* o = obs + (row0 + c.lane) * G::OBS;
#pragma unroll
            for (int k = 0; k < G::OBS; k++) o[k] = (uint8_t)((bits[k >> 5] >> (k & 31)) & 1u);
        }
    }
}

// one obs row straight from a lane (final observations: only the lanes whose game just ended write)
template <class G>
__device__ __forceinline__ void write_obs_direct(uint8_t* o, const uint32_t (&bits)[G::NB])
{
    if constexpr (G::RAW_OBS) {
#pragma unroll
        for (int k = 0; k < G::OBS; k++) o[k] = (uint8_t)(bits[k >> 2] >> (8 * (k & 3)));
    } else if constexpr (G::OBS % 4 == 0) {
#pragma unroll
        for (int j = 0; j < G::OBS / 4; j++)
            ((uint32_t*)o)[j] = RowWriter<G::OBS>::expand4(bits[j / 8] >> (4 * (j % 8)));
    } else {
#pragma unroll
        for (int k = 0; k < G::OBS; k++) o[k] = (uint8_t)((bits[k >> 5] >> (k & 31)) & 1u);
    }
}

// games whose obs rows are one-hot with SPARSE_K known positions (observe_pos) write them with row_write_sparse
template <class G, class = void>
struct SparseObs : std::false_type {};
template <class G>
struct SparseObs<G, std::void_t<decltype(G::SPARSE_K)>> : std::bool_constant<(G::SPARSE_K > 0)> {};
template <class G, class = void>
struct SparseK {   // positions per sparse row (1 where the game has none: a placeholder array)
    static constexpr int value = 1;
};
template <class G>
struct SparseK<G, std::void_t<decltype(G::SPARSE_K)>> {
    static constexpr int value = G::SPARSE_K > 0 ? G::SPARSE_K : 1;
};

template <class G>
__device__ __forceinline__ void emit_legal(uint8_t* legal, int64_t row, uint64_t lg)
{
#pragma unroll
    for (int k = 0; k < G::LB; k++) out_store(legal + row * G::LB + k, (uint8_t)(lg >> (8 * k)));
}

// the 8-B reward row's value made opaque before its nontemporal store (per game, G::REWARD_OPAQUE, default off):
// without it the optimizer may split the store back into two float stores and drop the nontemporal hint on the way
// (No-limit's rollout); with it where the hint survives anyway (Leduc, Limit) the step schedules worse (Leduc 4.23 ->
// 4.48 ms, round 5)
template <class G, class = void>
struct RewardOpaque {
    static constexpr bool value = false;
};
template <class G>
struct RewardOpaque<G, std::void_t<decltype(G::REWARD_OPAQUE)>> {
    static constexpr bool value = G::REWARD_OPAQUE;
};
template <class G>
__device__ __forceinline__ void emit_reward(float* reward, int64_t row, const float (&r)[G::P])
{
    if constexpr (G::P == 2) {
        uint64_t v = (uint64_t)__float_as_uint(r[0]) | (uint64_t)__float_as_uint(r[1]) << 32;
        if constexpr (RewardOpaque<G>::value) asm volatile("" : "+v"(v));
        out_store((uint64_t*)(reward + row * 2), v);
    } else {
#pragma unroll
        for (int k = 0; k < G::P; k++) reward[row * G::P + k] = r[k];
    }
}

// LDS words of a wave's obs span image: bit rows (RowWriter, dword multiples), raw byte rows (RowWriterRaw, even)
template <class G, int ROWS>
constexpr int obs_lds_words()
{
    if constexpr (!G::RAW_OBS && G::OBS % 4 == 0) return RowWriter<G::OBS, ROWS>::LDS_WORDS;
    else if constexpr (G::RAW_OBS && G::OBS % 2 == 0) return RowWriterRaw<G::OBS, ROWS>::LDS_WORDS;
    else return 1;
}
template <class G, int ROWS = WAVE>
struct ObsLds {
    static constexpr int WORDS = obs_lds_words<G, ROWS>();
};
template <int W, int PAD, int ROWS, bool LDS>
struct StageBytesOf {
    static constexpr int value = 16;
};
template <int W, int PAD, int ROWS>
struct StageBytesOf<W, PAD, ROWS, true> {
    static constexpr int value = Stage<W, PAD, ROWS>::BYTES;
};
template <class G>
struct StageBytes {
    static constexpr int value = StageBytesOf<G::STAGE_W, G::STAGE_PAD, G::EPW, G::STAGE_MODE == STAGE_LDS>::value;
    // the staged-byte scans read one dword past their last staged byte (RingLane::interval, draw_intervals)
    static_assert(G::STAGE_MODE != STAGE_LDS || G::STAGE_PAD >= 4, "stage rows need a pad of at least a dword");
};
// batch restage threshold (ring_restage_wave): the game's STAGE_RF, else its STAGE_R (restage exactly the needy lanes)
template <class G, class = void>
struct StageRF {
    static constexpr int value = G::STAGE_R;
};
template <class G>
struct StageRF<G, std::void_t<decltype(G::STAGE_RF)>> {
    static constexpr int value = G::STAGE_RF;
};
// restage after the refill, per the game's staging mode (see MtLaneT)
template <class G, class M>
__device__ __forceinline__ void restage(M& m, uint8_t* area, int lane, bool valid)
{
    if constexpr (G::STAGE_MODE == STAGE_LDS)
        ring_restage_wave<G::STAGE_W, G::STAGE_PAD, G::STAGE_R, G::RESTAGE_B, StageRF<G>::value>(m, area, lane, valid);
}
template <class G>
struct Scratch {   // per-lane LDS words of games that keep state in LDS (blackjack); one word per wave otherwise
    static constexpr int WORDS = G::SCRATCH_WORDS > 0 ? G::SCRATCH_WORDS * WAVE : 1;
};
template <class G>
__device__ __forceinline__ uint32_t* scratch_of(uint32_t* wave_area, int lane)
{
    return G::SCRATCH_WORDS > 0 ? wave_area + lane : nullptr;
}
// Env.get_payoffs at the step that ends the game: games whose judge may draw from the env's stream (N-player hold'em's
// odd split remainders, limitholdem/judger.py:80-83) take the lane's RNG
template <class G, class = void>
struct PayoffDraws {
    static constexpr bool value = false;
};
template <class G>
struct PayoffDraws<G, std::void_t<decltype(G::PAYOFF_DRAWS)>> {
    static constexpr bool value = G::PAYOFF_DRAWS;
};
template <class G, class Rng>
__device__ __forceinline__ void game_payoffs(G& g, float (&r)[G::P], Rng& rng)
{
    if constexpr (PayoffDraws<G>::value) g.payoffs(r, rng);
    else g.payoffs(r);
}

// reset of the env's game through its deal queue where the game has one (cs_dq.h)
template <class G, class Rng>
__device__ __forceinline__ void game_reset(G& g, Rng& rng, uint32_t* st, int64_t n, int64_t env)
{
    game_reset_hbm(g, rng, st, n, env);
}

// StepRecord (cs_engine.h): the wave holding env rec.env writes its state words and, after a system-scope fence (it
// waits for every store the wave issued: its obs rows, legal bytes, player, reward, done), the sequence number
template <class G>
__device__ __forceinline__ void step_record(const StepRecord& rec, const uint32_t* st, int64_t n, const LaneCtx& c)
{
    if (rec.seq == nullptr || rec.env < c.wave_first || rec.env >= c.wave_first + WAVE) return;   // wave-uniform
    if (c.valid && c.env == rec.env) {
#pragma unroll
        for (int w = 0; w < G::WORDS; w++) rec.words[w] = st[(int64_t)w * n + c.env];
    }
    __threadfence_system();
    if (c.valid && c.env == rec.env) __hip_atomic_store(rec.seq, rec.seqv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CS_SMEM_ROWS(G, ROWS)                                         \
    __shared__ uint32_t lds[WAVES_PER_BLOCK][ObsLds<G, ROWS>::WORDS]; \
    __shared__ uint32_t scr[WAVES_PER_BLOCK][Scratch<G>::WORDS]
#define CS_SMEM(G) CS_SMEM_ROWS(G, WAVE)

// ------------------------------------------------------------------------------------------------------------------
template <class G>
__global__ __launch_bounds__(BLOCK) void k_seed(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                 const uint32_t* keys, const int32_t* klen, int64_t first,
                                                 int64_t count, int flags, GameParams prm)
{
    __shared__ uint32_t scr[WAVES_PER_BLOCK][Scratch<G>::WORDS];
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const bool valid = i < count;
    const int64_t env = first + i;
    if constexpr (G::RING) {   // byte ring: S0 = init_by_array(key) in wbuf, blocks 0..RING_GEN-1 generated in place
        if (!valid) return;
        uint32_t* wbuf = mt + env * RING_ENV_WORDS;
        const int kl = klen[i] == 2 ? 2 : 1;                    // validated on the host; never trust it here
        const uint32_t phx = prm.rng_mode == CS_RNG_PHILOX ? CTL_PHILOX : 0u;
        const uint32_t kb = seed_blocks(env);                  // blocks 0..kb-1 now (cs_ring.h seed_blocks)
        if (phx) {   // Philox byte stream: key = the init_by_array key, blocks 0..kb-1 into slots 0..kb-1, counter kb
            wbuf[0] = 0u;
            wbuf[1] = keys[2 * i];
            wbuf[2] = kl == 2 ? keys[2 * i + 1] : 0u;
            ring_gen_philox((gu32*)wbuf, SLOT_MASK, 0, 1, (int)kb);
            wbuf[0] = kb;
        } else {
            mt_init_by_array(wbuf, keys + 2 * i, kl);
            for (uint32_t b = 0; b < kb; b++) {     // numpy's first draws: block 0 = twist(S0)
                mt_twist_inplace(wbuf);
                ring_bytes_serial(wbuf, (uint8_t*)(wbuf + MT_N), b);
            }
        }
        G g;
        g.bind(scratch_of<G>(scr[threadIdx.x / WAVE], lane), prm);
        g.blank();
        g.store(st, n, env);
        if constexpr (DqOf<G>::value > 0) st[(int64_t)G::GW * n + env] = 0u;   // empty deal queue
        ctl[env] = 0u | (kb - 1u) << CTL_LAT_SHIFT | phx;   // position 0, latest block in slot kb - 1
        return;
    }
    MtLane m;
    m.init(mt, 0, 0);
    // Philox mode (doudizhu's word layout, cs_doudizhu.hip WaveMt): the key in words 0..1, draw count 0 in word 2
    const bool phx = prm.rng_mode == CS_RNG_PHILOX;   // uniform
    if (valid) {
        uint32_t* base = mt + env * MT_WORDS;
        const int kl = klen[i] == 2 ? 2 : 1;                    // validated on the host; never trust it here
        if (phx) {
            base[0] = keys[2 * i];
            base[1] = kl == 2 ? keys[2 * i + 1] : 0u;
            base[2] = 0u;
        } else {
            mt_init_by_array(base + MT_N, keys + 2 * i, kl);    // S0 in block 1 (scratch)
            mt_twist_serial(base + MT_N, base);                 // block 0 = twist(S0): numpy's first draws
            m.base = base;
            m.stale = 1;                                        // block 1 = twist(block 0), refilled below
        }
        G g;
        g.bind(scratch_of<G>(scr[threadIdx.x / WAVE], lane), prm);
        g.blank();
        g.store(st, n, env);
    }
    if (!phx) {
        if (flags & 1) {
            if (valid) mt_twist_serial(m.base, m.base + MT_N);
            m.stale = 0;
        } else {
            mt_refill_wave(m, lane);
        }
    }
    if (valid) ctl[env] = phx ? CTL_PHILOX : 0u;
}

template <class G>
__global__ __launch_bounds__(BLOCK) void k_reset(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                  cs_step_out out, int flags, GameParams prm, StepRecord rec)
{
    CS_SMEM(G);
    const LaneCtx c = lane_ctx(n);
    RingLane<> m = ring_lane(mt, ctl, c);
    G g;
    g.bind(scratch_of<G>(scr[c.wid], c.lane), prm);
    g.blank();
    if (c.valid) {
        g.load(st, n, c.env);   // the Game object outlives init_game (limit-holdem's raise history, :98/:101)
        game_reset(g, m, st, n, c.env);
    }
    refill<G>(m, c.lane, flags & 1);
    uint32_t bits[G::NB];
    const int p = g.current();
    g.observe(p, bits);
    if (out.obs) emit_obs<G>(lds[c.wid], bits, (uint8_t*)out.obs, c.wave_first, flags, c);
    if (c.valid) {
        if (out.legal) emit_legal<G>((uint8_t*)out.legal, c.env, g.legal());
        if (out.player) ((uint8_t*)out.player)[c.env] = (uint8_t)p;
        if (out.reward) {
            float r[G::P];
#pragma unroll
            for (int k = 0; k < G::P; k++) r[k] = 0.f;
            emit_reward<G>((float*)out.reward, c.env, r);
        }
        if (out.done) ((uint8_t*)out.done)[c.env] = (uint8_t)g.is_over();
        g.store(st, n, c.env);
        ctl[c.env] = m.ctl_word();
    }
    step_record<G>(rec, st, n, c);
}

template <class G>
__global__ __launch_bounds__(BLOCK) void k_step(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                 const int32_t* actions, cs_step_out out, int flags,
                                                 GameParams prm, StepRecord rec)
{
    CS_SMEM(G);
    const LaneCtx c = lane_ctx(n);
    RingLane<> m = ring_lane(mt, ctl, c);
    G g;
    g.bind(scratch_of<G>(scr[c.wid], c.lane), prm);
    g.blank();
    float r[G::P];
#pragma unroll
    for (int k = 0; k < G::P; k++) r[k] = 0.f;
    bool done = false;
    if (c.valid) {
        g.load(st, n, c.env);
        if (g.is_over()) {
            game_reset(g, m, st, n, c.env);
        } else {
            g.step(actions[c.env], m);
            done = g.is_over();
            if (done) game_payoffs(g, r, m);
        }
    }
    refill<G>(m, c.lane, flags & 1);
    uint32_t bits[G::NB];
    const int p = g.current();
    g.observe(p, bits);
    if (out.obs) emit_obs<G>(lds[c.wid], bits, (uint8_t*)out.obs, c.wave_first, flags, c);
    if (c.valid) {
        if (out.legal) emit_legal<G>((uint8_t*)out.legal, c.env, g.legal());
        if (out.player) ((uint8_t*)out.player)[c.env] = (uint8_t)p;
        if (out.reward) emit_reward<G>((float*)out.reward, c.env, r);
        if (out.done) ((uint8_t*)out.done)[c.env] = (uint8_t)done;
        g.store(st, n, c.env);
        ctl[c.env] = m.ctl_word();
    }
    step_record<G>(rec, st, n, c);
}

template <class G>
__global__ __launch_bounds__(BLOCK) void k_observe(const uint32_t* st, int64_t n, int player, cs_step_out out,
                                                    GameParams prm, StepRecord rec)
{
    CS_SMEM(G);
    const LaneCtx c = lane_ctx(n);
    G g;
    g.bind(scratch_of<G>(scr[c.wid], c.lane), prm);
    g.blank();
    if (c.valid) g.load(st, n, c.env);
    uint32_t bits[G::NB];
    g.observe(player, bits);
    if (out.obs) emit_obs<G>(lds[c.wid], bits, (uint8_t*)out.obs, c.wave_first, 0, c);
    if (c.valid) {
        if (out.legal) emit_legal<G>((uint8_t*)out.legal, c.env, g.legal());
        if (out.player) ((uint8_t*)out.player)[c.env] = (uint8_t)g.current();
        if (out.done) ((uint8_t*)out.done)[c.env] = (uint8_t)g.is_over();
    }
    step_record<G>(rec, st, n, c);
}

// k_rollout's arguments as one struct, read from the kernarg segment through a pointer that every step makes opaque
// again (RolloutArgsK): the loop's uses (outputs, policy key, flags) are scalar loads where the step needs them instead
// of SGPRs live for the whole kernel, which the compiler spilled to VGPR lanes and restored with v_readlane (a VALU
// instruction) at every use (ddz::PairArgs, the same for DouDizhu)
struct RolloutArgs {
    uint32_t* mt;
    uint32_t* ctl;
    uint32_t* st;
    int64_t n;
    uint64_t seed, t0, env_base;
    cs_traj_out out;
    GameParams prm;
    uint32_t* sctl;
    uint8_t* sbuf;
    int32_t T, flags;
};
typedef const __attribute__((address_space(4))) RolloutArgs* RolloutArgsK;
// k_rollout reads its argument back through __builtin_amdgcn_kernarg_segment_ptr(), so RolloutArgs must stay the
// kernel's ONLY explicit parameter (then it sits at kernarg offset 0 with exactly the host layout): any new argument
// goes inside the struct
static_assert(std::is_standard_layout<RolloutArgs>::value && std::is_trivially_copyable<RolloutArgs>::value,
              "RolloutArgs is copied into the kernarg segment bytewise");
static_assert(offsetof(RolloutArgs, mt) == 0 && alignof(RolloutArgs) == 8 && sizeof(RolloutArgs) % 8 == 0,
              "RolloutArgs: first kernarg at offset 0, 8-byte aligned");

template <class G>
__global__ __launch_bounds__(BLOCK, G::MIN_WAVES) void k_rollout(RolloutArgs args)
{
    RolloutArgsK ak = (RolloutArgsK)__builtin_amdgcn_kernarg_segment_ptr();
    auto arg = [&]() -> const RolloutArgs& {
        asm volatile("" : "+s"(ak));
        return *(const RolloutArgs*)ak;
    };
    uint32_t* const mt = args.mt;
    uint32_t* const ctl = args.ctl;
    uint32_t* const st = args.st;
    const int64_t n = args.n;
    const int T = args.T, flags = args.flags;
    const GameParams prm = args.prm;
    uint32_t* const sctl = args.sctl;
    uint8_t* const sbuf = args.sbuf;
    CS_SMEM_ROWS(G, G::EPW);
    __shared__ __attribute__((aligned(16))) uint8_t stage[WAVES_PER_BLOCK][StageBytes<G>::value];
    const LaneCtx c = lane_ctx<G::EPW>(n);
    RingLane<G::STAGE_MODE> m = ring_lane<G::STAGE_MODE>(mt, ctl, c);
    // MT staging needs both blocks valid at every restage, i.e. the cooperative refill (flag bit 0 off);
    // flag bit 1 disables it (one global load per draw) for A/B runs and fallback-path tests
    const bool staged = !(flags & 3);
    constexpr bool persist = G::STAGE_MODE == STAGE_LDS;
    uint8_t* rows = nullptr;
    if constexpr (persist) {
        // the staged rows left by the previous launch stay valid while ctl bit 17 is set (single-step kernels and
        // seeding rewrite ctl without it)
        rows = sbuf + c.wave_first * G::STAGE_W;
        if (staged) {
            if (c.valid && ((ctl[c.env] >> 17) & 1u)) {
                const uint32_t w = sctl[c.env];
                m.sp = w & 0xFFFFu;
                m.sn = w >> 16;
            }
            stage_rows_copy<G::STAGE_W, G::STAGE_PAD>(stage[c.wid], rows, c.lane, c.nvalid, true);
        }
    }
    // the deal queues of the wave's envs for the launch in LDS (DQW consecutive words per lane: odd stride)
    constexpr int DQ = DqOf<G>::value, DQW = DqOf<G>::words;
    __shared__ uint32_t dql[DQ > 0 ? WAVES_PER_BLOCK * G::EPW * DQW : 1];
    DqMem q{};
    if constexpr (DQ > 0) {
        q = DqMem{dql + (c.wid * G::EPW + (c.lane < G::EPW ? c.lane : 0)) * DQW, 1};
        if (c.valid) {
#pragma unroll
            for (int w = 0; w < DQW; w++) q.set(w, st[(int64_t)(G::GW + w) * n + c.env]);
        }
    }
    G g;
    g.bind(scratch_of<G>(scr[c.wid], c.lane), prm);
    g.blank();
    if (c.valid) {
        g.load(st, n, c.env);
        if (g.is_over()) {
            if constexpr (DQ > 0) dq_reset(g, m, q);
            else g.reset(m);
        }
    }
    refill<G>(m, c.lane, flags & 1);
    if (staged) restage<G>(m, stage[c.wid], c.lane, c.valid);
    PolicyRng pol;
    const uint64_t genv0 = args.env_base + (uint64_t)c.env;   // the policy counter's env id
    for (int t = 0; t < T; t++) {
        const RolloutArgs& A = arg();
        // the lane id made opaque at every step, so lane-derived values (env id, row and LDS addresses) are recomputed
        // from it instead of held across the step -- at 6 waves per SIMD (80 VGPRs) the held copies were spilled, and
        // a spill reload waits on every store the wave has in flight (vmcnt)
        LaneCtx cl = c;
        if constexpr (LaneOpaque<G>::value) {
            int ol = c.lane;
            asm volatile("" : "+v"(ol));
            cl.lane = ol;
            cl.env = c.wave_first + ol;
        }
        const cs_traj_out& out = A.out;
        uint8_t* obs = (uint8_t*)out.obs;
        uint8_t* legal = (uint8_t*)out.legal;
        uint8_t* player = (uint8_t*)out.player;
        float* reward = (float*)out.reward;
        uint8_t* done_o = (uint8_t*)out.done;
        const uint64_t seed = A.seed, t0 = A.t0;

        const int64_t rowbase = (int64_t)t * n;
        const int p = g.current();
        const uint64_t lg = g.legal();
        uint32_t bits[G::NB];
        g.observe(p, bits);
        // each row stored where it is produced (round 5: the rows after the step's refill / restage loads ran 6-7 %
        // slower on every torch allocation, profiles/EXPERIMENTS.md)
        const uint32_t pr = pol.at(seed, genv0, t0 + (uint64_t)t, t == 0);
        int a;
        if constexpr (G::A <= 8) a = pick_legal_small<G::A>((uint32_t)lg, pr);
        else a = G::A <= 32 ? pick_legal32((uint32_t)lg, pr) : pick_legal(lg, pr);
#if !CS_PROF_NO_OBS
        if constexpr (SparseObs<G>::value) {
            uint32_t pos[SparseK<G>::value];
            const uint32_t tail = g.observe_pos(p, pos);
            row_write_sparse<G::OBS, G::EPW, SparseK<G>::value, G::RAW_OBS>(
                lds[c.wid], pos, obs + (rowbase + c.wave_first) * G::OBS, cl.lane, c.nvalid, !(flags & 4), tail);
        } else {
            emit_obs<G, G::EPW>(lds[c.wid], bits, obs, rowbase + c.wave_first, flags, cl);
        }
#endif
        // the reward row starts from a zero the compiler cannot hoist out of the loop: a loop-invariant zero pair was
        // kept in a scratch spill whose reload, before each step's reward store, waited on vmcnt(0) -- on gfx950 every
        // store the wave had issued (the obs rows): a drain per step
        uint32_t zr = 0;
        asm volatile("" : "+v"(zr));
        float r[G::P];
#pragma unroll
        for (int k = 0; k < G::P; k++) r[k] = __uint_as_float(zr);
        bool done = false;
        if (c.valid) {
            const int64_t row = rowbase + cl.env;
#if !CS_PROF_NO_SMALL
            emit_legal<G>(legal, row, lg);
            out_store(player + row, (uint8_t)p);
#endif
            if constexpr (G::ACTION_BYTES == 1) out_store((uint8_t*)out.action + row, (uint8_t)a);
            else out_store((int16_t*)out.action + row, (int16_t)a);
            g.step(a, m);
            done = g.is_over();
            if (done) {
                game_payoffs(g, r, m);
                if (out.final_obs) {   // Env.run's final state of every player (envs/env.py:161-164)
#pragma unroll
                    for (int q = 0; q < G::P; q++) {
                        uint32_t fb[G::NB];
                        g.observe(q, fb);
                        write_obs_direct<G>((uint8_t*)out.final_obs + (row * G::P + q) * G::OBS, fb);
                    }
                }
            }
#if !CS_PROF_NO_SMALL
            emit_reward<G>(reward, row, r);
            out_store(done_o + row, (uint8_t)done);
#endif
            if constexpr (DQ == 0) {
                if (done) g.reset(m);
            }
        }
        if constexpr (DQ > 0) {
            // a lane ending its game with an empty queue makes every lane with room draw one deal ahead, in lockstep
            constexpr uint32_t CM = (1u << DqOf<G>::cb) - 1u;   // the header's count field
            if (__ballot(c.valid && done && (q.get(0) & CM) == 0u)) {
                if (c.valid && (q.get(0) & CM) < (uint32_t)DQ) dq_push(g, m, q);
            }
            if (c.valid && done) dq_reset(g, m, q);
        }
        refill<G>(m, cl.lane, flags & 1);
        if (staged) restage<G>(m, stage[c.wid], cl.lane, c.valid);
    }
    bool keep = false;
    if constexpr (persist) {
        if (staged) {
            stage_rows_copy<G::STAGE_W, G::STAGE_PAD>(stage[c.wid], rows, c.lane, c.nvalid, false);
            keep = true;
        }
    }
    if (c.valid) {
        g.store(st, n, c.env);
        if constexpr (DQ > 0) {
#pragma unroll
            for (int w = 0; w < DQW; w++) st[(int64_t)(G::GW + w) * n + c.env] = q.get(w);
        }
        ctl[c.env] = m.ctl_word() | ((uint32_t)keep << 17);
        if (keep) sctl[c.env] = m.sp | (m.sn << 16);
    }
}

// ------------------------------------------------------------------------------------------------------------------
static inline GameParams params_of(const Buffers& b)
{
    return GameParams{b.num_players, b.num_decks, b.chips_for_each, b.dealer_id, b.rng_mode};
}
static inline dim3 grid_for(int64_t n, int epw = WAVE)
{
    const int64_t per = (int64_t)WAVES_PER_BLOCK * epw;
    return dim3((unsigned)((n + per - 1) / per));
}

template <class G>
static hipError_t seed_g(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                         hipStream_t s)
{
    hipLaunchKernelGGL(k_seed<G>, grid_for(count), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, keys, klen, first,
                       count, b.serial_refill, params_of(b));
    return hipGetLastError();
}
template <class G>
static hipError_t reset_g(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(k_reset<G>, grid_for(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, o, b.serial_refill,
                       params_of(b), b.rec);
    return hipGetLastError();
}
template <class G>
static hipError_t step_g(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(k_step<G>, grid_for(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, a, o, b.serial_refill,
                       params_of(b), b.rec);
    return hipGetLastError();
}
template <class G>
static hipError_t observe_g(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(k_observe<G>, grid_for(b.n), dim3(BLOCK), 0, s, b.state, b.n, p, o, params_of(b), b.rec);
    return hipGetLastError();
}
template <class G>
static hipError_t rollout_g(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                            const cs_traj_out& o, hipStream_t s)
{
    const RolloutArgs a{b.mt, b.ctl, b.state, b.n, seed, t0, env_base, o, params_of(b), b.sctl, b.sbuf, T, b.serial_refill};
    hipLaunchKernelGGL(k_rollout<G>, grid_for(b.n, G::EPW), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

template <class G>
static void fill_info(cs_game_info* info)
{
    info->obs_dim = G::OBS;
    info->num_actions = G::A;
    info->num_players = G::P;
    info->legal_bytes = G::LB;
    info->action_bytes = G::ACTION_BYTES;
    info->state_words = G::WORDS;
    info->action_feature_dim = G::A;
    info->rng_period = (int32_t)RING;
    info->deal_queue_depth = DqOf<G>::value;
    info->game_words = G::WORDS - DqOf<G>::words;
    info->envs_per_wave = G::EPW;
}

template <class G>
static int64_t stage_bytes_of() { return G::STAGE_MODE == STAGE_LDS ? G::STAGE_W : 0; }

}  // namespace cs
