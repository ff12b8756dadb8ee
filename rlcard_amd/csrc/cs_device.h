// cs_device.h -- device building blocks shared by every game kernel (gfx950 / CDNA4, wave64).
//
// Per-env RNG contract: numpy's legacy RandomState (MT19937) seeded by init_by_array with the key of
// rlcard/utils/seeding.py:33-113, never re-seeded across resets (rlcard/envs/env.py:228-231). Layout in HBM:
//   mt[env][2][624]  u32, env-major. The env's tempered stream is block0, block1, block0', ... where every block is
//                    the MT19937 twist of the previous one. A lane reads its own words sequentially (every 128-B line
//                    is reused 32 times out of L2), and a block refill is ONE contiguous 2.5 KB read + write done by
//                    the whole wave cooperatively (mt_twist_wave), so the refill traffic is fully coalesced.
//   ctl[env]         u32: bits 0..10 = stream position (0..1247), bit 16 = "the block not holding pos is stale".
// A lane that steps past the end of its current block marks the block it left stale; at the end of every lockstep step
// the wave refills all stale blocks (ballot + one cooperative twist per stale lane). A lane that would enter a stale
// block inside a step (more than 624 draws in one step -- only possible through the rejection loop's tail) twists it
// in-lane (mt_twist_serial): slow, never on the fast path, same numbers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cs_prof.h"

namespace cs {

// rollout output stores: nontemporal (streamed past the caches: written once, GBs per launch, read by the consumer
// long after), measured faster than default-policy stores (Leduc 2.37 -> 2.08 ms, Limit 1.39 -> 1.33 ms per launch)
// and than explicit gfx950 cache-policy bits (round 5, profiles/EXPERIMENTS.md)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void out_store16(uint4* p, const uint4& v)
{
    const u32x4_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (u32x4_t*)p);
}
template <class T>
__device__ __forceinline__ void out_store(T* p, T v)
{
    __builtin_nontemporal_store(v, p);
}

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MT_WORDS = 2 * MT_N;
constexpr uint32_t CTL_STALE = 1u << 16;
constexpr int WAVE = 64;

// runtime game configuration (cs_config): blackjack reads players / decks, no-limit hold'em stacks / dealer
struct GameParams {
    int32_t num_players;
    int32_t num_decks;
    int32_t chips_for_each;   // no-limit: stack per player
    int32_t dealer_id;        // no-limit: -1 = drawn by the first reset (rlcard's None), else fixed
    int32_t rng_mode;         // CS_RNG_MT19937 (reference-compatible) or CS_RNG_PHILOX (cs_ring.h)
};

__device__ __forceinline__ uint32_t mt_temper(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// the low byte of mt_temper(y) (bits 8.. differ): the last two steps only reach the low byte through bits 0..10 and
// 18..25 of the second step's value y2, as y2 ^ (y2 >> 18) ^ ((y2 >> 3) & 0xF1) -- no left shift (a quarter-rate
// instruction on gfx950) in the third step. Both maps are GF(2)-linear; equal on the 32 unit vectors.
__device__ __forceinline__ uint32_t mt_temper_lo8(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    return y ^ (y >> 18) ^ ((y >> 3) & 0xF1u);
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far)
{
    // (cur & 0x80000000) | (nxt & 0x7fffffff) as one bitfield insert (v_bfi_b32) instead of and + and_or; y & 1 is
    // nxt & 1, so the matrix term does not wait for the insert
    uint32_t y;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(y) : "s"(0x7fffffffu), "v"(nxt), "v"(cur));
    return far ^ (y >> 1) ^ ((0u - (nxt & 1u)) & 0x9908b0dfu);
}

// dst = twist(src), one lane, in-order (rare slow path and the seeding kernel)
__device__ inline void mt_twist_serial(const uint32_t* src, uint32_t* dst)
{
    for (int k = 0; k < MT_N - MT_M; k++) dst[k] = mt_mix(src[k], src[k + 1], src[k + MT_M]);
    for (int k = MT_N - MT_M; k < MT_N - 1; k++) dst[k] = mt_mix(src[k], src[k + 1], dst[k - (MT_N - MT_M)]);
    dst[MT_N - 1] = mt_mix(src[MT_N - 1], dst[0], dst[MT_M - 1]);
}

// dst = twist(src) computed by all 64 lanes of the wave (every lane must call it with the same src/dst).
// The recurrence new[k] = f(old[k], old[k+1] | new[0], old[k+397] | new[k-227]) splits into three dependency
// phases of <= 227 words; phase p's dependency for word k sits in the SAME lane and chunk of phase p-1, so
// everything stays in registers; only new[0] crosses lanes (readlane).
__device__ __forceinline__ void mt_twist_wave(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int lane)
{
    constexpr int H = MT_N - MT_M;  // 227
    uint32_t n1[4], n2[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = 64 * c + lane;
        if (k < H) {
            n1[c] = mt_mix(src[k], src[k + 1], src[k + MT_M]);
            dst[k] = n1[c];
        } else {
            n1[c] = 0;
        }
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = H + 64 * c + lane;
        if (k < 2 * H) {
            n2[c] = mt_mix(src[k], src[k + 1], n1[c]);
            dst[k] = n2[c];
        } else {
            n2[c] = 0;
        }
    }
    const uint32_t new0 = __builtin_amdgcn_readlane(n1[0], 0);
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int k = 2 * H + 64 * c + lane;
        if (k < MT_N - 1) dst[k] = mt_mix(src[k], src[k + 1], n2[c]);
        else if (k == MT_N - 1) dst[k] = mt_mix(src[k], new0, n2[c]);
    }
}

// Global-address-space view of a pointer into HBM: pointers rebuilt from integers (readlane) are generic, and generic
// accesses compile to flat_load/flat_store, which count on lgkmcnt too, so every use waits with vmcnt(0) lgkmcnt(0)
// -- draining the wave's outstanding trajectory stores each time (measured in the k_rollout ISA)
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint8_t gu8;
__device__ __forceinline__ gu32* to_global(uint32_t* p) { return (gu32*)p; }

// 64-bit pointer held by lane j (readlane returns int: go through uint32_t so bit 31 of the low half is not
// sign-extended into the high half)
__device__ __forceinline__ gu32* lane_ptr(uint32_t* p, int j)
{
    const uint64_t b = (uint64_t)(uintptr_t)p;
    const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, j);
    const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), j);
    return (gu32*)(uintptr_t)(lo | (hi << 32));
}

// One lane's view of its env's stream. MODE selects how draws are served:
//   STAGE_NONE  one global load per draw (single-step kernels: staging would cost more than it saves);
//   STAGE_LDS   W staged bytes in a per-lane LDS row (the rollout kernels).
// Why staging: lanes sit at different stream positions, so one load per draw is a 64-line gather per wave
// instruction, and a reset's rejection loops issue one such gather per trip of the slowest lane (rocprofv3 on
// k_rollout<Leduc>: TA busy 68% of the kernel, ~300 L1 accesses per wave-step, waves waiting 80% of their cycles).
// Every draw of this engine is random_interval(max <= 53), which looks only at the low 8 bits of the tempered word,
// so at step boundaries (after the refill: both blocks valid) lanes running low restage their next words, temper
// them and keep the low bytes; draws then read LDS, global only as a fallback when a lane outruns its stage.
// Measured on MI355X (tools/ab_rollout.py): staging beat one load per draw by 13-30 %; register variants (a per-draw
// 8-word window, 8/16-word bursts inside the reset, 16 staged bytes in 4 VGPRs) all lost to it.
enum { STAGE_NONE = 0, STAGE_LDS = 2 };

template <int MODE = STAGE_NONE>
struct MtLaneT {
    static constexpr int kMode = MODE;
    uint32_t* base;  // mt + env * MT_WORDS
    uint32_t pos;
    uint32_t stale;
    uint32_t sp, sn;            // stream position of staged byte 0; staged bytes
    const uint8_t* stg;         // STAGE_LDS: this lane's row

    __device__ __forceinline__ void init(uint32_t* p_base, uint32_t p, uint32_t s)
    {
        base = p_base;
        pos = p;
        stale = s;
        sp = 0;
        sn = 0;
        stg = nullptr;
    }

    __device__ __forceinline__ void advance()
    {
        pos++;
        if (pos == MT_N || pos == MT_WORDS) {
            const uint32_t from = pos - MT_N;           // start of the block just finished
            if (pos == MT_WORDS) pos = 0;
            if (stale) mt_twist_serial(base + from, base + pos);   // entering a block nobody refilled yet
            stale = 1;
        }
    }

    __device__ __forceinline__ uint32_t next()
    {
        const uint32_t y = base[pos];
        advance();
        return mt_temper(y);
    }

    __device__ __forceinline__ uint32_t staged_offset() const { return pos >= sp ? pos - sp : pos + MT_WORDS - sp; }

    // low 8 bits of the next tempered word
    __device__ __forceinline__ uint32_t next8()
    {
        uint32_t v;
        if constexpr (MODE == STAGE_NONE) {
            v = mt_temper(base[pos]) & 255u;
        } else {
            const uint32_t k = staged_offset();
            if (k < sn) {
                v = stg[k];
            } else {
                v = mt_temper(base[pos]) & 255u;
            }
        }
        advance();
        return v;
    }

    // numpy random_interval(max): smallest all-ones mask >= max, reject while (u32 & mask) > max
    __device__ __forceinline__ uint32_t interval(uint32_t max)
    {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        if (max <= 255u) {
            do {
                v = next8() & mask;
            } while (v > max);
        } else {
            do {
                v = next() & mask;
            } while (v > max);
        }
        return v;
    }

    // pos += n (n < 624 staged words), with advance()'s block bookkeeping
    __device__ __forceinline__ void advance_by(uint32_t n)
    {
        uint32_t np = pos + n;
        const bool crossed = pos < (uint32_t)MT_N ? np >= (uint32_t)MT_N : np >= (uint32_t)MT_WORDS;
        if (np >= (uint32_t)MT_WORDS) np -= MT_WORDS;
        if (crossed) {
            if (stale) mt_twist_serial(base + (np < (uint32_t)MT_N ? MT_N : 0), base + (np < (uint32_t)MT_N ? 0 : MT_N));
            stale = 1;
        }
        pos = np;
    }

    // random_interval(i) for i = hi, hi - 1, ..., 1 with every result discarded (shuffle positions nobody is dealt
    // from): acceptance only decides how many words are consumed, so the staged bytes are scanned branch-free, four
    // per LDS read. A lane that runs out of staged bytes finishes through interval() (global loads).
    __device__ __forceinline__ void skip_intervals(uint32_t hi)
    {
        uint32_t i = hi;
        if constexpr (MODE == STAGE_LDS) {
            const uint32_t k0 = staged_offset();
            uint32_t k = k0;
            while (i != 0 && k < sn) {
                const uint32_t sh = k & 3u;
                const uint32_t w = *(const uint32_t*)(stg + (k - sh)) >> (8 * sh);
#pragma unroll
                for (uint32_t t = 0; t < 4; t++) {
                    if (t < 4 - sh && i != 0 && k < sn) {
                        const uint32_t u = (w >> (8 * t)) & (0xFFFFFFFFu >> __builtin_clz(i));
                        i -= u <= i ? 1u : 0u;
                        k++;
                    }
                }
            }
            advance_by(k - k0);
        }
        for (; i >= 1; i--) (void)interval(i);
    }
};
using MtLane = MtLaneT<STAGE_NONE>;

// dst[s] = twist(src[s]) for K streams at once, phases interleaved so the K twists' loads overlap (see mt_twist_wave)
template <int K>
__device__ __forceinline__ void mt_twist_wave_k(const gu32* const (&src)[K], gu32* const (&dst)[K], int lane)
{
    constexpr int H = MT_N - MT_M;  // 227
    uint32_t n1[K][4], n2[K][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = 64 * c + lane;
#pragma unroll
        for (int s = 0; s < K; s++) n1[s][c] = k < H ? mt_mix(src[s][k], src[s][k + 1], src[s][k + MT_M]) : 0u;
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = 64 * c + lane;
#pragma unroll
        for (int s = 0; s < K; s++)
            if (k < H) dst[s][k] = n1[s][c];
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = H + 64 * c + lane;
#pragma unroll
        for (int s = 0; s < K; s++) n2[s][c] = k < 2 * H ? mt_mix(src[s][k], src[s][k + 1], n1[s][c]) : 0u;
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = H + 64 * c + lane;
#pragma unroll
        for (int s = 0; s < K; s++)
            if (k < 2 * H) dst[s][k] = n2[s][c];
    }
#pragma unroll
    for (int s = 0; s < K; s++) {
        const uint32_t new0 = __builtin_amdgcn_readlane(n1[s][0], 0);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const int k = 2 * H + 64 * c + lane;
            if (k < MT_N - 1) dst[s][k] = mt_mix(src[s][k], src[s][k + 1], n2[s][c]);
            else if (k == MT_N - 1) dst[s][k] = mt_mix(src[s][k], new0, n2[s][c]);
        }
    }
}

// End-of-step convergence point: the wave refills every stale block of its lanes, two lanes' twists at a time
// (their loads overlap; an odd last lane is paired with itself: identical writes, harmless). All 64 lanes must call.
template <int K = 2, class M>
__device__ __forceinline__ void mt_refill_wave(M& m, int lane)
{
    uint64_t need = __ballot(m.stale != 0);
    while (need) {
        const gu32* src[K];
        gu32* dst[K];
        int j0 = -1;
#pragma unroll
        for (int s = 0; s < K; s++) {
            const int j = need ? __builtin_ctzll(need) : j0;
            need &= need - 1;
            if (s == 0) j0 = j;
            gu32* b = lane_ptr(m.base, j);
            const uint32_t c = __builtin_amdgcn_readlane(m.pos, j) < MT_N ? 0 : MT_N;
            src[s] = b + c;
            dst[s] = b + (MT_N - c);
        }
        mt_twist_wave_k<K>(src, dst, lane);
    }
    m.stale = 0;
    // the refilled words are read later by their owner lane of this same wave: order the stores before those loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// STAGE_LDS rows: W bytes per lane (W multiple of 64), row stride W + PAD (per game): LDS bounds occupancy, so the
// pad is as small as the measurements allow (steady-state A/B on MI355X: Leduc W 64 + 4 fits 6 blocks per CU and is
// 13 % faster than W + 16; Limit W 128 + 8 fits 3 blocks per CU where + 16 fitted 2, and beats + 4 by 1.5 %). The
// persist copies move 16 / 8 / 4 B per lane, whatever the stride allows.
template <int W, int PAD, int ROWS = WAVE>
struct Stage {
    static_assert(W % 16 == 0 && WAVE % (W / 4) == 0, "a staged row is copied by W / 4 lanes of one wave instruction");
    static_assert(PAD % 4 == 0, "rows are written as dwords");
    static constexpr int STRIDE = W + PAD;
    static constexpr int CHUNK = STRIDE % 16 == 0 ? 16 : (STRIDE % 8 == 0 ? 8 : 4);   // bytes per persist copy
    static constexpr int BYTES = ROWS * STRIDE + 16;   // + 16: Leduc's reset reads a 20-B window at any row offset
};

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// STAGE_LDS restage, after mt_refill_wave: every lane with fewer than R staged draws left gets its next W words,
// loaded COALESCED by the whole wave (all 64 lanes read one lane's consecutive words), tempered and packed to bytes
// (lanes 4q gather lanes 4q+1..3 with DPP row shifts: VALU, no LDS traffic). area = the wave's staging area (lane j's
// row at area + j * STRIDE). All 64 lanes must call.
template <int W, int PAD, int R, int B>
__device__ __forceinline__ void mt_restage_wave(MtLaneT<STAGE_LDS>& m, uint8_t* area, int lane, bool valid)
{
    constexpr int STRIDE = Stage<W, PAD>::STRIDE, C = W / WAVE;
    m.stg = area + lane * STRIDE;
    const uint32_t k = m.staged_offset();
    uint64_t todo = __ballot(valid && (k >= m.sn || m.sn - k < (uint32_t)R));
    while (todo) {
        // B needy lanes per pass, all their loads issued before the first is used (a pass with fewer than B left
        // repeats its first lane: same words, same bytes, harmless)
        int js[B];
        js[0] = __builtin_ctzll(todo);
        todo &= todo - 1;
#pragma unroll
        for (int b = 1; b < B; b++) {
            js[b] = todo ? __builtin_ctzll(todo) : js[0];
            todo &= todo - 1;
        }
        uint32_t ps[B], v[B][C];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const gu32* jb = lane_ptr(m.base, js[b]);
            ps[b] = __builtin_amdgcn_readlane(m.pos, js[b]);
#pragma unroll
            for (int c = 0; c < C; c++) {
                uint32_t idx = ps[b] + (uint32_t)(c * WAVE + lane);
                if (idx >= (uint32_t)MT_WORDS) idx -= MT_WORDS;
                v[b][c] = jb[idx];
            }
        }
#pragma unroll
        for (int b = 0; b < B; b++) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                const int t = (int)(mt_temper(v[b][c]) & 255u);
                const uint32_t t1 = (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x101, 0xF, 0xF, true);  // row_shl:1
                const uint32_t t2 = (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x102, 0xF, 0xF, true);  // row_shl:2
                const uint32_t t3 = (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x103, 0xF, 0xF, true);  // row_shl:3
                if ((lane & 3) == 0)
                    *(uint32_t*)(area + js[b] * STRIDE + c * WAVE + lane) =
                        (uint32_t)t | (t1 << 8) | (t2 << 16) | (t3 << 24);
            }
            if (lane == js[b]) {
                m.sp = ps[b];
                m.sn = W;
            }
        }
    }
    wave_sync_lds();
}

// Persist / restore a wave's staging rows (W bytes per env, HBM row-major [env][W]) with coalesced 16-B / 8-B copies, so a
// launch does not restage every lane from scratch. nvalid = envs of this wave.
template <int W, int PAD>
__device__ __forceinline__ void stage_rows_copy(uint8_t* area, uint8_t* hbm_rows, int lane, int nvalid, bool to_lds)
{
    constexpr int STRIDE = Stage<W, PAD>::STRIDE, CH = Stage<W, PAD>::CHUNK, CPR = W / CH;   // chunks per row
#pragma unroll
    for (int i = 0; i < CPR; i++) {
        const int q = i * WAVE + lane, row = q / CPR, col = q - row * CPR;
        if (row < nvalid) {
            uint8_t* l = area + row * STRIDE + col * CH;
            uint8_t* g = hbm_rows + (size_t)q * CH;
            if constexpr (CH == 16) {
                if (to_lds) *(uint4*)l = *(const uint4*)g;
                else *(uint4*)g = *(const uint4*)l;
            } else if constexpr (CH == 8) {
                if (to_lds) *(uint2*)l = *(const uint2*)g;
                else *(uint2*)g = *(const uint2*)l;
            } else {
                if (to_lds) *(uint32_t*)l = *(const uint32_t*)g;
                else *(uint32_t*)g = *(const uint32_t*)l;
            }
        }
    }
    wave_sync_lds();
}

// ---- Philox4x32-10 policy RNG: counter (env, t), key = policy seed. Identical to oracle/or_rng.c. ---------------
__device__ __forceinline__ void philox4(uint64_t seed, uint64_t env, uint64_t blk, uint32_t (&out)[4])
{
    uint32_t c0 = (uint32_t)env, c1 = (uint32_t)(env >> 32), c2 = (uint32_t)blk, c3 = (uint32_t)(blk >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

// The policy's u32 for (env, step t): word t % 4 of Philox4x32-10(key = seed, counter = (env, t / 4)), so one block
// serves four consecutive steps (PolicyRng keeps it in registers across steps). Identical to oracle/or_rng.c.
__device__ __forceinline__ uint32_t philox_u32(uint64_t seed, uint64_t env, uint64_t t)
{
    uint32_t w[4];
    philox4(seed, env, t >> 2, w);
    const uint32_t q = (uint32_t)t & 3u;
    return q == 0 ? w[0] : (q == 1 ? w[1] : (q == 2 ? w[2] : w[3]));
}

struct PolicyRng {
    uint32_t w0, w1, w2, w3;
    // the u32 of absolute step t; steps are visited in order, a new block every fourth one
    __device__ __forceinline__ uint32_t at(uint64_t seed, uint64_t env, uint64_t t, bool first)
    {
        const uint32_t q = (uint32_t)t & 3u;
        if (first || q == 0) {
            uint32_t w[4];
            philox4(seed, env, t >> 2, w);
            w0 = w[0]; w1 = w[1]; w2 = w[2]; w3 = w[3];
        }
        return q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
    }
};

// uniform pick among the set bits of a <= 64-action legal mask (k = floor(r * count / 2^32), k-th set bit)
__device__ __forceinline__ int pick_legal32(uint32_t legal, uint32_t r)
{
    const int count = __popc(legal);
    if (count == 0) return -1;
    int k = (int)__umulhi(r, (uint32_t)count);
    while (k--) legal &= legal - 1;
    return __builtin_ctz(legal);
}
// the same pick for masks of at most A bits (A <= 8), branch-free: the k-th set bit after k clears of the lowest
// (k < A), so a wave's lanes never loop to the largest k among them
template <int A>
__device__ __forceinline__ int pick_legal_small(uint32_t legal, uint32_t r)
{
    static_assert(A >= 1 && A <= 8, "small action sets");
    const uint32_t count = (uint32_t)__popc(legal);
    const uint32_t k = __umulhi(r, count);
#pragma unroll
    for (uint32_t i = 0; i + 1 < (uint32_t)A; i++) legal = i < k ? legal & (legal - 1u) : legal;
    return count == 0 ? -1 : __builtin_ctz(legal);
}
__device__ __forceinline__ int pick_legal(uint64_t legal, uint32_t r)
{
    const int count = __popcll(legal);
    if (count == 0) return -1;
    int k = (int)(((uint64_t)r * (uint64_t)count) >> 32);
    while (k--) legal &= legal - 1;
    return __builtin_ctzll(legal);
}

// ---- coalesced output of per-lane byte rows ------------------------------------------------------------------------
// A wave's 64 envs own 64 consecutive rows of `ROW` bytes in every [.., N, ROW] output, i.e. one contiguous
// 64*ROW-byte span. Lanes build their row as bit-planes (bit b of bits[] = byte b is 1), expand it to bytes in
// registers, stage it through LDS (odd dword stride: conflict-free ds_write_b32), and the wave writes the span
// with 256-B dword stores.
template <int ROW, int ROWS = WAVE>   // ROWS: envs (rows) per wave, lanes >= ROWS hold none
struct RowWriter {
    static_assert(ROW % 4 == 0, "byte rows must be dword multiples");
    static constexpr int DW = ROW / 4;
    static constexpr int LDS_WORDS = ROWS * DW;   // the LDS image IS the output span (row-major, no padding)
    static constexpr int NB = (ROW + 31) / 32;
    static constexpr int Q = (ROWS * DW) / 4;     // 16-B pieces in a full span

    // 4 bits -> 4 bytes of 0/1: x * (1 + 2^7 + 2^14 + 2^21) puts bit i at bit 8i and the four shifted copies of a
    // 4-bit x never overlap (bits 0-3, 7-10, 14-17, 21-24), so one 24-bit multiply + mask does it
    __device__ static __forceinline__ uint32_t expand4(uint32_t x)
    {
        return __umul24(x & 15u, 0x204081u) & 0x01010101u;
    }

    // bits: NB words of a one-bit-per-byte bitmap; out_span: first byte of the wave's 64 rows; nvalid rows written.
    // LDS writes use an odd stride when DW is odd (conflict-free) and 2-way at worst otherwise; the span leaves LDS
    // with ds_read_b128 and goes out with 16-B stores (dword stores if the span is not 16-B aligned or partial).
    __device__ static __forceinline__ void write(uint32_t* lds, const uint32_t (&bits)[NB], uint8_t* out_span,
                                                 int lane, int nvalid, bool wide = true)
    {
        if (lane < ROWS) {
#pragma unroll
            for (int j = 0; j < DW; j++) lds[lane * DW + j] = expand4(bits[j / 8] >> (4 * (j % 8)));
        }
        write_out(lds, bits, out_span, lane, nvalid, wide);
    }
    // the span image in LDS (written by this wave) to the output span
    __device__ static __forceinline__ void write_out(uint32_t* lds, const uint32_t (&)[NB], uint8_t* out_span,
                                                     int lane, int nvalid, bool wide)
    {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (wide && nvalid == ROWS && (((uintptr_t)out_span) & 15u) == 0) {
            uint4* o = (uint4*)out_span;
            const uint4* src = (const uint4*)lds;
#pragma unroll
            for (int j = 0; j < (Q + WAVE - 1) / WAVE; j++) {
                const int q = j * WAVE + lane;
                if (q < Q) out_store16(o + q, src[q]);
            }
        } else {
            uint32_t* o = (uint32_t*)out_span;
            const int total = nvalid * DW;
#pragma unroll
            for (int j = 0; j < DW; j++) {
                const int e = j * WAVE + lane;
                if (e < total) o[e] = lds[e];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
};

// Same span writer for rows of raw byte values (ROW even): words[] holds the row's bytes four per word (byte k in
// byte k % 4 of words[k / 4]); lanes write their row into the LDS image as 16-bit pieces (ROW % 4 == 2) or dwords,
// and the span leaves with 16-B stores when it is a whole, aligned number of 16-B pieces.
template <int ROW, int ROWS = WAVE>
struct RowWriterRaw {
    static_assert(ROW % 2 == 0, "raw rows are staged as 16-bit pieces");
    static constexpr int NW = (ROW + 3) / 4;
    static constexpr int SPAN = ROWS * ROW;
    static constexpr int LDS_WORDS = (SPAN + 3) / 4;

    __device__ static __forceinline__ void write(uint32_t* lds, const uint32_t (&words)[NW], uint8_t* out_span,
                                                 int lane, int nvalid, bool wide = true)
    {
        if (lane < ROWS) {
            if constexpr (ROW % 4 == 0) {
#pragma unroll
                for (int j = 0; j < ROW / 4; j++) lds[lane * (ROW / 4) + j] = words[j];
            } else {
                uint16_t* l16 = (uint16_t*)lds + lane * (ROW / 2);
#pragma unroll
                for (int j = 0; j < ROW / 2; j++) l16[j] = (uint16_t)(words[j / 2] >> (16 * (j & 1)));
            }
        }
        write_out(lds, out_span, lane, nvalid, wide);
    }
    __device__ static __forceinline__ void write_out(uint32_t* lds, uint8_t* out_span, int lane, int nvalid, bool wide)
    {
        wave_sync_lds();
        const int bytes = nvalid * ROW;
        if (SPAN % 16 == 0 && wide && nvalid == ROWS && (((uintptr_t)out_span) & 15u) == 0) {
            uint4* o = (uint4*)out_span;
            const uint4* src = (const uint4*)lds;
#pragma unroll
            for (int j = 0; j < (SPAN / 16 + WAVE - 1) / WAVE; j++) {
                const int q = j * WAVE + lane;
                if (q < SPAN / 16) out_store16(o + q, src[q]);
            }
        } else if (bytes % 4 == 0 && (((uintptr_t)out_span) & 3u) == 0) {
            uint32_t* o = (uint32_t*)out_span;
            for (int e = lane; e < bytes / 4; e += WAVE) o[e] = lds[e];
        } else {
            uint16_t* o = (uint16_t*)out_span;
            const uint16_t* src = (const uint16_t*)lds;
            for (int e = lane; e < bytes / 2; e += WAVE) o[e] = src[e];
        }
        wave_sync_lds();
    }
};

// The span writer for one-hot rows with few ones at known positions (Leduc: K = 4 byte positions per row, a repeated
// position for an absent one): the lanes zero the span image with 16-B LDS stores, then write their K ones as byte
// stores (a wave's LDS operations complete in order), instead of expanding every dword of the row (4 VALU + one LDS
// store per dword). The span leaves LDS exactly as write() sends it.
// RAW: the row is raw bytes (RowWriterRaw) whose last two bytes are the 16-bit value `tail` (No-limit's chips); the
// ones sit among the bytes before them.
template <int ROW, int ROWS, int K, bool RAW = false>
__device__ __forceinline__ void row_write_sparse(uint32_t* lds, const uint32_t (&pos)[K], uint8_t* out_span, int lane,
                                                 int nvalid, bool wide, uint32_t tail = 0)
{
    constexpr int SPAN16 = (ROWS * ROW + 15) / 16;
    uint4* z = (uint4*)lds;
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));   // made here: a hoisted zero register ends up in a scratch spill (vmcnt(0) reload)
#pragma unroll
    for (int j = 0; j < (SPAN16 + WAVE - 1) / WAVE; j++) {
        const int q = j * WAVE + lane;
        if (q < SPAN16) z[q] = make_uint4(zero, zero, zero, zero);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < ROWS) {
        uint8_t* row = (uint8_t*)lds + lane * ROW;
#pragma unroll
        for (int k = 0; k < K; k++) row[pos[k]] = 1;
        if constexpr (RAW) *(uint16_t*)(row + ROW - 2) = (uint16_t)tail;   // ROW even: 2-B aligned
    }
    if constexpr (RAW) {
        RowWriterRaw<ROW, ROWS>::write_out(lds, out_span, lane, nvalid, wide);
    } else {
        uint32_t none[RowWriter<ROW, ROWS>::NB];
        RowWriter<ROW, ROWS>::write_out(lds, none, out_span, lane, nvalid, wide);
    }
}

// XCD-aware block order: the dispatcher hands block b to XCD b % 8 (MI355X: 8 XCDs, each with its own L2), so with
// the identity map neighbouring env ranges -- whose trajectory rows share 128-B lines where a row is not a line
// multiple (DouDizhu's 901 / 3 434-byte rows) -- are written through different L2s, and every shared line reaches HBM
// as two partial writes. xcd_block maps block b to env-block x * q + min(x, r) + b / 8 (x = b % 8, nb = 8 q + r): each
// XCD takes one contiguous eighth of the env range. A bijection of [0, nb) for any nb (results do not depend on it).
constexpr int NUM_XCD = 8;
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb)
{
    const uint32_t x = b % NUM_XCD, q = nb / NUM_XCD, r = nb % NUM_XCD;
    return x * q + (x < r ? x : r) + b / NUM_XCD;
}

// set bit p of a multi-word bitmap without dynamic register indexing
template <int NB>
__device__ __forceinline__ void set_bit(uint32_t (&bits)[NB], int p)
{
#pragma unroll
    for (int j = 0; j < NB; j++) bits[j] |= ((p >> 5) == j) ? (1u << (p & 31)) : 0u;
}

}  // namespace cs
