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

namespace cs {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MT_WORDS = 2 * MT_N;
constexpr uint32_t CTL_STALE = 1u << 16;
constexpr int WAVE = 64;

// runtime game configuration (cs_config): only blackjack reads it
struct GameParams {
    int32_t num_players;
    int32_t num_decks;
};

__device__ __forceinline__ uint32_t mt_temper(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far)
{
    uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
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

// One lane's view of its env's stream.
struct MtLane {
    uint32_t* base;  // mt + env * MT_WORDS
    uint32_t pos;
    uint32_t stale;

    __device__ __forceinline__ uint32_t next()
    {
        const uint32_t y = base[pos];
        pos++;
        if (pos == MT_N || pos == MT_WORDS) {
            const uint32_t from = pos - MT_N;           // start of the block just finished
            if (pos == MT_WORDS) pos = 0;
            if (stale) mt_twist_serial(base + from, base + pos);   // entering a block nobody refilled yet
            stale = 1;
        }
        return mt_temper(y);
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
        do {
            v = next() & mask;
        } while (v > max);
        return v;
    }
};

// End-of-step convergence point: the wave refills every stale block of its lanes. All 64 lanes must call this.
__device__ __forceinline__ void mt_refill_wave(MtLane& m, int lane)
{
    uint64_t need = __ballot(m.stale != 0);
    while (need) {
        const int j = __builtin_ctzll(need);
        need &= need - 1;
        const uint64_t b = (uint64_t)(uintptr_t)m.base;
        // readlane returns int: go through uint32_t so bit 31 of the low half is not sign-extended into the high half
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, j);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), j);
        const uint32_t* jb = (const uint32_t*)(uintptr_t)(lo | (hi << 32));
        const uint32_t jpos = __builtin_amdgcn_readlane(m.pos, j);
        const uint32_t cur = jpos < MT_N ? 0 : MT_N;
        mt_twist_wave(jb + cur, (uint32_t*)jb + (MT_N - cur), lane);
    }
    m.stale = 0;
    // the refilled words are read later by their owner lane of this same wave: order the stores before those loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---- Philox4x32-10 policy RNG: counter (env, t), key = policy seed. Identical to oracle/or_rng.c. ---------------
__device__ __forceinline__ uint32_t philox_u32(uint64_t seed, uint64_t env, uint64_t t)
{
    uint32_t c0 = (uint32_t)env, c1 = (uint32_t)(env >> 32), c2 = (uint32_t)t, c3 = (uint32_t)(t >> 32);
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
    return c0;
}

// uniform pick among the set bits of a <= 64-action legal mask (k = floor(r * count / 2^32), k-th set bit)
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
template <int ROW>
struct RowWriter {
    static_assert(ROW % 4 == 0, "byte rows must be dword multiples");
    static constexpr int DW = ROW / 4;
    static constexpr int STRIDE = DW | 1;
    static constexpr int LDS_WORDS = WAVE * STRIDE;
    static constexpr int NB = (ROW + 31) / 32;

    __device__ static __forceinline__ uint32_t expand4(uint32_t x)
    {
        return (x & 1u) | ((x & 2u) << 7) | ((x & 4u) << 14) | ((x & 8u) << 21);
    }

    // bits: NB words of a one-bit-per-byte bitmap; out_span: first byte of the wave's 64 rows; nvalid rows written
    __device__ static __forceinline__ void write(uint32_t* lds, const uint32_t (&bits)[NB], uint8_t* out_span,
                                                 int lane, int nvalid)
    {
#pragma unroll
        for (int j = 0; j < DW; j++) lds[lane * STRIDE + j] = expand4(bits[j / 8] >> (4 * (j % 8)));
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t* o = (uint32_t*)out_span;
        const int total = nvalid * DW;
#pragma unroll
        for (int j = 0; j < DW; j++) {
            const int e = j * WAVE + lane;
            if (e < total) {
                const int r = e / DW, c = e - r * DW;
                o[e] = lds[r * STRIDE + c];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
};

// set bit p of a multi-word bitmap without dynamic register indexing
template <int NB>
__device__ __forceinline__ void set_bit(uint32_t (&bits)[NB], int p)
{
#pragma unroll
    for (int j = 0; j < NB; j++) bits[j] |= ((p >> 5) == j) ? (1u << (p & 31)) : 0u;
}

}  // namespace cs
