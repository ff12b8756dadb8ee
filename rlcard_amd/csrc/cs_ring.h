// cs_ring.h -- the per-env MT19937 stream of the lane-per-env games as a ring of tempered low BYTES.
//
// Every draw of Leduc / Limit / No-limit Hold'em / Blackjack is numpy's random_interval(max <= 52), which reads only
// the low 8 bits of a tempered output word (cs_device.h, MtLaneT). So the stream does not need to be kept as words:
// per env the engine holds
//   wbuf[624]  u32       the untempered state words of the LATEST generated block L (the only input of the next twist)
//   ring[S][624] u8      the low bytes of the tempered outputs of blocks L-S+1 .. L, block b in slot b % S
// (S = RING_SLOTS = 16: 624 + 2 496 u32 per env). A refill twists S - 1 = 15 blocks in a row in registers --
// L+1 .. L+15 -- writes their bytes into the consumed slots and only the last block's words back to wbuf.
// Per 9 360 draws that is one 2.5 KB word read + one 2.5 KB word write (0.53 B per draw; 8 slots 1.14, 4 slots 2.67) + the bytes written and later read, where the word layout moved ~12 B per draw (block
// read + block write by the refill, and a 4-B word re-read per draw to temper it). Staging (restage into the LDS rows)
// becomes a byte copy: no tempering, no packing.
//
// ctl[env] u32: bits 0..13 = ring position (draws consumed mod RING), bits 19..22 = slot of block L, bit 17 = the
// rollout's staged LDS rows are valid (cs_kernels.hip). A lane needs a refill when it is inside block L; the
// wave refills at step boundaries (ring_refill_wave); a lane that would step past L inside a step (more than 624
// draws in one step: only a rejection loop's tail) generates in-lane (ring_gen_serial): slow, never on the fast path,
// same numbers.
//
// Philox mode (cs_config.rng_mode = CS_RNG_PHILOX, ctl bit 18; not seed-compatible with the reference): the ring
// layout, staging and every game's draw code stay as they are, but a refill fills the S - 1 slots with Philox4x32-10
// bytes -- key = the env's init_by_array key, counter = (absolute block index, 16-byte chunk) -- instead of twisting:
// wbuf holds only the block counter and the key (words 0..2), so the refill reads nothing and writes the ring bytes
// (~2 B per draw: written once, read once).
#pragma once
#include "cs_device.h"
#include "cs_engine.h"

namespace cs {

// Ring slots (RING_SLOTS_HOST, cs_engine.h): a refill twists SLOTS - 1 blocks in a row from one read of wbuf and writes
// wbuf back once, so the block-word traffic per draw is 2 x 2 496 B / ((SLOTS - 1) x 624): 4 slots 2.67 B/draw, 8 slots
// 1.14 B/draw (per env 624 + SLOTS x 156 u32 = RING_ENV_WORDS).
constexpr int RING_SLOTS = RING_SLOTS_HOST;
static_assert(RING_SLOTS == 4 || RING_SLOTS == 8 || RING_SLOTS == 16, "ring slots: a power of two, position < 2^14");
constexpr uint32_t SLOT_MASK = (uint32_t)RING_SLOTS - 1u;
constexpr int RING_GEN = RING_SLOTS - 1;        // blocks generated per refill
constexpr uint32_t RING = RING_SLOTS * MT_N;    // ring bytes: 2 496 (4 slots) / 4 992 (8 slots)
static_assert(RING_ENV_WORDS_HOST == MT_N + RING_SLOTS * MT_N / 4, "host and device agree on the ring footprint");
constexpr int RING_ENV_WORDS = RING_ENV_WORDS_HOST;   // u32 per env in the mt buffer: wbuf + the ring bytes
constexpr uint32_t CTL_POS_MASK = 0x3FFFu;   // ctl bits 0..13: ring position
constexpr int CTL_LAT_SHIFT = 19;            // ctl bits 19..22: slot of the latest block (16..18: flags)
constexpr uint32_t CTL_PHILOX = 1u << 18;       // ctl bit: the env's stream is the Philox byte stream
constexpr int PHX_CHUNKS = MT_N / 16;           // 39 Philox blocks (16 bytes) per ring block
// ctl word of a lane that holds no env (tail lanes of a wave): position 0 inside the latest block, so it never
// reaches a refill (cs_skeleton.h ring_lane, cs_cfr.hip)
constexpr uint32_t CTL_IDLE = (uint32_t)(RING_GEN - 1) << CTL_LAT_SHIFT;

__device__ __forceinline__ uint32_t shfl(uint32_t v, int src_lane)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// numpy's twist (genrand_int32's reload), in place: mt[k] only reads mt[k+1], mt[k+397] (not yet rewritten) and the
// already-new mt[k-227]
__device__ inline void mt_twist_inplace(uint32_t* mt)
{
    for (int k = 0; k < MT_N - MT_M; k++) mt[k] = mt_mix(mt[k], mt[k + 1], mt[k + MT_M]);
    for (int k = MT_N - MT_M; k < MT_N - 1; k++) mt[k] = mt_mix(mt[k], mt[k + 1], mt[k + MT_M - MT_N]);
    mt[MT_N - 1] = mt_mix(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
}

// bytes of one block (low byte of every tempered word) into ring slot `slot`, one lane
__device__ inline void ring_bytes_serial(const uint32_t* w, uint8_t* ring, uint32_t slot)
{
    uint32_t* dst = (uint32_t*)(ring + slot * MT_N);
    for (int i = 0; i < MT_N / 4; i++) {
        const uint32_t* q = w + 4 * i;
        dst[i] = (mt_temper(q[0]) & 255u) | (mt_temper(q[1]) & 255u) << 8 | (mt_temper(q[2]) & 255u) << 16 |
                 (mt_temper(q[3]) & 255u) << 24;
    }
}

// Philox mode: chunks c0, c0 + step, .. of the next RING_GEN blocks after slot lat (chunk c = 16 bytes: block c / 39,
// 16-byte piece c % 39), counter (block index wbuf[0] + c / 39, c % 39), key wbuf[1..2]. The caller advances wbuf[0].
__device__ __forceinline__ void ring_gen_philox(gu32* wbuf, uint32_t lat, int c0, int step, int nblk = RING_GEN)
{
    const uint32_t blk0 = wbuf[0];
    const uint64_t key = (uint64_t)wbuf[1] | (uint64_t)wbuf[2] << 32;
    gu32* ring = wbuf + MT_N;
    for (int c = c0; c < nblk * PHX_CHUNKS; c += step) {
        const int b = c / PHX_CHUNKS, j = c - b * PHX_CHUNKS;
        uint32_t w[4];
        philox4(key, (uint64_t)(blk0 + (uint32_t)b), (uint64_t)j, w);
        const uint32_t slot = (lat + 1u + (uint32_t)b) & SLOT_MASK;
        gu32* d = ring + slot * (MT_N / 4) + 4 * j;
        d[0] = w[0]; d[1] = w[1]; d[2] = w[2]; d[3] = w[3];
    }
}

// Blocks generated at seeding: env e starts with 1 + e % RING_GEN blocks (slots 0..k-1, latest in slot k-1), so its
// first refill comes after (k - 1) x 624 draws and the envs' refills -- 15 twists each, all 64 lanes of a wave busy --
// are spread evenly over the refill cycle instead of all falling in the same launches. The stream is the same
// (block b always sits in slot b % SLOTS); only when the blocks are generated differs.
__device__ __forceinline__ uint32_t seed_blocks(int64_t env) { return 1u + (uint32_t)(env % RING_GEN); }

// one lane generates blocks L+1..L+RING_GEN after L (slot lat): the rare in-step path
__device__ __attribute__((noinline)) void ring_gen_serial(uint32_t* wbuf, uint32_t lat, uint32_t phx = 0)
{
    if (phx) {
        ring_gen_philox((gu32*)wbuf, lat, 0, 1);
        wbuf[0] += (uint32_t)RING_GEN;
        return;
    }
    uint8_t* ring = (uint8_t*)(wbuf + MT_N);
    for (uint32_t b = 1; b <= (uint32_t)RING_GEN; b++) {
        mt_twist_inplace(wbuf);
        ring_bytes_serial(wbuf, ring, (lat + b) & SLOT_MASK);
    }
}

// Block words in registers, word k = 64c + lane in o[c] (c = 9 holds words 576..623 in lanes 0..47). One twist:
//   new[k] = mix(old[k], old[k+1] | new[0] (k = 623), old[k+397] (k < 227) | new[k-227])
// with the cross-lane operands fetched by ds_bpermute, but the k+1 operand (the next lane) through a DPP wavefront
// shift (wave_shl:1, a VALU modifier) instead of a ds_bpermute round trip through the LDS crossbar; n[c] only depends
// on n[c-4], n[c-3] and n[0] (computed first).
__device__ __forceinline__ void twist_regs(const uint32_t (&o)[10], uint32_t (&n)[10], int lane)
{
    const int l13 = (lane + 13) & 63, l29 = (lane + 29) & 63;
#pragma unroll
    for (int c = 0; c < 10; c++) {
        // wave_shl:1 without bound_ctrl: lane 63 has no source lane and keeps `old` -- the wrap word (the next chunk's
        // lane 0) goes in as `old`, so the shift needs no select (chunk 9 wraps at lane 47: below)
        const int old = c < 9 ? (int)__builtin_amdgcn_readlane(o[c < 9 ? c + 1 : 9], 0) : 0;
        uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp(old, (int)o[c], 0x130, 0xF, 0xF, false);
        if (c == 9) {
            const uint32_t n0 = __builtin_amdgcn_readlane(n[0], 0);
            nxt = lane == 47 ? n0 : nxt;
        }
        uint32_t far_old = 0, far_new = 0;
        if (c <= 3) {                                        // k + 397 = 64 (c + 6) + lane + 13
            const uint32_t x6 = shfl(o[c + 6], l13);
            const uint32_t x7 = c + 7 <= 9 ? shfl(o[c + 7 <= 9 ? c + 7 : 9], l13) : 0u;
            far_old = lane < 51 ? x6 : x7;
        }
        if (c >= 3) {                                        // k - 227 = 64 (c - 4) + lane + 29
            const uint32_t y3 = shfl(n[c - 3], l29);
            const uint32_t y4 = c >= 4 ? shfl(n[c >= 4 ? c - 4 : 0], l29) : 0u;
            far_new = lane < 35 ? y4 : y3;
        }
        const int k = 64 * c + lane;
        const uint32_t far = k < MT_N - MT_M ? far_old : far_new;
        n[c] = mt_mix(o[c], nxt, far);
    }
}

// stream traffic: default-policy loads and stores (nontemporal ones measured slower for Leduc)
__device__ __forceinline__ uint32_t ring_ld(const gu32* p) { return *p; }
__device__ __forceinline__ void ring_st(gu32* p, uint32_t v) { *p = v; }

// Wave-cooperative refill of one env: blocks L+1..L+3 from wbuf (block L, slot lat). All 64 lanes must call.
__device__ __forceinline__ void ring_gen_wave(gu32* wbuf, uint32_t lat, int lane, uint32_t phx = 0)
{
    if (phx) {   // Philox mode: 117 chunks over the 64 lanes, then the block counter (read by every lane first)
        const uint32_t blk0 = wbuf[0];
        ring_gen_philox(wbuf, lat, lane, WAVE);
        if (lane == 0) wbuf[0] = blk0 + (uint32_t)RING_GEN;
        return;
    }
    uint32_t o[10], n[10];
#pragma unroll
    for (int c = 0; c < 10; c++) o[c] = (c < 9 || lane < 48) ? ring_ld(wbuf + 64 * c + lane) : 0u;
    gu32* ring = wbuf + MT_N;   // 624 dwords of bytes
    // the blocks in a rolled loop: one block's code (unrolled 15 times, the refill alone would be ~40 KB of the
    // rollout kernels' instruction footprint)
#pragma unroll 1
    for (int b = 1; b <= RING_GEN; b++) {
        twist_regs(o, n, lane);
        const uint32_t slot = (lat + (uint32_t)b) & SLOT_MASK;
#pragma unroll
        for (int c = 0; c < 10; c++) {
            // every lane stores its word's byte (one global_store_byte per 64 words): faster than packing four
            // lanes' bytes with DPP moves into a dword store by every fourth lane
            if (c < 9 || lane < 48) ((gu8*)(ring + slot * (MT_N / 4)))[64 * c + lane] = (uint8_t)mt_temper_lo8(n[c]);
            o[c] = n[c];
        }
    }
#pragma unroll
    for (int c = 0; c < 10; c++)
        if (c < 9 || lane < 48) ring_st(wbuf + 64 * c + lane, o[c]);
}

// One lane's view of its env's byte ring. MODE as MtLaneT: STAGE_NONE reads the ring in HBM per draw; STAGE_LDS
// reads the lane's staged LDS row (ring_restage_wave), HBM only past its end.
template <int MODE = STAGE_NONE>
struct RingLane {
    static constexpr int kMode = MODE;
    uint32_t* base;   // wbuf of the env (mt + env * RING_ENV_WORDS); the ring bytes follow it
    uint32_t pos;     // ring position
    uint32_t lat;     // slot of the latest generated block
    uint32_t sp, sn;  // ring position of staged byte 0; staged bytes
    const uint8_t* stg;
    uint32_t phx;     // CTL_PHILOX when the env's stream is the Philox byte stream

    __device__ __forceinline__ void init(uint32_t* p_base, uint32_t ctlw)
    {
        base = p_base;
        pos = ctlw & CTL_POS_MASK;
        lat = (ctlw >> CTL_LAT_SHIFT) & SLOT_MASK;
        phx = ctlw & CTL_PHILOX;
        sp = 0;
        sn = 0;
        stg = nullptr;
    }
    __device__ __forceinline__ uint32_t ctl_word() const { return pos | lat << CTL_LAT_SHIFT | phx; }
    __device__ __forceinline__ const uint8_t* ring() const { return (const uint8_t*)(base + MT_N); }
    __device__ __forceinline__ uint32_t limit() const { return ((lat + 1u) & SLOT_MASK) * (uint32_t)MT_N; }
    // draws left before the end of the generated data (1 .. RING)
    __device__ __forceinline__ uint32_t ahead() const
    {
        const uint32_t d = limit() + RING - pos;
        return d > RING ? d - RING : d;
    }
    __device__ __forceinline__ bool needs_refill() const { return ahead() <= (uint32_t)MT_N; }   // inside block L

    __device__ __forceinline__ void gen_serial()
    {
        ring_gen_serial(base, lat, phx);
        lat = (lat + (uint32_t)RING_GEN) & SLOT_MASK;
    }

    __device__ __forceinline__ void advance()
    {
        pos = pos + 1u == RING ? 0u : pos + 1u;
        if (pos == limit()) gen_serial();
    }

    __device__ __forceinline__ uint32_t staged_offset() const { return pos >= sp ? pos - sp : pos + RING - sp; }

    // the ring byte at pos, read as its dword: a byte load here would let the compiler merge it with the staged LDS
    // byte load into one load through a select of pointers of two address spaces (clang crashes on that)
    __device__ __forceinline__ uint32_t ring_byte() const
    {
        return (((const uint32_t*)ring())[pos >> 2] >> (8 * (pos & 3u))) & 255u;
    }

    // low 8 bits of the next tempered word
    __device__ __forceinline__ uint32_t next8()
    {
        uint32_t v;
        if constexpr (MODE == STAGE_NONE) {
            v = ring_byte();
        } else {
            const uint32_t k = staged_offset();
            if (k < sn) v = stg[k];
            else v = ring_byte();
        }
        advance();
        return v;
    }

    // numpy random_interval(max) for max <= 255: smallest all-ones mask >= max, reject while (byte & mask) > max
    __device__ __forceinline__ uint32_t interval(uint32_t max)
    {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        if (__builtin_constant_p(max) && max == mask) return next8() & mask;   // e.g. randint(0, 2): never rejects
        if constexpr (MODE == STAGE_LDS) {
            // the next four staged bytes at once: per byte t = b & mask, (t | 0x80) - (max + 1) has bit 7 set exactly
            // when t > max (no borrow between bytes for max < 128); the first accepted byte is the draw. The loop
            // below only runs past four rejections in a row (~0.1 % of a 52-card deal) or at the staged row's end.
            // The second dword may reach into the row's pad (PAD >= 4), its bytes past sn unused.
            const uint32_t k0 = staged_offset();
            if (max < 128u && k0 + 4u <= sn) {
                const uint32_t* row = (const uint32_t*)(stg + (k0 & ~3u));
                const uint32_t x = __builtin_amdgcn_alignbyte(row[1], row[0], k0 & 3u) & (mask * 0x01010101u);
                const uint32_t acc = ~((x | 0x80808080u) - (max + 1u) * 0x01010101u) & 0x80808080u;
                if (acc) {
                    const uint32_t b = (uint32_t)__builtin_ctz(acc) >> 3;
                    advance_by(b + 1u);
                    return (x >> (8u * b)) & 255u;
                }
                advance_by(4u);
            }
        }
        return interval_loop(max, mask);
    }
    // the same draw one byte at a time (cold paths: keeps the kernels' code small)
    __device__ __forceinline__ uint32_t interval_loop(uint32_t max)
    {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        return interval_loop(max, mask);
    }
    __device__ __forceinline__ uint32_t interval_loop(uint32_t max, uint32_t mask)
    {
        uint32_t v;
        do {
            v = next8() & mask;
        } while (v > max);
        return v;
    }

    // pos += n (n < 624)
    __device__ __forceinline__ void advance_by(uint32_t n)
    {
        const uint32_t a = ahead();
        uint32_t np = pos + n;
        if (np >= RING) np -= RING;
        if (n >= a) gen_serial();
        pos = np;
    }

    // random_interval(i) for i = hi .. 1 with every result discarded: only how many bytes the draws consume matters.
    // The staged bytes are read as whole dwords at any byte offset (alignbyte of two aligned dwords) and scanned
    // branch-free -- per byte: the mask width of i, a bit-field extract, one compare -- for the draws i = hi .. 2; the
    // last draw (mask 1) always takes exactly one byte. A lane that runs out of staged bytes finishes through interval_loop().
    __device__ __forceinline__ void skip_intervals(uint32_t hi)
    {
        uint32_t i = hi;
        if constexpr (MODE == STAGE_LDS) {
            const uint32_t k0 = staged_offset();
            if (i >= 2 && k0 < sn) {
                const uint32_t* row = (const uint32_t*)(stg + (k0 & ~3u));
                const uint32_t sh = k0 & 3u, nd = (sn - k0) >> 2;   // whole dwords staged from k0
                uint32_t cnt = 0, lo = row[0], d = 0;
                // while i >= 6 a dword cannot take i below 2: no per-byte liveness
                for (; d < nd && i >= 6; d++) {
                    const uint32_t hw = row[d + 1];
                    const uint32_t x = __builtin_amdgcn_alignbyte(hw, lo, sh);
                    lo = hw;
#pragma unroll
                    for (uint32_t t = 0; t < 4; t++) {
                        const uint32_t u = __builtin_amdgcn_ubfe(x, 8 * t, 32u - __builtin_clz(i));
                        i -= u <= i ? 1u : 0u;
                    }
                    cnt += 4;
                }
                for (; d < nd && i >= 2; d++) {
                    const uint32_t hw = row[d + 1];
                    const uint32_t x = __builtin_amdgcn_alignbyte(hw, lo, sh);
                    lo = hw;
#pragma unroll
                    for (uint32_t t = 0; t < 4; t++) {
                        const bool live = i >= 2;
                        const uint32_t u = __builtin_amdgcn_ubfe(x, 8 * t, 32u - __builtin_clz(i));
                        cnt += live ? 1u : 0u;
                        i -= (live && u <= i) ? 1u : 0u;
                    }
                }
                advance_by(cnt);
            }
        }
        for (; i >= 1; i--) (void)interval_loop(i);
    }

    // random_interval(i) for i = hi, hi - 1, .., 1 in stream order, put(k, value of draw k): one branch-free pass over
    // the staged bytes (per byte: extract under the mask of the current i, accept, count), interval_loop() past their end
    template <class F>
    __device__ __forceinline__ void draw_intervals(uint32_t hi, F&& put)
    {
        uint32_t i = hi;
        if constexpr (MODE == STAGE_LDS) {
            const uint32_t k0 = staged_offset();
            if (i >= 1 && k0 < sn) {
                const uint32_t* row = (const uint32_t*)(stg + (k0 & ~3u));
                const uint32_t sh = k0 & 3u, nd = (sn - k0) >> 2;
                uint32_t cnt = 0, lo = row[0], d = 0;
                // while i >= 4 a dword cannot take i below 1: every byte is live (no per-byte liveness or count)
                for (; d < nd && i >= 4; d++) {
                    const uint32_t hw = row[d + 1];
                    const uint32_t x = __builtin_amdgcn_alignbyte(hw, lo, sh);
                    lo = hw;
#pragma unroll
                    for (uint32_t t = 0; t < 4; t++) {
                        const uint32_t u = __builtin_amdgcn_ubfe(x, 8 * t, 32u - __builtin_clz(i));
                        const bool acc = u <= i;
                        if (acc) put(hi - i, u);
                        i -= acc ? 1u : 0u;
                    }
                    cnt += 4;
                }
                for (; d < nd && i >= 1; d++) {
                    const uint32_t hw = row[d + 1];
                    const uint32_t x = __builtin_amdgcn_alignbyte(hw, lo, sh);
                    lo = hw;
#pragma unroll
                    for (uint32_t t = 0; t < 4; t++) {
                        const bool live = i >= 1;
                        const uint32_t u = __builtin_amdgcn_ubfe(x, 8 * t, 32u - __builtin_clz(i | 1u));
                        const bool acc = live && u <= i;
                        if (acc) put(hi - i, u);
                        cnt += live ? 1u : 0u;
                        i -= acc ? 1u : 0u;
                    }
                }
                advance_by(cnt);
            }
        }
        for (; i >= 1; i--) put(hi - i, interval_loop(i));
    }
};

// End-of-step convergence point: the wave refills every lane that is inside its latest block. All 64 lanes call.
template <class M>
__device__ __forceinline__ void ring_refill_wave(M& m, int lane)
{
    uint64_t need = __ballot(m.needs_refill());
    while (need) {
        const int j = __builtin_ctzll(need);
        need &= need - 1;
        ring_gen_wave(lane_ptr(m.base, j), __builtin_amdgcn_readlane(m.lat, j), lane,
                      __builtin_amdgcn_readlane(m.phx, j));
        if (lane == j) m.lat = (m.lat + (uint32_t)RING_GEN) & SLOT_MASK;
    }
    // the ring bytes are read later by their owner lane of this same wave: order the stores before those loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// STAGE_LDS restage, after ring_refill_wave: every lane with fewer than R staged bytes left gets the W ring bytes from
// its position rounded down to a dword (the refill left >= 624 generated bytes ahead of every lane). W / 4 lanes copy
// one lane's row with dword loads (the ring is a multiple of 4 bytes, so no dword straddles its end); 64 / (W / 4)
// rows per load instruction, B instructions in flight per pass. The needy lanes are ranked with mbcnt and a ds_permute
// pushes each one's id to the lane of its rank, so a pass picks its rows with one bpermute (no scalar bit-scan loops).
// All 64 lanes must call.
// RF > R batches the restages: nothing happens until some lane has fewer than R bytes left, then every lane with
// fewer than RF is restaged (fewer restage events per launch, more rows per event).
template <int W, int PAD, int R, int B, int RF = R>
__device__ __forceinline__ void ring_restage_wave(RingLane<STAGE_LDS>& m, uint8_t* area, int lane, bool valid)
{
    constexpr int STRIDE = Stage<W, PAD>::STRIDE, DW = W / 4, RPI = WAVE / DW, PER = B * RPI;
    static_assert(DW <= WAVE && WAVE % DW == 0, "a staged row is copied by W / 4 lanes");
    static_assert(RF >= R && RF <= W, "restage thresholds");
    m.stg = area + lane * STRIDE;
    const uint32_t k = m.staged_offset();
    const uint32_t left = k >= m.sn ? 0u : m.sn - k;
    uint64_t todo = __ballot(valid && left < (uint32_t)R);
    if (RF > R && todo) todo = __ballot(valid && left < (uint32_t)RF);
    const bool needy = (todo >> lane) & 1u;
    if (todo) {
        const int count = __popcll(todo);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(todo >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)todo, 0u));
        // a full permutation: needy lanes to their rank, the others after them
        const int dst = needy ? rank : count + (lane - rank);
        const int who = __builtin_amdgcn_ds_permute(dst << 2, lane);   // lane q < count: the q-th needy lane
        const int row = lane / DW, col = lane - row * DW;
        const uint32_t rbase_lo = (uint32_t)(uintptr_t)m.ring(), rbase_hi = (uint32_t)((uintptr_t)m.ring() >> 32);
        const uint32_t p4 = m.pos & ~3u;
        for (int base = 0; base < count; base += PER) {
            uint32_t v[B];
            int src[B];
#pragma unroll
            for (int b = 0; b < B; b++) {
                const int q = base + b * RPI + row;
                const int s = (int)shfl((uint32_t)who, q < count ? q : base);   // past the end: repeat (harmless)
                src[b] = s;
                const uint64_t rb = (uint64_t)shfl(rbase_lo, s) | (uint64_t)shfl(rbase_hi, s) << 32;
                uint32_t off = shfl(p4, s) + 4u * (uint32_t)col;
                if (off >= RING) off -= RING;
                const gu32* rp = (const gu32*)(uintptr_t)rb;
                v[b] = ring_ld(rp + (off >> 2));
            }
#pragma unroll
            for (int b = 0; b < B; b++) *(uint32_t*)(area + src[b] * STRIDE + 4 * col) = v[b];
        }
        if (needy) {
            m.sp = p4;
            m.sn = W;
        }
    }
    wave_sync_lds();
}

}  // namespace cs
