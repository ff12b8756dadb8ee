// cs_leduc.h -- Leduc Hold'em as a lane-per-env lockstep state machine (2 players).
//
// Behaviour (reference file:line):
//   rlcard/games/leducholdem/dealer.py:4-12, limitholdem/dealer.py:11-21  6-card deck [SJ,HJ,SQ,HQ,SK,HK], shuffle, pop()
//   rlcard/games/leducholdem/game.py:46-95     init_game: hands deck[5], deck[4]; SB = randint(0,2); SB acts first
//   rlcard/games/leducholdem/game.py:97-133    step: proceed_round; end of round 0 -> public card deck[3], raise 2 -> 4
//   rlcard/games/limitholdem/round.py:53-127   proceed_round / get_legal_actions (allowed_raise_num = 2) / is_over
//   rlcard/games/leducholdem/game.py:148-178   is_over, payoffs = judger chips / big_blind
//   rlcard/games/leducholdem/judger.py:11-64   fold winner / pair with the public card / high card / split
//   rlcard/envs/leducholdem.py:41-96           obs[36] one-hot (hand rank, public rank+3, my chips+6,
//                                              others' chips+21) and the illegal-id fallback (check, else fold)
// Packed state (2 u32 words per env, word-major [2][N] so a wave's loads/stores are coalesced):
//   w0: h0:3 h1:3 pub:3 in0:5 in1:5 r0:4 r1:4 have_raised:2 not_raise_num:2 over:1
//   w1: round_counter:2 pointer:1 folded0:1 folded1:1
#pragma once
#include "cs_device.h"

#include "cs_prof.h"

namespace cs {

struct Leduc {
    // (no deal queue: drawing deals ahead, as Limit / No-limit do, measured slower here -- profiles/EXPERIMENTS.md)
    static constexpr int OBS = 36, A = 4, P = 2, LB = 1, WORDS = 2, ACTION_BYTES = 1;
    static constexpr int NB = 2;  // obs bitmap words
    static constexpr bool RING = true;          // MT stream as the byte ring (cs_ring.h)
    static constexpr bool RAW_OBS = false;
    static constexpr int SCRATCH_WORDS = 0;
    // MT staging (see MtLaneT)
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 64, STAGE_PAD = 4, STAGE_R = 12;
    static constexpr int STAGE_RF = 24;   // batch restage threshold (ring_restage_wave): 24 > 40 > 56
    static constexpr int RESTAGE_B = 4;   // lanes restaged per pass (loads in flight): 4 > 8 > 1
    static constexpr int MIN_WAVES = 6;   // rollout waves per SIMD the register budget must allow
    static constexpr int EPW = 64;        // rollout envs per wave (lane_ctx)
    static constexpr int REFILL_K = 1;    // refills are rare here, and K = 2 costs 12 VGPRs = 1 wave/SIMD
    __device__ __forceinline__ void bind(uint32_t*, const GameParams&) {}
    enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };

    int h0, h1, pub, in0, in1, r0, r1, hr, nrn, over, rc, ptr, f0, f1;

    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
        const uint32_t w0 = st[env], w1 = st[n + env];
        h0 = w0 & 7; h1 = (w0 >> 3) & 7; pub = (w0 >> 6) & 7; in0 = (w0 >> 9) & 31; in1 = (w0 >> 14) & 31;
        r0 = (w0 >> 19) & 15; r1 = (w0 >> 23) & 15; hr = (w0 >> 27) & 3; nrn = (w0 >> 29) & 3; over = w0 >> 31;
        rc = w1 & 3; ptr = (w1 >> 2) & 1; f0 = (w1 >> 3) & 1; f1 = (w1 >> 4) & 1;
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
        st[env] = (uint32_t)h0 | (uint32_t)h1 << 3 | (uint32_t)pub << 6 | (uint32_t)in0 << 9 | (uint32_t)in1 << 14 |
                  (uint32_t)r0 << 19 | (uint32_t)r1 << 23 | (uint32_t)hr << 27 | (uint32_t)nrn << 29 |
                  (uint32_t)over << 31;
        st[n + env] = (uint32_t)rc | (uint32_t)ptr << 2 | (uint32_t)f0 << 3 | (uint32_t)f1 << 4;
    }
    __device__ __forceinline__ void blank() { h0 = h1 = pub = in0 = in1 = r0 = r1 = hr = nrn = rc = ptr = f0 = f1 = 0; over = 1; }

    __device__ __forceinline__ int current() const { return ptr; }
    __device__ __forceinline__ bool is_over() const { return over != 0; }

    __device__ __forceinline__ uint32_t legal() const
    {
        const int mx = r0 > r1 ? r0 : r1, rp = ptr ? r1 : r0;
        uint32_t m = 0xF;
        if (hr >= 2) m &= ~(1u << RAISE);
        if (rp < mx) m &= ~(1u << CHECK);
        if (rp == mx) m &= ~(1u << CALL);
        return m;
    }

    __device__ __forceinline__ void observe(int player, uint32_t (&bits)[NB]) const
    {
        const int my = player ? in1 : in0, hand = player ? h1 : h0;
        uint64_t b = (1ull << (hand >> 1)) | (1ull << (my + 6)) | (1ull << (in0 + in1 - my + 21));
        if (rc >= 1) b |= 1ull << ((pub >> 1) + 3);
        bits[0] = (uint32_t)b;
        bits[1] = (uint32_t)(b >> 32);
    }

    // the same row as the byte positions of its ones (row_write_sparse): hand rank, public rank + 3 (absent: the hand
    // position again), my chips + 6, the others' chips + 21
    static constexpr int SPARSE_K = 4;
    __device__ __forceinline__ uint32_t observe_pos(int player, uint32_t (&pos)[4]) const
    {
        const int my = player ? in1 : in0, hand = (player ? h1 : h0) >> 1;
        pos[0] = (uint32_t)hand;
        pos[1] = (uint32_t)(rc >= 1 ? (pub >> 1) + 3 : hand);
        pos[2] = (uint32_t)(my + 6);
        pos[3] = (uint32_t)(in0 + in1 - my + 21);
        return 0;
    }

    // dealer.py shuffle (intervals 5..1, swap) then randint(0, 2) for the small blind: six random_interval draws as
    // one state machine over the draw bytes (stage q: 0..4 = the swaps, 5 = the blind), so a wave steps every lane
    // through the staged bytes together instead of looping per interval until its slowest lane accepts
    // The deal depends only on the first three Fisher-Yates draws: j1 fixes position 5 (p0's hand), j2 position 4
    // (p1's hand), j3 position 3 (the public card); the draws for positions 2 and 1 and the blind's randint only
    // consume bytes or pick the blind. random_interval on the low byte, per stage: i=5 mask 7 rejects 6,7; i=4 mask 7
    // rejects 5..7; i=3 mask 3 never rejects; i=2 mask 3 rejects 3; i=1 and the blind (mask 1) never reject. So with
    // the next 16 staged bytes as 4 dwords, per-byte accept flags for the three rejecting stages are a few SWAR ops
    // each, and the stage positions are first-set searches: p0 (i=5), p1 (i=4, after p0), p2 = p1 + 1, p3 (i=2, after
    // p2), p4 = p3 + 1, p5 = p4 + 1 (the blind). false: the staged window does not hold the whole reset (the caller
    // runs the byte state machine instead).
    // A deal as one word (the deal queue's entry, cs_dq.h): hand 0 | hand 1 << 3 | public << 6 | small blind << 9
    template <class Rng>
    __device__ __forceinline__ static bool deal_swar(Rng& rng, uint32_t& code)
    {
        const uint32_t k0 = rng.staged_offset();
        const uint32_t avail = k0 < rng.sn ? rng.sn - k0 : 0u, nv = avail < 16u ? avail : 16u;
        if (nv < 6u) return false;   // also the first reset of a launch, before any row is staged (stg unset)
        const uint32_t* row = (const uint32_t*)(rng.stg + (k0 & ~3u));
        uint32_t w[5];
#pragma unroll
        for (int i = 0; i < 5; i++) w[i] = row[i];
        uint32_t m0 = 0, m1 = 0, m3 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t x = __builtin_amdgcn_alignbyte(w[i + 1], w[i], k0 & 3u);   // staged bytes k0 + 4i ..
            const uint32_t b1 = x >> 1, b2 = x >> 2;
            const uint32_t a0 = ~(b1 & b2) & 0x01010101u;          // (b & 7) <= 5
            const uint32_t a1 = ~(b2 & (b1 | x)) & 0x01010101u;    // (b & 7) <= 4
            const uint32_t a3 = ~(x & b1) & 0x01010101u;           // (b & 3) <= 2
            // byte flags (bits 0, 8, 16, 24) -> 4-bit mask: the product's top nibble (no overlapping partial sums)
            m0 |= ((a0 * 0x10204080u) >> 28) << (4 * i);
            m1 |= ((a1 * 0x10204080u) >> 28) << (4 * i);
            m3 |= ((a3 * 0x10204080u) >> 28) << (4 * i);
        }
        const uint32_t valid = (1u << nv) - 1u;
        m0 &= valid;
        if (!m0) return false;
        const uint32_t p0 = __builtin_ctz(m0);
        const uint32_t r1 = m1 & valid & (0xFFFFFFFEu << p0);
        if (!r1) return false;
        const uint32_t p1 = __builtin_ctz(r1), p2 = p1 + 1;
        const uint32_t r3 = m3 & valid & (0xFFFFFFFEu << p2);
        if (!r3) return false;
        const uint32_t p5 = __builtin_ctz(r3) + 2;
        if (p5 >= nv) return false;
        const uint8_t* b = rng.stg + k0;
        const uint32_t j1 = b[p0] & 7u, j2 = b[p1] & 7u, j3 = b[p2] & 3u, s = b[p5] & 1u;
        rng.advance_by(p5 + 1);
        // deck positions after the swaps (deck[i] = i before): 5 <- j1; 4 <- deck'[j2]; 3 <- deck''[j3]
        const uint32_t hh0 = j1, hh1 = j2 == j1 ? 5u : j2;
        const uint32_t pb = j3 == j2 ? (j1 == 4u ? 5u : 4u) : (j3 == j1 ? 5u : j3);
        code = hh0 | hh1 << 3 | pb << 6 | s << 9;
        return true;
    }

    template <class Rng>
    __device__ __forceinline__ static uint32_t draw_deal(Rng& rng)
    {
#if CS_PROF_NO_RESET   // profiling builds only (cs_prof.h)
        rng.advance_by(7u);
        return 0u | 2u << 3 | 4u << 6 | (rng.pos & 1u) << 9;
#endif
        if constexpr (Rng::kMode == STAGE_LDS) {
            uint32_t code;
            if (deal_swar(rng, code)) return code;
        }
        uint32_t deck = 0x543210u;  // nibble i = card at deck position i
        uint32_t q = 0, s = 0;
        auto take = [&](uint32_t b) {
            const uint32_t mx = q < 5 ? 5 - q : 1;
            const uint32_t u = b & (mx >= 4 ? 7u : (mx >= 2 ? 3u : 1u));
            if (u <= mx) {
                if (q < 5) {
                    const uint32_t ci = (deck >> (4 * mx)) & 15u, cj = (deck >> (4 * u)) & 15u, x = ci ^ cj;
                    deck ^= (x << (4 * mx)) | (x << (4 * u));
                } else {
                    s = u;
                }
                q++;
            }
        };
        if constexpr (Rng::kMode == STAGE_LDS) {
            const uint32_t k0 = rng.staged_offset();
            uint32_t k = k0;
            while (q < 6 && k < rng.sn) {
                const uint32_t sh = k & 3u;
                const uint32_t w = *(const uint32_t*)(rng.stg + (k - sh)) >> (8 * sh);
#pragma unroll
                for (uint32_t t = 0; t < 4; t++)
                    if (t < 4 - sh && q < 6 && k < rng.sn) {
                        take((w >> (8 * t)) & 255u);
                        k++;
                    }
            }
            rng.advance_by(k - k0);
        }
        while (q < 6) take(rng.next8());
        return ((deck >> 20) & 15u) | ((deck >> 16) & 15u) << 3 | ((deck >> 12) & 15u) << 6 | s << 9;
    }

    __device__ __forceinline__ void deal_blinds(int s)
    {
        in0 = s == 0 ? 1 : 2;
        in1 = s == 0 ? 2 : 1;
        ptr = s;
        r0 = in0; r1 = in1;
        hr = 0; nrn = 0; rc = 0; f0 = 0; f1 = 0; over = 0;
    }

    // Game.init_game from a deal word (draw_deal)
    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        const uint32_t e0 = draw_deal(rng);
        h0 = (int)(e0 & 7u);
        h1 = (int)((e0 >> 3) & 7u);
        pub = (int)((e0 >> 6) & 7u);
        deal_blinds((int)((e0 >> 9) & 1u));
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng&)
    {
        const uint32_t lg = legal();
        if (a < 0 || a > 3 || !((lg >> a) & 1u)) a = ((lg >> CHECK) & 1u) ? CHECK : FOLD;
        const int mx = r0 > r1 ? r0 : r1, rp = ptr ? r1 : r0, ra = rc == 0 ? 2 : 4;
        int add = 0, nr = rp;
        if (a == CALL) { add = mx - rp; nr = mx; nrn += 1; }
        else if (a == RAISE) { add = mx - rp + ra; nr = mx + ra; hr += 1; nrn = 1; }
        else if (a == FOLD) { if (ptr) f1 = 1; else f0 = 1; }
        else { nrn += 1; }
        if (ptr) { in1 += add; r1 = nr; } else { in0 += add; r0 = nr; }
        ptr ^= 1;
        if (ptr ? f1 : f0) ptr ^= 1;  // skip the folded player
        if (nrn >= 2) {               // round over: deal the public card after round 0, start a new round
            rc += 1;
            hr = 0; nrn = 0; r0 = 0; r1 = 0;
        }
        over = (f0 + f1 == 1) || rc >= 2;
    }

    __device__ __forceinline__ void payoffs(float (&r)[P]) const
    {
        int w0, w1;
        if (f0 || f1) { w0 = !f0; w1 = !f1; }
        else {
            const int pr = pub >> 1, k0 = h0 >> 1, k1 = h1 >> 1;
            if (k0 == pr) { w0 = 1; w1 = 0; }
            else if (k1 == pr) { w0 = 0; w1 = 1; }
            else { w0 = k0 >= k1; w1 = k1 >= k0; }
        }
        const float tot = (float)(in0 + in1), each = (w0 & w1) ? tot * 0.5f : tot;   // total / #winners, exact
        r[0] = (w0 ? each - (float)in0 : -(float)in0) * 0.5f;
        r[1] = (w1 ? each - (float)in1 : -(float)in1) * 0.5f;
    }
};

}  // namespace cs
