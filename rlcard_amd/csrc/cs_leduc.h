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

#ifndef CS_LEDUC_RESTAGE_B
#define CS_LEDUC_RESTAGE_B 4
#endif
#ifndef CS_LEDUC_REFILL_K
#define CS_LEDUC_REFILL_K 1
#endif
#ifndef CS_LEDUC_RESET_SCAN
#define CS_LEDUC_RESET_SCAN 1
#endif
#ifndef CS_LEDUC_MIN_WAVES
#define CS_LEDUC_MIN_WAVES 6
#endif
#ifndef CS_LEDUC_STAGE_R

#define CS_LEDUC_STAGE_R 12
#endif

namespace cs {

struct Leduc {
    static constexpr int OBS = 36, A = 4, P = 2, LB = 1, WORDS = 2, ACTION_BYTES = 1;
    static constexpr int NB = 2;  // obs bitmap words
    static constexpr bool RAW_OBS = false;
    static constexpr int SCRATCH_WORDS = 0;
    // MT staging (see MtLaneT)
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 64, STAGE_PAD = 4, STAGE_R = CS_LEDUC_STAGE_R;
    static constexpr int RESTAGE_B = CS_LEDUC_RESTAGE_B;  // lanes restaged per pass (loads in flight): 4 > 8 > 1
    static constexpr int MIN_WAVES = CS_LEDUC_MIN_WAVES;  // rollout waves per SIMD the register budget must allow
    static constexpr int EPW = 64;        // rollout envs per wave (lane_ctx)
    static constexpr int REFILL_K = CS_LEDUC_REFILL_K;    // 1: refills are rare here, and K = 2 costs 12 VGPRs = 1 wave/SIMD
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
        bits[0] = bits[1] = 0;
        const int my = player ? in1 : in0, hand = player ? h1 : h0;
        set_bit(bits, hand >> 1);
        if (rc >= 1) set_bit(bits, (pub >> 1) + 3);
        set_bit(bits, my + 6);
        set_bit(bits, in0 + in1 - my + 21);
    }

    // dealer.py shuffle (intervals 5..1, swap) then randint(0, 2) for the small blind: six random_interval draws as
    // one state machine over the draw bytes (stage q: 0..4 = the swaps, 5 = the blind), so a wave steps every lane
    // through the staged bytes together instead of looping per interval until its slowest lane accepts
    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
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
        if constexpr (Rng::kMode == STAGE_LDS && CS_LEDUC_RESET_SCAN) {
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
        h0 = (deck >> 20) & 15; h1 = (deck >> 16) & 15; pub = (deck >> 12) & 15;
        in0 = s == 0 ? 1 : 2;
        in1 = s == 0 ? 2 : 1;
        ptr = s;
        r0 = in0; r1 = in1;
        hr = 0; nrn = 0; rc = 0; f0 = 0; f1 = 0; over = 0;
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
        const float each = (float)(in0 + in1) / (float)(w0 + w1);
        r[0] = (w0 ? each - (float)in0 : -(float)in0) * 0.5f;
        r[1] = (w1 ? each - (float)in1 : -(float)in1) * 0.5f;
    }
};

}  // namespace cs
