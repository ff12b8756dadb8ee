// cs_holdem_n.h -- Leduc / Limit / No-limit hold'em with 3..22 players (Leduc 3..5) ('game_num_players', envs/env.py:33-39), as
// lane-per-env lockstep state machines over the shared skeleton (cs_skeleton.h). The heads-up games keep their
// specialised kernels (cs_leduc.h, cs_limit.h, cs_nolimit.h); these follow the reference's per-player loops directly.
//
// Behaviour (reference file:line), on top of the heads-up headers:
//   rlcard/games/leducholdem/game.py:40-95      N hands deck.pop() p0..pN-1 (positions 5, 4, ..), public = the next
//                                               pop; SB = randint(0, N), BB = SB + 1, SB acts first
//   rlcard/games/limitholdem/game.py:46-103     2N holes round-robin (hole i -> player i % N from deck[51 - i]), board
//                                               deck[51 - 2N ..]; SB = randint(0, N); first actor BB + 1
//   rlcard/games/nolimitholdem/game.py:58-185   dealer = randint(0, N) once (kept), SB = dealer + 1, BB = dealer + 2,
//                                               first actor BB + 1; bypass rule with players_in_bypass.index(0)
//   rlcard/games/limitholdem/round.py:53-127    (and nolimitholdem/round.py:62-173) with N players: a round is over
//                                               once not_raise_num (+ not_playing_num) reaches N -- folded players
//                                               are skipped but still counted in N (rounds run longer after a fold)
//   rlcard/games/leducholdem/judger.py:11-64    the first player, folded or not, whose rank matches the public card
//                                               wins; else the highest rank over every player; total / #winners
//                                               (fp64, then / 2)
//   rlcard/games/limitholdem/judger.py:11-108   side pots: repeat { best hand among those still in wins the pots it is
//                                               in }, odd split remainders -> np_random.choice(winners in the pot)
//                                               (the env's own stream: PAYOFF_DRAWS), see holdem_judge
//   rlcard/envs/leducholdem.py:61-64            obs[21 + others' chips]: past slot 35 (3+ players) the reference raises
//                                               IndexError; this ABI sets no bit there
// No deal queue: a judge may draw from the stream at a game's end, so deals cannot be drawn ahead.
// Packed state, word-major [WORDS][N]: one word per player, then shared words (layouts per struct below).
#pragma once
#include "cs_device.h"
#include "cs_limit.h"

namespace cs {

// per-player words in registers; a runtime index goes through select chains, so the array never spills to scratch
template <int P>
struct PlayerWords {
    uint32_t w[P];
    __device__ __forceinline__ uint32_t get(int i) const
    {
        uint32_t r = w[0];
#pragma unroll
        for (int k = 1; k < P; k++) r = i == k ? w[k] : r;
        return r;
    }
    __device__ __forceinline__ void set(int i, uint32_t v)
    {
#pragma unroll
        for (int k = 0; k < P; k++) w[k] = i == k ? v : w[k];
    }
};

__device__ __forceinline__ uint32_t bf(uint32_t w, int at, int bits) { return (w >> at) & ((1u << bits) - 1u); }
__device__ __forceinline__ uint32_t bf_set(uint32_t w, int at, int bits, uint32_t v)
{
    const uint32_t m = ((1u << bits) - 1u) << at;
    return (w & ~m) | ((v << at) & m);
}

// limitholdem/judger.py:11-108 for P players. value[i] = holdem_rank7 of player i's seven cards (0 = hand None: folded);
// in_chips = chips bet; pay = chips won. Every array index is a compile-time constant after unrolling.
template <int P, class Rng>
__device__ __forceinline__ void holdem_judge(const uint32_t (&value)[P], const int (&in0)[P], Rng& rng, int (&pay)[P])
{
    int in_chips[P], remaining = 0;
    bool in_hand[P];
#pragma unroll
    for (int i = 0; i < P; i++) {
        in_hand[i] = value[i] != 0u;
        in_chips[i] = in0[i];
        remaining += in0[i];
        pay[i] = 0;
    }
    for (int pass = 0; pass < P && remaining > 0; pass++) {   // each pass retires >= 1 hand
        uint32_t best = 0;
#pragma unroll
        for (int i = 0; i < P; i++) best = in_hand[i] && value[i] > best ? value[i] : best;
        if (best == 0u) break;   // every hand None: the reference raises in compare_hands; chips stay where returned
        bool win[P];
        int each[P], left[P];
#pragma unroll
        for (int i = 0; i < P; i++) {
            win[i] = in_hand[i] && value[i] == best;
            each[i] = 0;
            left[i] = in_chips[i];
        }
        // split_pots_among_players: pot after pot (judger.py:45-108) until every bet is allocated
        for (int pot = 0; pot < P; pot++) {
            int nwin = 0, nply = 0, amount = 0x7FFFFFFF;
#pragma unroll
            for (int i = 0; i < P; i++) {
                nwin += (win[i] && left[i] > 0) ? 1 : 0;
                nply += left[i] > 0 ? 1 : 0;
                amount = left[i] > 0 && left[i] < amount ? left[i] : amount;
            }
            if (nply == 0) break;
            if (nwin == 0 || nwin == nply) {   // nobody / only winners in this pot: everyone takes their chips back
#pragma unroll
                for (int i = 0; i < P; i++) { each[i] += left[i]; left[i] = 0; }
                break;
            }
            const int total = amount * nply, one = total / nwin, rem = total - one * nwin;
            int k = rem > 0 ? (int)rng.interval((uint32_t)(nwin - 1)) : -1;   // np_random.choice(winners in the pot)
#pragma unroll
            for (int i = 0; i < P; i++) {
                if (left[i] > 0) {
                    if (win[i]) {
                        each[i] += one + (k == 0 ? rem : 0);
                        k--;
                    }
                    left[i] -= amount;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < P; i++) {
            if (win[i]) {
                remaining -= each[i];
                pay[i] += each[i] - in_chips[i];
                in_hand[i] = false;
                in_chips[i] = 0;
            } else if (in_chips[i] > 0) {
                pay[i] += each[i] - in_chips[i];
                in_chips[i] = each[i];
            }
        }
    }
}

// The deal of a P-player hold'em game (limitholdem/dealer.py: shuffle 52, deal_card = pop): the K = 2P + 5 dealt
// positions 51 .. 51 - K + 1 are fixed by the first K Fisher-Yates swaps, tracked in registers as in holdem_deal2;
// the other 51 - K draws only consume the stream. d[k] = card dealt k-th.
template <int K, class Rng>
__device__ __forceinline__ void holdem_deal_k(Rng& rng, uint32_t (&d)[K])
{
    // the K draws first (stream order), then every dealt position 51 - k traced back through the swaps q = K-1 .. 0
    // four per word (SWAR byte compares, as holdem_deal2): ~K^2/4 word steps instead of the K^2/2 pairwise lookups
    constexpr int NW = (K + 3) / 4;
    uint32_t js[NW], X[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
        js[w] = 0;
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) x |= (4 * w + b < K ? 51u - (uint32_t)(4 * w + b) : 63u) << (8 * b);
        X[w] = x;
    }
#pragma unroll
    for (int k = 0; k < K; k++) js[k >> 2] |= rng.interval(51u - (uint32_t)k) << (8 * (k & 3));
#pragma unroll
    for (int q = K - 1; q >= 0; q--) {
        const uint32_t I = (uint32_t)(51 - q) * 0x01010101u;
        const uint32_t J = __builtin_amdgcn_perm(0u, js[q >> 2], (uint32_t)(q & 3) * 0x01010101u);
        const uint32_t D = I ^ J;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            if (q > 4 * w + 3) continue;   // swap q never touches positions 51 - k, k < q
            const uint32_t both = ((X[w] ^ I) + 0x7F7F7F7Fu) & ((X[w] ^ J) + 0x7F7F7F7Fu);
            const uint32_t m = ~both & 0x80808080u;
            X[w] ^= D & (m - (m >> 7));
        }
    }
#pragma unroll
    for (int k = 0; k < K; k++) d[k] = (X[k >> 2] >> (8 * (k & 3))) & 63u;
    rng.skip_intervals(51u - K);
}

template <int P>
__device__ __forceinline__ int next_seat(int i) { return i + 1 == P ? 0 : i + 1; }

// ---- Leduc Hold'em, P = 3..5 (6-card deck: P hands + the public card) -------------------------------------------
// player word: hand:3 in:5 (3) raised:5 (8) folded:1 (13)
// shared word S: pub:3 rc:2 (3) ptr:3 (5) have_raised:2 (8) not_raise_num:4 (10) over:1 (31)
template <int NP>
struct LeducN {
    static_assert(NP >= 3 && NP <= 5, "leduc: 3..5 players");
    static constexpr int OBS = 36, A = 4, P = NP, LB = 1, WORDS = NP + 1, ACTION_BYTES = 1, NB = 2;
    static constexpr bool RING = true, RAW_OBS = false, PAYOFF_DRAWS = false;
    static constexpr int SCRATCH_WORDS = 0;
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 64, STAGE_PAD = 4, STAGE_R = 16, STAGE_RF = 24, RESTAGE_B = 4;
    static constexpr int MIN_WAVES = 4, EPW = 64, REFILL_K = 1;
    enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };
    __device__ __forceinline__ void bind(uint32_t*, const GameParams&) {}

    PlayerWords<NP> pw;
    uint32_t s;

    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = st[i * n + env];
        s = st[NP * n + env];
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
#pragma unroll
        for (int i = 0; i < NP; i++) st[i * n + env] = pw.w[i];
        st[NP * n + env] = s;
    }
    __device__ __forceinline__ void blank()
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = 0;
        s = 1u << 31;
    }
    __device__ __forceinline__ int current() const { return (int)bf(s, 5, 3); }
    __device__ __forceinline__ bool is_over() const { return (s >> 31) != 0; }
    __device__ __forceinline__ int max_raised() const
    {
        int m = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) m = max(m, (int)bf(pw.w[i], 8, 5));
        return m;
    }

    __device__ __forceinline__ uint32_t legal() const
    {
        const int mx = max_raised(), rp = (int)bf(pw.get(current()), 8, 5);
        uint32_t m = 0xF;
        if (bf(s, 8, 2) >= 2) m &= ~(1u << RAISE);
        if (rp < mx) m &= ~(1u << CHECK);
        if (rp == mx) m &= ~(1u << CALL);
        return m;
    }

    __device__ __forceinline__ void observe(int player, uint32_t (&bits)[NB]) const
    {
        int total = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) total += (int)bf(pw.w[i], 3, 5);
        const uint32_t me = pw.get(player);
        const int my = (int)bf(me, 3, 5), others = total - my + 21;
        uint64_t b = (1ull << (bf(me, 0, 3) >> 1)) | (1ull << (my + 6));
        if (others < 36) b |= 1ull << others;   // past slot 35 the reference raises IndexError: no bit
        if (bf(s, 3, 2) >= 1) b |= 1ull << ((bf(s, 0, 3) >> 1) + 3);
        bits[0] = (uint32_t)b;
        bits[1] = (uint32_t)(b >> 32);
    }

    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        uint32_t deck = 0x543210u;   // nibble i = card at deck position i
#pragma unroll
        for (uint32_t i = 5; i >= 1; i--) {
            const uint32_t j = rng.interval(i);
            const uint32_t ci = (deck >> (4 * i)) & 15u, cj = (deck >> (4 * j)) & 15u, x = ci ^ cj;
            deck ^= (x << (4 * i)) | (x << (4 * j));
        }
        const int sb = (int)rng.interval((uint32_t)(NP - 1)), bb = next_seat<NP>(sb);
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t chips = i == sb ? 1u : (i == bb ? 2u : 0u);
            pw.w[i] = ((deck >> (4 * (5 - i))) & 15u) | chips << 3 | chips << 8;   // raised = in_chips
        }
        s = ((deck >> (4 * (5 - NP))) & 15u) | (uint32_t)sb << 5;             // public card (hidden until rc 1)
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng&)
    {
        const uint32_t lg = legal();
        if (a < 0 || a > 3 || !((lg >> a) & 1u)) a = ((lg >> CHECK) & 1u) ? CHECK : FOLD;
        const int p = current(), mx = max_raised(), rc = (int)bf(s, 3, 2);
        int hr = (int)bf(s, 8, 2), nrn = (int)bf(s, 10, 4);
        uint32_t w = pw.get(p);
        const int rp = (int)bf(w, 8, 5), ra = rc == 0 ? 2 : 4;
        if (a == CALL) { w = bf_set(w, 3, 5, bf(w, 3, 5) + (uint32_t)(mx - rp)); w = bf_set(w, 8, 5, mx); nrn += 1; }
        else if (a == RAISE) { w = bf_set(w, 3, 5, bf(w, 3, 5) + (uint32_t)(mx - rp + ra)); w = bf_set(w, 8, 5, mx + ra); hr += 1; nrn = 1; }
        else if (a == FOLD) { w |= 1u << 13; }
        else { nrn += 1; }
        pw.set(p, w);
        int q = next_seat<NP>(p);
#pragma unroll
        for (int k = 0; k < NP; k++)   // skip the folded players (at least one is not)
            if ((pw.get(q) >> 13) & 1u) q = next_seat<NP>(q);
        int r = rc;
        if (nrn >= NP) {               // round over: public card after round 0 (raise 2 -> 4), raised reset
            r += 1; hr = 0; nrn = 0;
#pragma unroll
            for (int i = 0; i < NP; i++) pw.w[i] = bf_set(pw.w[i], 8, 5, 0);
        }
        int alive = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) alive += (int)(((pw.w[i] >> 13) & 1u) ^ 1u);
        const uint32_t over = alive == 1 || r >= 2;
        s = bf(s, 0, 3) | (uint32_t)r << 3 | (uint32_t)q << 5 | (uint32_t)hr << 8 | (uint32_t)nrn << 10 | over << 31;
    }

    __device__ __forceinline__ void payoffs(float (&out)[P]) const
    {
        int fold_count = 0, alive_idx = 0, total = 0, nwin = 0;
        bool win[NP];
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const bool f = (pw.w[i] >> 13) & 1u;
            fold_count += f ? 1 : 0;
            alive_idx = f ? alive_idx : i;
            total += (int)bf(pw.w[i], 3, 5);
            win[i] = false;
        }
        if (fold_count == NP - 1) {
#pragma unroll
            for (int i = 0; i < NP; i++) win[i] = i == alive_idx;
        } else {
            const int pr = (int)(bf(s, 0, 3) >> 1);
            int first = -1, mxr = -1;
#pragma unroll
            for (int i = NP - 1; i >= 0; i--) {   // the first (lowest) seat matching the public card, folded or not
                const int k = (int)(bf(pw.w[i], 0, 3) >> 1);
                first = k == pr ? i : first;
                mxr = k > mxr ? k : mxr;
            }
#pragma unroll
            for (int i = 0; i < NP; i++)
                win[i] = first >= 0 ? i == first : (int)(bf(pw.w[i], 0, 3) >> 1) == mxr;
        }
#pragma unroll
        for (int i = 0; i < NP; i++) nwin += win[i] ? 1 : 0;
        const double each = (double)total / (double)nwin;
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const double in = (double)bf(pw.w[i], 3, 5);
            out[i] = (float)((win[i] ? each - in : -in) / 2.0);
        }
    }
};

// ---- Limit Texas Hold'em, P = 3..22 ----------------------------------------------------------------------------------
// player word: c0:6 c1:6 in:8 (12) raised:6 (20) folded:1 (26)
// S0: board c0..c4 6 bits each; S1: ptr:5 rc:3 (5) have_raised:3 (8) not_raise_num:5 (11) use_prev:1 (16) over:1 (31)
// S2: raise_nums 4 x 3 (0..11), prev_raise_nums 4 x 3 (12..23) (the reset obs shows the previous game's, game.py:98)
template <int NP>
struct LimitN {
    static_assert(NP >= 3 && NP <= 22, "limit: 3..22 players (2P + 5 <= 52 dealt cards)");
    static constexpr int OBS = 72, A = 4, P = NP, LB = 1, WORDS = NP + 3, ACTION_BYTES = 1, NB = 3;
    static constexpr bool RING = true, RAW_OBS = false, PAYOFF_DRAWS = true;
    static constexpr int SCRATCH_WORDS = 0;
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 128, STAGE_PAD = 8, STAGE_R = 100, STAGE_RF = 120;
    static constexpr int RESTAGE_B = 8, MIN_WAVES = NP <= 10 ? 3 : 2, EPW = 64, REFILL_K = 2;
    enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };
    __device__ __forceinline__ void bind(uint32_t*, const GameParams&) {}

    PlayerWords<NP> pw;
    uint32_t s0, s1, s2;

    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = st[i * n + env];
        s0 = st[NP * n + env]; s1 = st[(NP + 1) * n + env]; s2 = st[(NP + 2) * n + env];
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
#pragma unroll
        for (int i = 0; i < NP; i++) st[i * n + env] = pw.w[i];
        st[NP * n + env] = s0; st[(NP + 1) * n + env] = s1; st[(NP + 2) * n + env] = s2;
    }
    __device__ __forceinline__ void blank()
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = 0;
        s0 = 0; s1 = 1u << 31; s2 = 0;
    }
    __device__ __forceinline__ int current() const { return (int)bf(s1, 0, 5); }
    __device__ __forceinline__ bool is_over() const { return (s1 >> 31) != 0; }
    __device__ __forceinline__ int max_raised() const
    {
        int m = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) m = max(m, (int)bf(pw.w[i], 20, 6));
        return m;
    }

    __device__ __forceinline__ uint32_t legal() const
    {
        const int mx = max_raised(), rp = (int)bf(pw.get(current()), 20, 6);
        uint32_t m = 0xF;
        if (bf(s1, 8, 3) >= 4) m &= ~(1u << RAISE);
        if (rp < mx) m &= ~(1u << CHECK);
        if (rp == mx) m &= ~(1u << CALL);
        return m;
    }

    __device__ __forceinline__ void observe(int player, uint32_t (&bits)[NB]) const
    {
        bits[0] = bits[1] = bits[2] = 0;
        const int r = (int)bf(s1, 5, 3), npub = r == 0 ? 0 : (r == 1 ? 3 : (r == 2 ? 4 : 5));
#pragma unroll
        for (int k = 0; k < 5; k++)
            if (k < npub) set_bit(bits, (int)bf(s0, 6 * k, 6));
        const uint32_t me = pw.get(player);
        set_bit(bits, (int)bf(me, 0, 6));
        set_bit(bits, (int)bf(me, 6, 6));
        const uint32_t rn = bf(s1, 16, 1) ? (s2 >> 12) : s2;
#pragma unroll
        for (int i = 0; i < 4; i++) set_bit(bits, 52 + 5 * i + (int)((rn >> (3 * i)) & 7u));
    }

    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        uint32_t d[2 * NP + 5];
        holdem_deal_k<2 * NP + 5>(rng, d);
        const int sb = (int)rng.interval((uint32_t)(NP - 1)), bb = next_seat<NP>(sb);
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t chips = i == sb ? 1u : (i == bb ? 2u : 0u);
            pw.w[i] = d[i] | d[NP + i] << 6 | chips << 12 | chips << 20;   // hole i -> player i % N, card i / N
        }
        s0 = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) s0 |= d[2 * NP + k] << (6 * k);
        s1 = (uint32_t)next_seat<NP>(bb) | 1u << 16;                    // first actor BB + 1; use_prev
        s2 = (s2 & 0xFFFu) << 12;                                       // prev <- current, current <- 0
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng&)
    {
        const uint32_t lg = legal();
        if (a < 0 || a > 3 || !((lg >> a) & 1u)) a = ((lg >> CHECK) & 1u) ? CHECK : FOLD;
        const int p = current(), mx = max_raised(), rc = (int)bf(s1, 5, 3);
        int hr = (int)bf(s1, 8, 3), nrn = (int)bf(s1, 11, 5);
        uint32_t w = pw.get(p);
        const int rp = (int)bf(w, 20, 6), ra = rc >= 2 ? 4 : 2;
        if (a == CALL) { w = bf_set(w, 12, 8, bf(w, 12, 8) + (uint32_t)(mx - rp)); w = bf_set(w, 20, 6, mx); nrn += 1; }
        else if (a == RAISE) { w = bf_set(w, 12, 8, bf(w, 12, 8) + (uint32_t)(mx - rp + ra)); w = bf_set(w, 20, 6, mx + ra); hr += 1; nrn = 1; }
        else if (a == FOLD) { w |= 1u << 26; }
        else { nrn += 1; }
        pw.set(p, w);
        int q = next_seat<NP>(p);
#pragma unroll
        for (int k = 0; k < NP; k++)
            if ((pw.get(q) >> 26) & 1u) q = next_seat<NP>(q);
        s2 = (s2 & ~(7u << (3 * rc))) | ((uint32_t)hr << (3 * rc));    // history_raise_nums[round] = have_raised
        int r = rc;
        if (nrn >= NP) {
            r += 1; hr = 0; nrn = 0;
#pragma unroll
            for (int i = 0; i < NP; i++) pw.w[i] = bf_set(pw.w[i], 20, 6, 0);
        }
        int alive = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) alive += (int)(((pw.w[i] >> 26) & 1u) ^ 1u);
        const uint32_t over = alive == 1 || r >= 4;
        s1 = (uint32_t)q | (uint32_t)r << 5 | (uint32_t)hr << 8 | (uint32_t)nrn << 11 | over << 31;   // use_prev cleared
    }

    template <class Rng>
    __device__ __forceinline__ void payoffs(float (&out)[P], Rng& rng) const
    {
        uint32_t value[NP];
        int in[NP], pay[NP], alive = 0;
        uint64_t bc = 0, bs = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) tally_card((int)bf(s0, 6 * k, 6), bc, bs);
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t w = pw.w[i];
            in[i] = (int)bf(w, 12, 8);
            const bool folded = (w >> 26) & 1u;
            alive += folded ? 0 : 1;
            uint64_t c = bc, sm = bs;
            tally_card((int)bf(w, 0, 6), c, sm);
            tally_card((int)bf(w, 6, 6), c, sm);
            value[i] = folded ? 0u : holdem_rank7(c, sm);
        }
        if (alive == 1) {   // compare_hands: the one hand left wins unevaluated
#pragma unroll
            for (int i = 0; i < NP; i++) value[i] = value[i] ? 1u : 0u;
        }
        holdem_judge<NP>(value, in, rng, pay);
#pragma unroll
        for (int i = 0; i < NP; i++) out[i] = (float)pay[i] * 0.5f;
    }
};

// ---- No-limit Texas Hold'em, P = 3..22 -------------------------------------------------------------------------------
// player word: c0:6 c1:6 in:8 (12) raised:8 (20) status:2 (28; 0 alive, 1 folded, 2 all-in)
// S0: board c0..c4 6 bits each; S1: ptr:5 rc:3 (5) not_raise_num:8 (8) not_playing_num:8 (16) dealer:5 (24)
//     dealer drawn:1 (29) over:1 (31); S2: round pot + 1 (0 = the live pot; cs_nolimit.h round_pot). The stack is
//     chips_for_each - in (not stored).
template <int NP>
struct NolimitN {
    static_assert(NP >= 3 && NP <= 22, "no-limit: 3..22 players (2P + 5 <= 52 dealt cards)");
    static constexpr int OBS = 54, A = 5, P = NP, LB = 1, WORDS = NP + 3, ACTION_BYTES = 1, NB = 14;
    static constexpr bool RING = true, RAW_OBS = true, PAYOFF_DRAWS = true;
    static constexpr int SCRATCH_WORDS = 0;
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 128, STAGE_PAD = 8, STAGE_R = 100, STAGE_RF = 100;
    static constexpr int RESTAGE_B = 8, MIN_WAVES = NP <= 10 ? 3 : 2, EPW = 64, REFILL_K = 2;
    enum { FOLD = 0, CHECK_CALL = 1, RAISE_HALF_POT = 2, RAISE_POT = 3, ALL_IN = 4 };
    enum { ALIVE = 0, FOLDED = 1, ALLIN = 2 };

    int chips, dealer_cfg;
    PlayerWords<NP> pw;
    uint32_t s0, s1, s2;

    __device__ __forceinline__ void bind(uint32_t*, const GameParams& prm)
    {
        chips = prm.chips_for_each;
        dealer_cfg = prm.dealer_id;
    }
    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = st[i * n + env];
        s0 = st[NP * n + env]; s1 = st[(NP + 1) * n + env]; s2 = st[(NP + 2) * n + env];
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
#pragma unroll
        for (int i = 0; i < NP; i++) st[i * n + env] = pw.w[i];
        st[NP * n + env] = s0; st[(NP + 1) * n + env] = s1; st[(NP + 2) * n + env] = s2;
    }
    __device__ __forceinline__ void blank()
    {
#pragma unroll
        for (int i = 0; i < NP; i++) pw.w[i] = 0;
        s0 = 0; s1 = 1u << 31; s2 = 0;
    }
    __device__ __forceinline__ int current() const { return (int)bf(s1, 0, 5); }
    __device__ __forceinline__ bool is_over() const { return (s1 >> 31) != 0; }
    __device__ __forceinline__ int max_raised() const
    {
        int m = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) m = max(m, (int)bf(pw.w[i], 20, 8));
        return m;
    }
    __device__ __forceinline__ int pot() const   // the pot the round reads: dealer.pot = sum of in_chips, or S2
    {
        int t = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) t += (int)bf(pw.w[i], 12, 8);
        return s2 ? (int)s2 - 1 : t;
    }

    // round.py:132-165 for the player at the pointer
    __device__ __forceinline__ uint32_t legal() const
    {
        const uint32_t w = pw.get(current());
        const int mx = max_raised(), rp = (int)bf(w, 20, 8), rem = chips - (int)bf(w, 12, 8), pt = pot();
        const int half = pt >> 1, diff = mx - rp;
        uint32_t m = 0x1F;
        if (diff > 0 && diff >= rem) {
            m = (1u << FOLD) | (1u << CHECK_CALL);
        } else {
            if (pt > rem) m &= ~(1u << RAISE_POT);
            if (half > rem || half + rp <= mx) m &= ~(1u << RAISE_HALF_POT);
        }
        return m;
    }

    __device__ __forceinline__ void observe(int player, uint32_t (&raw)[NB]) const
    {
        uint64_t cards = 0;
        const int r = (int)bf(s1, 5, 3), npub = r == 0 ? 0 : (r + 2 < 5 ? r + 2 : 5);
#pragma unroll
        for (int k = 0; k < 5; k++)
            if (k < npub) cards |= 1ull << bf(s0, 6 * k, 6);
        const uint32_t me = pw.get(player);
        cards |= 1ull << bf(me, 0, 6);
        cards |= 1ull << bf(me, 6, 6);
#pragma unroll
        for (int j = 0; j < 13; j++) raw[j] = RowWriter<4>::expand4((uint32_t)(cards >> (4 * j)) & 15u);
        int mx = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) mx = max(mx, (int)bf(pw.w[i], 12, 8));
        raw[13] = bf(me, 12, 8) | (uint32_t)mx << 8;
    }

    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        int dealer;   // randint(0, N) by the first game when configured None, then kept (game.py:62-63)
        if (dealer_cfg >= 0) dealer = dealer_cfg;
        else if (bf(s1, 29, 1)) dealer = (int)bf(s1, 24, 5);
        else dealer = (int)rng.interval((uint32_t)(NP - 1));
        uint32_t d[2 * NP + 5];
        holdem_deal_k<2 * NP + 5>(rng, d);
        const int sb = next_seat<NP>(dealer), bb = next_seat<NP>(sb);
        const int bbc = chips < 2 ? chips : 2, sbc = chips < 1 ? chips : 1;   // bets clamp to the stack
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t c = i == bb ? (uint32_t)bbc : (i == sb ? (uint32_t)sbc : 0u);
            pw.w[i] = d[i] | d[NP + i] << 6 | c << 12 | c << 20;           // raised = in_chips, status alive
        }
        s0 = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) s0 |= d[2 * NP + k] << (6 * k);
        s1 = (uint32_t)next_seat<NP>(bb) | (uint32_t)dealer << 24 | 1u << 29;
        s2 = 0;
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng&)
    {
        const uint32_t lg = legal();
        if (a < 0 || a > 4 || !((lg >> a) & 1u)) a = CHECK_CALL;
        const int p = current(), mx = max_raised(), pt = pot();
        int r = (int)bf(s1, 5, 3), nrn = (int)bf(s1, 8, 8), npn = (int)bf(s1, 16, 8);
        uint32_t w = pw.get(p);
        int ip = (int)bf(w, 12, 8), rp = (int)bf(w, 20, 8), sp = (int)bf(w, 28, 2);
        int want = 0;   // chips asked for; bet() clamps to the stack
        if (a == CHECK_CALL) { want = mx - rp; rp = mx; nrn += 1; }
        else if (a == ALL_IN) { want = chips - ip; rp += want; nrn = 1; }
        else if (a == RAISE_POT) { want = pt; rp += pt; nrn = 1; }
        else if (a == RAISE_HALF_POT) { want = pt >> 1; rp += want; nrn = 1; }
        else { sp = FOLDED; }
        const int rem = chips - ip;
        ip += want < rem ? want : rem;
        if (ip == chips && sp != FOLDED) sp = ALLIN;
        if (sp == ALLIN) { npn += 1; nrn -= 1; }
        if (sp == FOLDED) npn += 1;
        pw.set(p, (w & 0xFFFu) | (uint32_t)ip << 12 | (uint32_t)(rp & 255) << 20 | (uint32_t)sp << 28);
        int q = next_seat<NP>(p);
#pragma unroll
        for (int k = 0; k < NP; k++)
            if (bf(pw.get(q), 28, 2) == FOLDED) q = next_seat<NP>(q);
        // game.py:135-141 bypass: folded / all-in players, and the last other one if already level
        uint32_t by = 0;
        int nby = 0, last = -1;
#pragma unroll
        for (int i = NP - 1; i >= 0; i--) {
            const bool b = bf(pw.w[i], 28, 2) != ALIVE;
            by |= b ? 1u << i : 0u;
            nby += b ? 1 : 0;
            last = b ? last : i;   // players_in_bypass.index(0)
        }
        if (NP - nby == 1 && (int)bf(pw.get(last), 20, 8) >= max_raised()) { by |= 1u << last; nby += 1; }
        if (nrn + npn >= NP) {   // round over: pointer dealer + 1 past bypassed players (unless all are), deal
            int g = next_seat<NP>((int)bf(s1, 24, 5));
            if (nby < NP) {
#pragma unroll
                for (int k = 0; k < NP; k++)
                    if ((by >> g) & 1u) g = next_seat<NP>(g);
            }
            q = g;
            r = nby == NP ? 4 : r + 1;   // everyone bypassed: flop, turn and river all dealt
            nrn = 0;
#pragma unroll
            for (int i = 0; i < NP; i++) pw.w[i] = bf_set(pw.w[i], 20, 8, 0);
        }
        int in_hand = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) in_hand += bf(pw.w[i], 28, 2) != FOLDED ? 1 : 0;
        const uint32_t over = in_hand == 1 || r >= 4;
        s1 = (uint32_t)q | (uint32_t)r << 5 | (uint32_t)(nrn & 255) << 8 | (uint32_t)(npn & 255) << 16 |
             (s1 & (0x3Fu << 24)) | over << 31;
    }

    template <class Rng>
    __device__ __forceinline__ void payoffs(float (&out)[P], Rng& rng) const
    {
        uint32_t value[NP];
        int in[NP], pay[NP], in_hand = 0;
        uint64_t bc = 0, bs = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) tally_card((int)bf(s0, 6 * k, 6), bc, bs);
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t w = pw.w[i];
            in[i] = (int)bf(w, 12, 8);
            const bool folded = bf(w, 28, 2) == FOLDED;
            in_hand += folded ? 0 : 1;
            uint64_t c = bc, sm = bs;
            tally_card((int)bf(w, 0, 6), c, sm);
            tally_card((int)bf(w, 6, 6), c, sm);
            value[i] = folded ? 0u : holdem_rank7(c, sm);
        }
        if (in_hand == 1) {
#pragma unroll
            for (int i = 0; i < NP; i++) value[i] = value[i] ? 1u : 0u;
        }
        holdem_judge<NP>(value, in, rng, pay);
#pragma unroll
        for (int i = 0; i < NP; i++) out[i] = (float)pay[i];
    }
};

}  // namespace cs
