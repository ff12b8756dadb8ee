// cs_blackjack.h -- Blackjack (1..4 players, 1 deck or infinite deck) as a lane-per-env lockstep state machine.
//
// Behaviour (reference file:line):
//   rlcard/games/blackjack/dealer.py:4-37   52-card deck shuffled once per game (np.array + np_random.shuffle); deal_card:
//                                           idx = np_random.choice(len(deck)), card = deck[idx], deck.pop(idx) unless
//                                           num_decks == 0 (infinite deck: the card stays)
//   rlcard/games/blackjack/game.py:22-54    init_game: two rounds of (player 0..P-1, dealer); judge_round all
//   rlcard/games/blackjack/game.py:56-123   step: any action but 'stand' hits; a bust or a stand by the last player
//                                           makes the dealer draw while score < 17, then judge_game for every player
//   rlcard/games/blackjack/game.py:160-205  state: own hand; dealer hand[1:] until the game is over; is_over
//   rlcard/games/blackjack/judger.py:2-73   scores with soft aces; winner codes 2 / 1 / -1
//   rlcard/envs/blackjack.py:38-103         obs = [score(own), score(dealer visible)], legal {hit, stand}, payoff 1/0/-1
// The shuffle is applied once per game, in the reset's pass over the staged stream bytes: each accepted draw swaps two
// bytes of the identity deck laid out in the lane's LDS scratch (in-order LDS: a swap waits only for its own two
// loads), and the shuffled deck then lives in registers (13 words). A dealt position's card is a select over those
// words (~18 VALU; undoing the 51 swaps per card instead cost ~270). "deck.pop(idx)" is an order-statistic removal: a
// 52-bit removed mask over the shuffled positions; the idx-th remaining card is the idx-th clear bit.
// Packed state, 32 u32 words per env (word-major [32][N]):
//   0..12  the shuffled deck: byte p = card id (sorted-deck index) at position p
//   13     removed mask bits 0..31;  14: removed bits 32..51 | deck_len << 20 | game_pointer << 26 | over << 29
//   15..29 hands: hand h (players 0..P-1, dealer = P) bytes 12h .. 12h+11 (words past 15 + 3 (P + 1) stay zero)
//   30     hand sizes 4 bits each (5 hands) | winner codes 2 bits per player << 20 (0 none, 1 tie, 2 win, 3 loss)
// Inside a kernel words 0..12 are registers; 13, 14, 30 and the hands a per-lane LDS scratch (lane-interleaved, so
// uniform word indices are bank-conflict free; the hands are indexed dynamically), which the reset's draw pass also
// uses to shuffle the deck (per-lane byte positions) before it moves to registers.
#pragma once
#include "cs_device.h"
#include "cs_prof.h"

namespace cs {

template <int NP>
struct Blackjack {
    static constexpr int OBS = 2, A = 2, P = NP, LB = 1, WORDS = 32, ACTION_BYTES = 1;
    static constexpr int NB = 1;               // raw obs dwords
    static constexpr bool RING = true;          // MT stream as the byte ring (cs_ring.h)
    static constexpr bool RAW_OBS = true;      // observe() returns byte values, not a 0/1 bitmap
    static constexpr int HAND_CAP = 12;
    static constexpr int HAND_W = 3 * (NP + 1);                 // state words 15.. the hands use
    static constexpr int SCRATCH_WORDS = 3 + HAND_W > 13 ? 3 + HAND_W : 13;   // >= 13: the reset's deck bytes
    // MT staging (see MtLaneT)
    // MT staging rows of 128 bytes: the reset's ~57 draws come out of one branch-free pass over them
    // (RingLane::draw_intervals); measured 17.2 ms per 2^20 x 64 launch vs 19.9 with 64-byte rows (3 waves per SIMD
    // instead of 2, but more draws past the row) and 35.0 with 256-byte rows (1 wave); R 72..112 the same
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 128, STAGE_PAD = 8, STAGE_R = 100;
    static constexpr int RESTAGE_B = 8;   // row loads in flight per lane and restage pass (128-byte rows: 8 > 4 > 1)
    static constexpr int MIN_WAVES = 3;   // the LDS (stage rows + scratch) allows 3 blocks of 4 waves per CU
    static constexpr int EPW = 64;        // rollout envs per wave (lane_ctx)
    static constexpr int REFILL_K = 2;   // stale blocks twisted per pass (see mt_refill_wave)

    uint32_t* s;       // lane scratch: word i at s[i * WAVE]: 0 = state word 13, 1 = 14, 2 = 30, 3 + q = 15 + q
    int infinite;
    uint32_t jw[13];   // state words 0..12: the shuffled deck, byte p = the card at position p
    // running judge totals (registers, rebuilt from the hands by load()): hand h's card values with aces as 11 |
    // its aces << 8; [NP + 1] the same over the dealer's cards after the first (the visible dealer score)
    uint32_t tot[NP + 2];

    __device__ __forceinline__ uint32_t& L(int i) const { return s[i * WAVE]; }
    __device__ __forceinline__ uint32_t& removed_lo() const { return L(0); }
    __device__ __forceinline__ uint32_t& meta() const { return L(1); }     // state word 14
    __device__ __forceinline__ uint32_t& sizes() const { return L(2); }    // state word 30
    __device__ __forceinline__ int hand_byte(int h, int k) const
    {
        const int b = HAND_CAP * h + k;
        return (L(3 + (b >> 2)) >> (8 * (b & 3))) & 255;
    }
    __device__ __forceinline__ void set_hand_byte(int h, int k, int v) const
    {
        const int b = HAND_CAP * h + k;
        uint32_t& w = L(3 + (b >> 2));
        const int sh = 8 * (b & 3);
        w = (w & ~(255u << sh)) | ((uint32_t)v << sh);
    }

    __device__ __forceinline__ void bind(uint32_t* lane_scratch, const GameParams& prm)
    {
        s = lane_scratch;
        infinite = prm.num_decks == 0;
    }
    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
#pragma unroll
        for (int i = 0; i < 13; i++) jw[i] = st[(int64_t)i * n + env];
        removed_lo() = st[13 * n + env];
        meta() = st[14 * n + env];
        sizes() = st[30 * n + env];
#pragma unroll
        for (int q = 0; q < HAND_W; q++) L(3 + q) = st[(int64_t)(15 + q) * n + env];
#pragma unroll
        for (int h = 0; h <= NP; h++) {
            uint32_t t = 0, t1 = 0;
            for (int k = 0; k < nhand(h); k++) {
                const uint32_t v = card_tot(hand_byte(h, k));
                t += v;
                t1 += k > 0 ? v : 0u;
            }
            tot[h] = t;
            if (h == NP) tot[NP + 1] = t1;
        }
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
#pragma unroll
        for (int i = 0; i < 13; i++) st[(int64_t)i * n + env] = jw[i];
        st[13 * n + env] = removed_lo();
        st[14 * n + env] = meta();
        st[30 * n + env] = sizes();
#pragma unroll
        for (int q = 0; q < 15; q++) st[(int64_t)(15 + q) * n + env] = q < HAND_W ? L(3 + q) : 0u;
        st[31 * n + env] = 0u;
    }
    __device__ __forceinline__ void clear_table()
    {
        removed_lo() = 0;
        meta() = 52u << 20;
        sizes() = 0;
#pragma unroll
        for (int q = 0; q < HAND_W; q++) L(3 + q) = 0;
#pragma unroll
        for (int h = 0; h < NP + 2; h++) tot[h] = 0;
    }
    __device__ __forceinline__ void blank()
    {
#pragma unroll
        for (int i = 0; i < 13; i++) jw[i] = 0;
        clear_table();
        meta() = 1u << 29;
    }

    __device__ __forceinline__ int nhand(int h) const { return (sizes() >> (4 * h)) & 15; }
    __device__ __forceinline__ int winner(int p) const { return (sizes() >> (20 + 2 * p)) & 3; }
    __device__ __forceinline__ int current() const { return (meta() >> 26) & 7; }
    __device__ __forceinline__ bool is_over() const { return (meta() >> 29) & 1; }
    __device__ __forceinline__ uint32_t legal() const { return 3u; }

    __device__ static __forceinline__ int card_value(int c)
    {
        const int r = c % 13;
        return r == 0 ? 11 : (r >= 9 ? 10 : r + 1);
    }
    // a card's judge value (judger.py judge_score: A = 11, J/Q/K = 10) | ace << 8
    __device__ static __forceinline__ uint32_t card_tot(int c)
    {
        const int r = c % 13;
        return r == 0 ? 11u + 256u : (r >= 9 ? 10u : (uint32_t)r + 1u);
    }
    // judge_score from a running total: aces count 1 instead of 11 while the score is over 21, i.e.
    // min(aces, ceil((score - 21) / 10)) of them ((x * 205) >> 11 == x / 10 for the x <= 132 here)
    __device__ static __forceinline__ int score_of(uint32_t t)
    {
        const int sc = (int)(t & 255u), aces = (int)(t >> 8);
        const int need = sc > 21 ? ((sc - 12) * 205) >> 11 : 0;
        return sc - 10 * (need < aces ? need : aces);
    }
    // judge_score of hand h (all its cards; from = 1: the dealer's cards after the first)
    __device__ __forceinline__ int score(int h, int from) const
    {
        uint32_t t = tot[0];
#pragma unroll
        for (int q = 1; q <= NP; q++) t = h == q ? tot[q] : t;
        return score_of(from ? tot[NP + 1] : t);
    }

    // the k-th (0-based) set bit of a 64-bit mask: popcount bisection, no per-bit loop
    __device__ static __forceinline__ int select_bit(uint64_t m, int k)
    {
        const uint32_t lo = (uint32_t)m;
        const int clo = __popc(lo);
        const bool up = k >= clo;
        uint32_t v = up ? (uint32_t)(m >> 32) : lo;
        k -= up ? clo : 0;
        int base = up ? 32 : 0;
#pragma unroll
        for (int sh = 16; sh >= 1; sh >>= 1) {
            const int c = __popc(v & ((1u << sh) - 1u));
            const bool u = k >= c;
            k -= u ? c : 0;
            v = u ? v >> sh : v;
            base += u ? sh : 0;
        }
        return base;
    }
    // the card at deck position x: byte x & 3 of word x >> 2, the word picked by a select tree on the bits of x >> 2
    // (bitwise selects, v_bfi_b32: as ?: on an array the compiler turns the tree into a dynamically indexed stack copy)
    __device__ __forceinline__ int card_at(int x) const
    {
        const uint32_t w = (uint32_t)x >> 2;
        const uint32_t m0 = 0u - (w & 1u), m1 = 0u - ((w >> 1) & 1u), m2 = 0u - ((w >> 2) & 1u), m3 = 0u - (w >> 3);
        const auto sel = [](uint32_t m, uint32_t hi, uint32_t lo) { return (hi & m) | (lo & ~m); };
        const uint32_t a0 = sel(m0, jw[1], jw[0]), a1 = sel(m0, jw[3], jw[2]), a2 = sel(m0, jw[5], jw[4]);
        const uint32_t a3 = sel(m0, jw[7], jw[6]), a4 = sel(m0, jw[9], jw[8]), a5 = sel(m0, jw[11], jw[10]);
        const uint32_t b0 = sel(m1, a1, a0), b1 = sel(m1, a3, a2), b2 = sel(m1, a5, a4);
        const uint32_t c0 = sel(m2, b1, b0), c1 = sel(m2, jw[12], b2);
        const uint32_t d = sel(m3, c1, c0);
        return (int)__builtin_amdgcn_ubfe(d, 8u * ((uint32_t)x & 3u), 8u);
    }

    // Dealer.deal_card's draw: idx = choice(len(deck)), the idx-th remaining position; deck.pop(idx) unless infinite
    template <class Rng>
    __device__ __forceinline__ int deal_pos(Rng& rng)
    {
        const uint32_t m1 = meta();
        const int len = (m1 >> 20) & 63;
        const int idx = (int)rng.interval((uint32_t)(len - 1));
        const uint64_t avail = ~((uint64_t)removed_lo() | (uint64_t)(m1 & 0xFFFFFu) << 32) & ((1ull << 52) - 1);
        const int pos = select_bit(avail, idx);
        if (!infinite) {
            uint32_t m2 = (m1 & ~(63u << 20)) | (uint32_t)(len - 1) << 20;
            if (pos < 32) removed_lo() |= 1u << pos;
            else m2 |= 1u << (pos - 32);
            meta() = m2;
        }
        return pos;
    }
    __device__ __forceinline__ void add_card(int h, int c)
    {
        const int n = nhand(h);
        if (n < HAND_CAP) {      // 12 cards always bust a 1-deck hand before this bound
            set_hand_byte(h, n, c);
            sizes() += 1u << (4 * h);
            const uint32_t v = card_tot(c);
#pragma unroll
            for (int q = 0; q <= NP; q++) tot[q] += h == q ? v : 0u;
            tot[NP + 1] += h == NP && n > 0 ? v : 0u;
        }
    }
    template <class Rng>
    __device__ __forceinline__ void deal(Rng& rng, int h)
    {
        add_card(h, card_at(deal_pos(rng)));
    }

    __device__ __forceinline__ void observe(int player, uint32_t (&raw)[NB]) const
    {
        const int mine = score(player, 0);
        const int dealer = is_over() ? score(NP, 0) : score(NP, 1);
        raw[0] = (uint32_t)mine | (uint32_t)dealer << 8;
    }

    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        // 52-card Fisher-Yates (i = 51..1, j = randint(0, i + 1); dealer.py:4-37) on the identity deck in scratch words
        // 0..12 (byte p of the lane's deck at (p >> 2) * WAVE words + p & 3), each accepted draw swapping positions i
        // and j where the draw pass finds it; then the deck into registers, and the initial deal (game.py:22-54): two
        // rounds of players 0..P-1 and the dealer
#pragma unroll
        for (int w = 0; w < 13; w++) L(w) = 0x03020100u + 0x04040404u * (uint32_t)w;
        uint8_t* deck = (uint8_t*)s;
        rng.draw_intervals(51u, [&](uint32_t k, uint32_t j) {
            const uint32_t i = 51u - k;
            // (p >> 2) * 256 + (p & 3) as p + 252 * (p >> 2): a shift and a 24-bit multiply-add
            static_assert(WAVE * 4 == 256, "deck byte address");
            uint8_t* pi = deck + (i + __umul24(i >> 2, 252u));
            uint8_t* pj = deck + (j + __umul24(j >> 2, 252u));
            const uint8_t ci = *pi, cj = *pj;
            *pi = cj;
            *pj = ci;
        });
#pragma unroll
        for (int w = 0; w < 13; w++) jw[w] = L(w);
        clear_table();
        constexpr int ND = 2 * (NP + 1);
#pragma unroll
        for (int d = 0; d < ND; d++) add_card(d % (NP + 1), card_at(deal_pos(rng)));
    }

    template <class Rng>
    __device__ __forceinline__ void finish(Rng& rng)
    {
        while (score(NP, 0) < 17) deal(rng, NP);
        const int d = score(NP, 0);
        uint32_t win = 0;
        for (int p = 0; p < NP; p++) {
            const int sp = score(p, 0);
            int code;
            if (sp > 21) code = 3;
            else if (d > 21) code = 2;
            else if (sp > d) code = 2;
            else if (sp < d) code = 3;
            else code = 1;
            win |= (uint32_t)code << (20 + 2 * p);
        }
        sizes() = (sizes() & 0xFFFFFu) | win;
        meta() = (meta() & ~(7u << 26)) | 1u << 29;   // game_pointer = 0, over
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng& rng)
    {
        const int gp = current();
        bool advance = true;
        if (a != 1) {
            deal(rng, gp);
            advance = score(gp, 0) > 21;
        }
        if (advance) {
            if (gp >= NP - 1) finish(rng);
            else meta() = (meta() & ~(7u << 26)) | (uint32_t)(gp + 1) << 26;
        }
    }

    __device__ __forceinline__ void payoffs(float (&r)[P]) const
    {
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const int w = winner(p);
            r[p] = w == 2 ? 1.f : (w == 1 ? 0.f : -1.f);
        }
    }
};

}  // namespace cs
