// cs_limit.h -- Limit Texas Hold'em (2 players) as a lane-per-env lockstep state machine.
//
// Behaviour (reference file:line):
//   rlcard/utils/utils.py:34-43                standard deck: suits S,H,D,C x ranks A..K  (card id = card2index)
//   rlcard/games/limitholdem/dealer.py:4-21    shuffle at construction, deal_card = deck.pop()
//   rlcard/games/limitholdem/game.py:46-103    init_game: hole i -> player i%2 from deck[51-i]; SB = randint(0,2);
//                                              first actor (BB+1)%2; the reset obs carries the PREVIOUS game's
//                                              raise counts (get_state at :98 runs before history_raise_nums is
//                                              re-bound at :101) -- kept as prev_raise_nums + use_prev
//   rlcard/games/limitholdem/game.py:105-158   step: history_raise_nums[round] = have_raised; flop deck[47..45],
//                                              turn deck[44], river deck[43]; raise amount 2 -> 4 after round 1
//   rlcard/games/limitholdem/round.py:53-127   betting FSM, allowed_raise_num = 4
//   rlcard/games/limitholdem/game.py:216-243   is_over: one alive or round_counter >= 4; payoffs / big_blind
//   rlcard/games/limitholdem/judger.py:11-108  pot split (2 players: the winner nets the loser's bet, ties return
//                                              the bets, np_random is never drawn)
//   rlcard/games/limitholdem/utils.py:3-614    7-card ranking (== standard poker order; bitmask evaluator below)
//   rlcard/envs/limitholdem.py:40-96           obs[72] (card bits + 52 + 5*round + raises) and the id fallback
// Shuffle: Fisher-Yates fixes position i at step i, and only deck[43..51] is ever dealt, so the first nine swaps are
// tracked in registers (a 9-entry position map) and the remaining 42 steps only consume their random_interval draws.
// Packed state, 4 u32 words per env (word-major [4][N]):
//   w0: hole cards p0c0:6 p0c1:6 p1c0:6 p1c1:6 in0:6 (bits 24..29) ptr:1 (30) over:1 (31)
//   w1: board c0..c4 6 bits each (0..29)
//   w2: in1:6 r0:5 r1:5 have_raised:3 not_raise_num:2 rc:3 f0:1 f1:1 use_prev:1 (bits 0..26)
//   w3: raise_nums 4x3 (0..11), prev_raise_nums 4x3 (12..23)
#pragma once
#include "cs_device.h"

namespace cs {

__device__ __forceinline__ int top_bit(uint32_t m) { return 31 - __builtin_clz(m); }

// highest straight top rank (2=0 .. A=12) in a 13-bit rank mask, -1 if none; the wheel tops at 5 (= 3)
__device__ __forceinline__ int top_straight13(uint32_t mask)
{
    const uint32_t m = (mask << 1) | ((mask >> 12) & 1u);
    const uint32_t x = m & (m >> 1) & (m >> 2) & (m >> 3) & (m >> 4);
    return x ? top_bit(x) + 3 : -1;
}

// 7-card hand value; larger = better, equal = split. cat << 20 | five 4-bit tiebreak ranks
// a card (card2index: suit * 13 + (A, 2..K)) into the evaluator's tallies: 13 rank-count nibbles (2 = 0 .. A = 12)
// and a 13-bit rank mask per suit (packed 4 x 16 bits)
__device__ __forceinline__ void tally_card(int c, uint64_t& cnt, uint64_t& sm)
{
    const int s = c / 13, q = c - 13 * s, r = q == 0 ? 12 : q - 1;
    cnt += 1ull << (4 * r);
    sm |= 1ull << (16 * s + r);
}

// 7-card category << 20 | five tiebreak ranks, from the tallies of the 7 cards (the board's are shared by both
// players: tallied once)
// Branch-free form (the default): the rank-count bit planes come from the four suit masks by a bit-sliced adder
// (count = a + b + c + d per rank bit), every category's tie-break ranks are computed and the category picks them,
// so a wave's lanes never diverge on the hand category (an if-chain executes the union of the categories its lanes
// hold: No-limit 3.09 -> 2.66 ms, Limit 2.61 -> 2.50 with this form).
// highest set bit of m removed; its rank (31 - clz) in r (0xFFFFFFFF for m = 0, never packed)
__device__ __forceinline__ uint32_t pop_top(uint32_t m, uint32_t& r)
{
    const uint32_t z = __clz(m);
    r = 31u - z;
    return m & ~(0x80000000u >> (z & 31u));
}
__device__ __forceinline__ uint32_t holdem_rank7_bf(uint64_t smp)
{
    const uint32_t a = (uint32_t)smp & 0x1FFFu, b = (uint32_t)(smp >> 16) & 0x1FFFu, c = (uint32_t)(smp >> 32) & 0x1FFFu,
                   d = (uint32_t)(smp >> 48) & 0x1FFFu;
    const uint32_t x1 = a ^ b, c1 = a & b, x2 = c ^ d, c2 = c & d, c3 = x1 & x2;
    const uint32_t B0 = x1 ^ x2, B1 = c1 ^ c2 ^ c3, m4 = c1 & c2;           // count = B0 + 2 B1 + 4 m4 per rank
    const uint32_t m3 = B0 & B1, m2 = B1 & ~B0, m1 = B0 & ~B1, all = a | b | c | d;
    uint32_t fm = __popc(a) >= 5 ? a : 0u;
    fm = __popc(b) >= 5 ? b : fm;
    fm = __popc(c) >= 5 ? c : fm;
    fm = __popc(d) >= 5 ? d : fm;
    const int sf = fm ? top_straight13(fm) : -1, st = top_straight13(all);
    const int n3 = __popc(m3), n2 = __popc(m2);
    const bool isSF = sf >= 0, isQ = m4 != 0u, isFH = n3 >= 2 || (n3 == 1 && n2 >= 1), isF = fm != 0u,
               isS = st >= 0, isT = n3 >= 1, is2P = n2 >= 2, isP = n2 >= 1;
    // the five highest of the flush suit (category flush) or of the single ranks (kickers of trips / pair / high)
    const bool flush_cat = isF && !isSF && !isQ && !isFH;
    uint32_t k0, k1, k2, k3, k4;
    uint32_t x = flush_cat ? fm : m1;
    x = pop_top(x, k0); x = pop_top(x, k1); x = pop_top(x, k2); x = pop_top(x, k3); (void)pop_top(x, k4);
    uint32_t q0, t0, p0, p1, rq, rfh, r2p;
    (void)pop_top(all & ~m4, rq);                    // quads: the kicker is the best other rank
    const uint32_t r3 = pop_top(m3, t0);
    (void)pop_top(r3 | m2, rfh);                     // full house: best pair among the other trips and the pairs
    uint32_t rem2 = pop_top(m2, p0);
    rem2 = pop_top(rem2, p1);
    (void)pop_top(all & ~(1u << (p0 & 31u)) & ~(1u << (p1 & 31u)), r2p);   // two pair: best other rank
    (void)pop_top(m4, q0);
    uint32_t cat, v;   // v = the five 4-bit tie-break ranks
    if (isSF) { cat = 9; v = (uint32_t)sf << 16; }
    else if (isQ) { cat = 8; v = q0 << 16 | rq << 12; }
    else if (isFH) { cat = 7; v = t0 << 16 | rfh << 12; }
    else if (isF) { cat = 6; v = k0 << 16 | k1 << 12 | k2 << 8 | k3 << 4 | k4; }
    else if (isS) { cat = 5; v = (uint32_t)st << 16; }
    else if (isT) { cat = 4; v = t0 << 16 | k0 << 12 | k1 << 8; }
    else if (is2P) { cat = 3; v = p0 << 16 | p1 << 12 | r2p << 8; }
    else if (isP) { cat = 2; v = p0 << 16 | k0 << 12 | k1 << 8 | k2 << 4; }
    else { cat = 1; v = k0 << 16 | k1 << 12 | k2 << 8 | k3 << 4 | k4; }
    return cat << 20 | v;
}

__device__ inline uint32_t holdem_rank7(uint64_t cnt, uint64_t smp)
{
#if CS_PROF_NO_EVAL   // profiling builds only: wrong showdowns, timing of the evaluator
    return (uint32_t)(cnt ^ (cnt >> 32) ^ smp ^ (smp >> 29)) & 0xFFFFFFu;
#endif
    (void)cnt;
    return holdem_rank7_bf(smp);
}

// The nine dealt draws (random_interval(i), i = 51..43, mask 63) from the staged bytes without rejection loops or a
// 24-step dependency chain. For i = 51..43 a byte u = b & 63 is accepted for every i if u <= 42, for none if u >= 52;
// only u in 43..51 ("maybe", 9/64 of the bytes) depends on i = 51 - (acceptances before it). SWAR per dword gives the
// sure-accept and maybe masks of the next 24 staged bytes; the maybes are then resolved in order (a few per lane) from
// the popcount of the acceptances before each. Same bytes, same draws. false: fewer than 28 staged bytes, or fewer
// than nine acceptances among the 24 (the caller draws with interval(), same numbers).
template <class Rng>
__device__ __forceinline__ bool deal9_swar(Rng& rng, uint32_t (&j)[9])
{
    const uint32_t k0 = rng.staged_offset();
    if (k0 >= rng.sn || rng.sn - k0 < 28u) return false;
    const uint32_t* row = (const uint32_t*)(rng.stg + (k0 & ~3u));
    const uint32_t sh = k0 & 3u;
    uint32_t w[7];
#pragma unroll
    for (int q = 0; q < 7; q++) w[q] = row[q];
    uint32_t acc = 0, may = 0;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const uint32_t x = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) & 0x3F3F3F3Fu;   // bytes k0 + 4q .., & 63
        const uint32_t ge43 = (x + 0x55555555u) & 0x80808080u, ge52 = (x + 0x4C4C4C4Cu) & 0x80808080u;
        const uint32_t a = (~ge43 & 0x80808080u) >> 7, m = (ge43 & ~ge52) >> 7;
        // byte flags (bits 0, 8, 16, 24) -> 4-bit mask: the product's top nibble
        acc |= ((a * 0x10204080u) >> 28) << (4 * q);
        may |= ((m * 0x10204080u) >> 28) << (4 * q);
    }
    while (may) {
        const uint32_t t = __builtin_ctz(may);
        may &= may - 1u;
        const uint32_t cnt = __popc(acc & ((1u << t) - 1u));
        if (cnt >= 9u) break;                    // past the ninth draw: not consumed
        const uint32_t u = rng.stg[k0 + t] & 63u;   // the staged byte again (LDS), not a select over x[]
        acc |= u <= 51u - cnt ? 1u << t : 0u;
    }
    if (__popc(acc) < 9) return false;
    uint32_t p = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        p = __builtin_ctz(acc);
        acc &= acc - 1u;
        j[k] = rng.stg[k0 + p] & 63u;
    }
    rng.advance_by(p + 1u);
    return true;
}

// The hold'em deal (limitholdem/dealer.py: shuffle the 52-card deck, deal_card = pop()) of a heads-up game: hole i ->
// player i % 2, card i / 2 from deck[51 - i]; flop deck[47..45], turn deck[44], river deck[43]. Fisher-Yates fixes
// position i at step i, and only deck[43..51] is ever dealt, so the first nine swaps are tracked and the other 42 only
// consume their draws. Out: holes packed p0c0 | p0c1 << 6 | p1c0 << 12 | p1c1 << 18, board c0..c4 6 bits each.
// Registers only (the rollout kernels' occupancy is register-bound).
template <class Rng>
__device__ __forceinline__ void holdem_deal2(Rng& rng, uint32_t& holes, uint32_t& board)
{
    uint32_t js[9];
    bool staged = false;
#if CS_PROF_NO_DEAL9   // profiling builds only: wrong deals, timing of the tracked draws
#pragma unroll
    for (int k = 0; k < 9; k++) js[k] = (uint32_t)k;
    rng.advance_by(12u);
    staged = true;
#else
    if constexpr (Rng::kMode == STAGE_LDS) staged = deal9_swar(rng, js);
#endif
    if (!staged) {
#pragma unroll
        for (int k = 0; k < 9; k++) js[k] = rng.interval_loop(51u - (uint32_t)k);
    }
    uint32_t d0 = 0, d1 = 0;
#if !CS_PROF_NO_TRACK
    // Dealt card k is the card at position 51 - k after the nine swaps (later swaps never touch positions >= 43): the
    // nine positions, four per word (bytes; 63 = unused, never matches), are traced back through the swaps q = 8 .. 0
    // -- a byte x in {i_q, j_q} flips by i_q ^ j_q; bytes < 64, so (b + 0x7F) sets bit 7 exactly when b != 0 -- and end
    // at their initial positions = the card ids. Six live words instead of the JV table's ~40 registers.
    uint32_t X[3] = {0x30313233u, 0x2C2D2E2Fu, 0x3F3F3F2Bu};   // byte b of X[w]: position 51 - (4 w + b)
#pragma unroll
    for (int q = 8; q >= 0; q--) {
        const uint32_t I = (uint32_t)(51 - q) * 0x01010101u;
        const uint32_t J = __builtin_amdgcn_perm(0u, js[q], 0u);   // byte 0 of js[q] in every byte
        const uint32_t D = I ^ J;
#pragma unroll
        for (int w = 0; w < 3; w++) {
            if (q > 4 * w + 3) continue;   // swap q never touches positions 51 - k, k < q (both of its are <= 51 - q)
            const uint32_t both = ((X[w] ^ I) + 0x7F7F7F7Fu) & ((X[w] ^ J) + 0x7F7F7F7Fu);
            const uint32_t m = ~both & 0x80808080u;
            X[w] ^= D & (m - (m >> 7));
        }
    }
    {
        constexpr int F0[4] = {0, 12, 6, 18};   // hole i -> player i % 2, card i / 2
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const uint32_t v = (X[k >> 2] >> (8 * (k & 3))) & 63u;
            if (k < 4) d0 |= v << F0[k < 4 ? k : 0];
            else d1 |= v << (6 * (k - 4));
        }
    }
#else   // profiling builds only (cs_prof.h): the draws as the cards
#pragma unroll
    for (int k = 0; k < 9; k++) {
        if (k < 4) d0 |= js[k] << (6 * k);
        else d1 |= js[k] << (6 * (k - 4));
    }
#endif
#if CS_PROF_NO_SKIP   // profiling builds only: wrong streams, timing of the skip scan
    rng.advance_by(60u);
#else
    rng.skip_intervals(42u);   // deck positions 42..1 are never dealt: only the words they consume matter
#endif
    holes = d0;
    board = d1;
}

// the showdown of a heads-up deal when both players stay in (Judger.judge_game -> compare_hands, judger.py:11-108,
// utils.py): bit 0 = player 0 wins or ties, bit 1 = player 1. It depends on the deal alone: no-limit evaluates it when
// the deal is drawn (in the rollout's lockstep deal passes) and keeps it in the state; limit at the game's end.
__device__ __forceinline__ uint32_t holdem_showdown(uint32_t holes, uint32_t board)
{
    uint64_t bc = 0, bs = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) tally_card((int)((board >> (6 * k)) & 63u), bc, bs);
    uint64_t c0 = bc, s0 = bs, c1 = bc, s1 = bs;
    tally_card((int)(holes & 63u), c0, s0);
    tally_card((int)((holes >> 6) & 63u), c0, s0);
    tally_card((int)((holes >> 12) & 63u), c1, s1);
    tally_card((int)((holes >> 18) & 63u), c1, s1);
    uint32_t v0 = holdem_rank7(c0, s0);
    // the second evaluation's inputs pass through an empty asm with the first result: the two branch-free evaluations
    // run one after the other instead of interleaved (half the live temporaries: occupancy, no spills)
    uint32_t s1lo = (uint32_t)s1, s1hi = (uint32_t)(s1 >> 32);
    asm volatile("" : "+v"(v0), "+v"(s1lo), "+v"(s1hi));
    s1 = (uint64_t)s1hi << 32 | s1lo;
    const uint32_t v1 = holdem_rank7(c1, s1);
    return (uint32_t)(v0 >= v1) | (uint32_t)(v1 >= v0) << 1;
}

// Deal queue (hold'em games): a hold'em deal depends only on the env's MT stream, never on the actions, so the
// rollout draws deals ahead -- one pass of all lanes with room in their queue, in lockstep, whenever a lane ends a
// game with its queue empty -- instead of a pass at every step in which any lane of the wave resets (a 32-env wave
// has a reset almost every step, with ~2/5 of its lanes active). Same deals in the same stream order, so outputs are
// unchanged. The queue lives after the game's words in the env state: a header (count:CB, head:CB-1, no-limit dealer
// drawn << XB, dealer << XB + 1, draws[8:7] of slot k << XB + 2 + 2 k; CB = log2(DQ) + 1, XB = 2 CB - 1: DQ 4 -> 3, 5;
// DQ 8 -> 4, 7) and DQ entries of two words (e0 = holes | seat bit << 24 | draws[6:0] << 25, e1 = board | showdown
// << 30; draws = MT words the deal consumed, for the host's stream position, saturating at 511).
// Depth 8 vs 4 (LDS queue): 0.39 vs 0.46 deal passes per wave-step (simulated), the pass costs ~1 200
// wave-instructions; with 4 waves per SIMD instead of 5: Limit -2.5 %, No-limit -0.7 %.
constexpr int HOLDEM_DQ = 8;
constexpr int HOLDEM_DQ_WORDS = HOLDEM_DQ > 0 ? 1 + 2 * HOLDEM_DQ : 0;
constexpr int DQ_CB = HOLDEM_DQ == 8 ? 4 : HOLDEM_DQ == 4 ? 3 : 2;   // count bits (0..DQ)
constexpr int DQ_XB = 2 * DQ_CB - 1;                                // first bit after count and head
static_assert(DQ_XB + 2 + 2 * HOLDEM_DQ <= 32, "deal queue header fits a word");

struct Limit {
    static constexpr int GW = 4;                        // game words; the deal queue follows
    static constexpr int DQ = HOLDEM_DQ;
    static constexpr int OBS = 72, A = 4, P = 2, LB = 1, WORDS = GW + HOLDEM_DQ_WORDS, ACTION_BYTES = 1;
    static constexpr int NB = 3;
    static constexpr bool RING = true;          // MT stream as the byte ring (cs_ring.h)
    static constexpr bool RAW_OBS = false;
    static constexpr int SCRATCH_WORDS = 0;
    // MT staging (see MtLaneT)
    static constexpr int STAGE_MODE = STAGE_LDS, STAGE_W = 128, STAGE_PAD = 8, STAGE_R = 100;
    static constexpr int STAGE_RF = 120;  // batch restage threshold (ring_restage_wave): 2.70 -> 2.65 ms per 128 steps
    static constexpr int RESTAGE_B = 8;   // lanes restaged per pass (loads in flight)
    static constexpr int MIN_WAVES = 4;   // 4 waves/SIMD (LDS-bound with the 8-deal queue; at a 4-deal queue 5 beat 4
                                          // and 6, which spilled 40 VGPRs)
    static constexpr int EPW = 32;   // rollout envs per wave: 262 144 envs need half-full waves (lane_ctx)
    static constexpr bool LANE_OPAQUE = false;   // k_rollout: lane id not made opaque per step (cs_skeleton.h LaneOpaque)
    static constexpr int REFILL_K = 2;   // stale blocks twisted per pass (see mt_refill_wave)
    __device__ __forceinline__ void bind(uint32_t*, const GameParams&) {}
    enum { CALL = 0, RAISE = 1, FOLD = 2, CHECK = 3 };

    uint32_t w0, w1, w2, w3;

    // field accessors on the packed words (kept packed in registers: few live values, cheap bitfield ops)
    __device__ __forceinline__ int hole(int p, int k) const { return (w0 >> (6 * (2 * p + k))) & 63; }
    __device__ __forceinline__ int board(int k) const { return (w1 >> (6 * k)) & 63; }
    __device__ __forceinline__ int in0() const { return (w0 >> 24) & 63; }
    __device__ __forceinline__ int in1() const { return w2 & 63; }
    __device__ __forceinline__ int r0() const { return (w2 >> 6) & 31; }
    __device__ __forceinline__ int r1() const { return (w2 >> 11) & 31; }
    __device__ __forceinline__ int hr() const { return (w2 >> 16) & 7; }
    __device__ __forceinline__ int nrn() const { return (w2 >> 19) & 3; }
    __device__ __forceinline__ int rc() const { return (w2 >> 21) & 7; }
    __device__ __forceinline__ int f0() const { return (w2 >> 24) & 1; }
    __device__ __forceinline__ int f1() const { return (w2 >> 25) & 1; }
    __device__ __forceinline__ int use_prev() const { return (w2 >> 26) & 1; }
    __device__ __forceinline__ int ptr() const { return (w0 >> 30) & 1; }

    __device__ __forceinline__ void load(const uint32_t* st, int64_t n, int64_t env)
    {
        w0 = st[env]; w1 = st[n + env]; w2 = st[2 * n + env]; w3 = st[3 * n + env];
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t n, int64_t env) const
    {
        st[env] = w0; st[n + env] = w1; st[2 * n + env] = w2; st[3 * n + env] = w3;
    }
    __device__ __forceinline__ void blank() { w0 = 1u << 31; w1 = 0; w2 = 0; w3 = 0; }

    __device__ __forceinline__ int current() const { return ptr(); }
    __device__ __forceinline__ bool is_over() const { return (w0 >> 31) != 0; }

    __device__ __forceinline__ uint32_t legal() const
    {
        const int a = r0(), b = r1(), mx = a > b ? a : b, rp = ptr() ? b : a;
        uint32_t m = 0xF;
        if (hr() >= 4) m &= ~(1u << RAISE);
        if (rp < mx) m &= ~(1u << CHECK);
        if (rp == mx) m &= ~(1u << CALL);
        return m;
    }

    // the cards as a 64-bit mask (ids < 52), the four raise one-hots as a 20-bit field at obs bit 52
    __device__ __forceinline__ void observe(int player, uint32_t (&bits)[NB]) const
    {
        const int r = rc(), npub = r == 0 ? 0 : (r == 1 ? 3 : (r == 2 ? 4 : 5));
        uint64_t cm = 1ull << hole(player, 0) | 1ull << hole(player, 1);
#pragma unroll
        for (int k = 0; k < 5; k++) cm |= (uint64_t)(k < npub) << board(k);
        const uint32_t rn = use_prev() ? (w3 >> 12) : w3;
        uint32_t R = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) R |= 1u << (5 * i + (int)((rn >> (3 * i)) & 7u));
        bits[0] = (uint32_t)cm;
        bits[1] = (uint32_t)(cm >> 32) | R << 20;
        bits[2] = R >> 12;
    }

    // the same row as the byte positions of its 11 ones (row_write_sparse): the two holes, the five board cards (not
    // yet public: the first hole again), obs byte 52 + 5 i + raise count of round i (i = 0..3)
    static constexpr int SPARSE_K = 11;
    __device__ __forceinline__ uint32_t observe_pos(int player, uint32_t (&pos)[11]) const
    {
        const int r = rc(), npub = r == 0 ? 0 : (r == 1 ? 3 : (r == 2 ? 4 : 5));
        const uint32_t c0 = (uint32_t)hole(player, 0);
        pos[0] = c0;
        pos[1] = (uint32_t)hole(player, 1);
#pragma unroll
        for (int k = 0; k < 5; k++) pos[2 + k] = k < npub ? (uint32_t)board(k) : c0;
        const uint32_t rn = use_prev() ? (w3 >> 12) : w3;
#pragma unroll
        for (int i = 0; i < 4; i++) pos[7 + i] = 52u + 5u * (uint32_t)i + ((rn >> (3 * i)) & 7u);
        return 0;
    }

    // the deal of init_game (game.py:46-95): shuffle + holes + board, then the small blind seat randint(0, 2)
    template <class Rng>
    __device__ __forceinline__ void make_deal(Rng& rng, uint32_t&, uint32_t& e0, uint32_t& e1) const
    {
        uint32_t d0, d1;
        holdem_deal2(rng, d0, d1);
        e0 = d0 | rng.interval(1u) << 24;
        e1 = d1;   // showdown at the game's end: evaluated with the deal it measured slower here (no-limit: faster)
    }
    template <class Rng>
    __device__ __forceinline__ void reset(Rng& rng)
    {
        uint32_t hdr = 0, e0, e1;
        make_deal(rng, hdr, e0, e1);
        reset_from(e0, e1);
    }
    __device__ __forceinline__ void reset_from(uint32_t e0, uint32_t e1)
    {
        const uint32_t d0 = e0 & 0xFFFFFFu, d1 = e1;
        const int s = (int)((e0 >> 24) & 1u);
        const int in_0 = s == 0 ? 1 : 2, in_1 = s == 0 ? 2 : 1;
        const int first = s;  // (BB + 1) % 2 with BB = (s + 1) % 2
        w0 = d0 | (uint32_t)in_0 << 24 | (uint32_t)first << 30;
        w1 = d1;
        w2 = (uint32_t)in_1 | (uint32_t)in_0 << 6 | (uint32_t)in_1 << 11 | 1u << 26;  // raised = in_chips, use_prev
        w3 = (w3 & 0xFFFu) << 12;                                                      // prev <- current, current <- 0
    }

    template <class Rng>
    __device__ __forceinline__ void step(int a, Rng&)
    {
        const uint32_t lg = legal();
        if (a < 0 || a > 3 || !((lg >> a) & 1u)) a = ((lg >> CHECK) & 1u) ? CHECK : FOLD;
        int i0 = in0(), i1 = in1(), ra0 = r0(), ra1 = r1(), h = hr(), nr = nrn(), r = rc(), p = ptr();
        int fo0 = f0(), fo1 = f1();
        const int mx = ra0 > ra1 ? ra0 : ra1, rp = p ? ra1 : ra0, amt = r >= 2 ? 4 : 2;
        int add = 0, nraised = rp;
        if (a == CALL) { add = mx - rp; nraised = mx; nr += 1; }
        else if (a == RAISE) { add = mx - rp + amt; nraised = mx + amt; h += 1; nr = 1; }
        else if (a == FOLD) { if (p) fo1 = 1; else fo0 = 1; }
        else { nr += 1; }
        if (p) { i1 += add; ra1 = nraised; } else { i0 += add; ra0 = nraised; }
        p ^= 1;
        if (p ? fo1 : fo0) p ^= 1;
        w3 = (w3 & ~(7u << (3 * r))) | ((uint32_t)h << (3 * r));   // history_raise_nums[round] = have_raised
        if (nr >= 2) {
            r += 1;
            h = 0; nr = 0; ra0 = 0; ra1 = 0;
        }
        const int over = (fo0 + fo1 == 1) || r >= 4;
        w0 = (w0 & 0x00FFFFFFu) | (uint32_t)i0 << 24 | (uint32_t)p << 30 | (uint32_t)over << 31;
        w2 = (uint32_t)i1 | (uint32_t)ra0 << 6 | (uint32_t)ra1 << 11 | (uint32_t)h << 16 | (uint32_t)nr << 19 |
             (uint32_t)r << 21 | (uint32_t)fo0 << 24 | (uint32_t)fo1 << 25;   // use_prev cleared
    }

    __device__ __forceinline__ void payoffs(float (&out)[P]) const
    {
        int win0, win1;
        if (f0() || f1()) {
            win0 = !f0(); win1 = !f1();
        } else {
            const uint32_t sd = holdem_showdown(w0 & 0xFFFFFFu, w1);
            win0 = (int)(sd & 1u);
            win1 = (int)(sd >> 1);
        }
        const int a = in0(), b = in1(), m = a < b ? a : b;
        float p0 = 0.f, p1 = 0.f;
        if (!(win0 && win1)) {
            p0 = win0 ? (float)m : -(float)m;
            p1 = -p0;
        }
        out[0] = p0 * 0.5f;
        out[1] = p1 * 0.5f;
    }
};

}  // namespace cs
