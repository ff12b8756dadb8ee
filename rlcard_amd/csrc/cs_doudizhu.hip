// cs_doudizhu.hip -- DouDizhu lockstep kernels for gfx950: ONE WAVE PER ENV.
//
// Per step a wave
//   1. builds the 27 472-bit legal mask in LDS (Judger.playable_cards_from_hand / get_gt_cards,
//      rlcard/games/doudizhu/judger.py:124-331, utils.py:517-621): the legal set of a hand is every table combo the
//      hand contains (leading), or pass + same-type greater-weight combos + bombs + rocket (following). Three passes,
//      all 64 lanes wide:
//        a. the 308 (type, weight) groups: does the hand contain the group's elementwise-min combo (and may the group
//           be played now)? -> ballot + prefix counts in LDS;
//        b. the 859 mask dwords: does any of the groups overlapping the dword pass? (two LDS reads per dword);
//        c. the few dwords that survive (about 6 for a 17-card hand): 32 lanes test one id each against the hand
//           (SWAR containment on packed nibble counts), ballot = the mask dword.
//   2. builds the obs row (envs/doudizhu.py:26-134) as a bit vector in LDS: 54-bit card blocks (_cards2array is a
//      thermometer code of every rank nibble, computed with four SWAR adds), the one-hot hand sizes;
//   3. writes both rows with 16-B stores at whatever alignment the row has (boundary chunks byte by byte);
//   4. (rollout) picks the policy action: uniform over the legal ids from Philox(seed, env, t) -- the k-th set bit
//      found with a wave prefix scan over the surviving dwords;
//   5. applies the action with wave-uniform (scalar) updates of the packed state (round.py:67-79, game.py:55-81).
// The deal (dealer.py:12-76: one 54-card np.random shuffle) runs the Fisher-Yates loop with the deck held one card
// per lane and the MT19937 words loaded 64 at a time (coalesced) and consumed with readlane.
// Output bytes per env-step: 901 obs + 3 434 legal + 12 reward + 4 -- HBM-bound by design.
#include "cs_device.h"
#include "cs_engine.h"
#include "cs_doudizhu.h"

namespace cs {
namespace ddz {

constexpr int BLOCK = 256;                        // the one-env kernels (reset / step / observe / debug)
constexpr int WPB = BLOCK / WAVE;
constexpr int MASK_PAD = 4;                       // zero dwords on both sides of the mask image
constexpr int KTH_LANES = 54, KTH_WORDS = 16;     // kth_legal: lane l scans mask dwords [16 l, 16 l + 16)
constexpr int MASK_WORDS = MASK_PAD + KTH_LANES * KTH_WORDS + MASK_PAD;
constexpr int NSEG = 20;                          // 54-bit obs blocks (16 used) + zero tail
constexpr int BV_WORDS = 32;                      // obs bits (912 + 16 front pad) as dwords

constexpr int LIST_RING = 128;                    // the step's tested mask dwords (a ring: see build_legal)
constexpr int LIST_CAP = 64;                      // kth_legal reads the list when it holds them all, one per lane
struct alignas(16) WaveLds {
    uint32_t mask[MASK_WORDS];   // legal bits: id i at bit (i & 31) of mask[MASK_PAD + i / 32]
    uint64_t segv[NSEG];         // obs 54-bit blocks
    uint32_t bv[BV_WORDS];       // obs bit x at bit 16 + x
    uint16_t pre[MAX_GROUPS + 8];
    uint16_t lst[LIST_RING];     // the mask dwords pass c tests this step, ascending (Legal::nl of them)
};

// the group table and the per-dword group ranges, copied once per block (read by every step's scan)
struct TabLds {
    uint4 grp[MAX_GROUPS];
    uint32_t drange[ND + 1];
};

__device__ __forceinline__ void load_tab(TabLds& T, const Tab& tb)
{
    const uint4* g = (const uint4*)tb.grp;
    for (int i = threadIdx.x; i < tb.ng; i += blockDim.x) T.grp[i] = g[i];
    for (int i = threadIdx.x; i < ND; i += blockDim.x) T.drange[i] = tb.drange[i];
    __syncthreads();
}

__device__ __forceinline__ uint32_t rl(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int k)
{
    return (uint64_t)rl((uint32_t)v, k) | ((uint64_t)rl((uint32_t)(v >> 32), k) << 32);
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t b)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
__device__ __forceinline__ bool contains(uint64_t hand, uint64_t combo)
{
    return (((hand | NIB_HI) - combo) & NIB_HI) == NIB_HI;
}
__device__ __forceinline__ uint32_t num_cards(uint64_t c)
{
    const uint64_t b = (c & 0x0F0F0F0F0F0F0F0Full) + ((c >> 4) & 0x0F0F0F0F0F0F0F0Full);
    return (uint32_t)((b * 0x0101010101010101ull) >> 56);
}

// x if c else 0, written so that a choice between fields of a local struct stays a register operation (a plain
// `c ? s.a : s.b` is folded into a load from a computed field address, which sends the whole struct to scratch)
__device__ __forceinline__ uint64_t keep64(bool c, uint64_t x) { return x & (0ull - (uint64_t)c); }
__device__ __forceinline__ uint32_t keep32(bool c, uint32_t x) { return x & (0u - (uint32_t)c); }

// ---- wave-uniform env state -------------------------------------------------------------------------------------
struct Env {
    uint64_t h0, h1, h2;        // hands
    uint64_t q0, q1, q2;        // played
    // the last 9 trace ids, oldest first, two per word (id k at bits 16 * (k & 1) of word k / 2; the high half of
    // hw4 is unused). Separate scalars, not an array: a lane-indexed pick from an array sends it to scratch.
    uint32_t hw0, hw1, hw2, hw3, hw4;
    uint32_t ntrace, greater, gplay, cur, winner;
    uint32_t ggrp;              // (type, weight) group of gplay (kept in the spare high half of state word 16)
    uint64_t hcnt;              // PER LANE: lane s = 3..11 holds the packed counts of hist(s - 3) (0: pass / none),
                                // shifted down one lane per action, so observations never reload the action table
    uint32_t deck;              // PER LANE: lane k < 54 holds the card dealt at shuffled position k (state W_DECK)

    __device__ __forceinline__ uint32_t hist(uint32_t k) const   // k may differ per lane
    {
        const uint32_t j = k >> 1;
        const uint32_t w = keep32(j == 0, hw0) | keep32(j == 1, hw1) | keep32(j == 2, hw2) | keep32(j == 3, hw3) |
                           keep32(j == 4, hw4);
        return (w >> (16 * (k & 1))) & 0xFFFFu;
    }

    __device__ __forceinline__ uint64_t hand(uint32_t p) const
    {
        return keep64(p == 0, h0) | keep64(p == 1, h1) | keep64(p == 2, h2);
    }
    __device__ __forceinline__ uint64_t played(uint32_t p) const
    {
        return keep64(p == 0, q0) | keep64(p == 1, q1) | keep64(p == 2, q2);
    }
    __device__ __forceinline__ bool over() const { return winner != NONE; }

    __device__ __forceinline__ void load(const uint32_t* st, int64_t env, int lane, const Tab& tb)
    {
        const uint32_t w = lane < WORDS ? st[env * WORDS + lane] : 0u;
        h0 = (uint64_t)rl(w, 0) | ((uint64_t)rl(w, 1) << 32);
        h1 = (uint64_t)rl(w, 2) | ((uint64_t)rl(w, 3) << 32);
        h2 = (uint64_t)rl(w, 4) | ((uint64_t)rl(w, 5) << 32);
        q0 = (uint64_t)rl(w, 6) | ((uint64_t)rl(w, 7) << 32);
        q1 = (uint64_t)rl(w, 8) | ((uint64_t)rl(w, 9) << 32);
        q2 = (uint64_t)rl(w, 10) | ((uint64_t)rl(w, 11) << 32);
        hw0 = rl(w, W_HIST);
        hw1 = rl(w, W_HIST + 1);
        hw2 = rl(w, W_HIST + 2);
        hw3 = rl(w, W_HIST + 3);
        const uint32_t w16 = rl(w, W_HIST + 4);
        hw4 = w16 | (NO_ACTION << 16);
        ggrp = w16 >> 16;
        const uint32_t id = lane >= 3 && lane <= 11 ? hist((uint32_t)(lane - 3)) : NO_ACTION;
        hcnt = id < (uint32_t)PASS ? tb.cnt[id] : 0ull;
        ntrace = rl(w, W_NTRACE);
        const uint32_t g = rl(w, W_GREATER), c = rl(w, W_CUR);
        greater = g & 0xFFFFu;
        gplay = g >> 16;
        cur = c & 0xFFu;
        winner = (c >> 8) & 0xFFu;
        deck = lane < 54 ? (uint32_t)((const uint8_t*)(st + env * WORDS + W_DECK))[lane] : 0u;
    }
    __device__ __forceinline__ void store(uint32_t* st, int64_t env, int lane) const
    {
        if (lane == 0) {
            uint4* o = (uint4*)(st + env * WORDS);   // 80-B rows: 16-B aligned
            o[0] = make_uint4((uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32));
            o[1] = make_uint4((uint32_t)h2, (uint32_t)(h2 >> 32), (uint32_t)q0, (uint32_t)(q0 >> 32));
            o[2] = make_uint4((uint32_t)q1, (uint32_t)(q1 >> 32), (uint32_t)q2, (uint32_t)(q2 >> 32));
            o[3] = make_uint4(hw0, hw1, hw2, hw3);
            o[4] = make_uint4((hw4 & 0xFFFFu) | (ggrp << 16), ntrace, greater | (gplay << 16), cur | (winner << 8));
        }
        ((uint8_t*)(st + env * WORDS + W_DECK))[lane] = (uint8_t)(lane < 54 ? deck : 0u);   // one 64-B segment
    }

    // Player.play + Round.proceed_round + Game.step (player.py:88-108, round.py:54-79, game.py:55-81)
    __device__ __forceinline__ void apply(uint32_t a, const Tab& tb, int lane)
    {
        apply_with(a, a != (uint32_t)PASS ? tb.cnt[a] : 0ull, a != (uint32_t)PASS ? (uint32_t)tb.gid[a] : 0u, lane);
    }
    // the same with the action's table entries (packed counts, group) already loaded
    __device__ __forceinline__ void apply_with(uint32_t a, uint64_t c, uint32_t gid, int lane)
    {
        const uint32_t p = cur;
        const uint64_t down = (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)hcnt, 1) |
                              ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(hcnt >> 32), 1) << 32);
        hcnt = lane == 11 ? c : (lane >= 3 && lane < 11 ? down : 0ull);
        hw0 = (hw0 >> 16) | (hw1 << 16);
        hw1 = (hw1 >> 16) | (hw2 << 16);
        hw2 = (hw2 >> 16) | (hw3 << 16);
        hw3 = (hw3 >> 16) | (hw4 << 16);
        hw4 = a | (NO_ACTION << 16);
        ntrace++;
        if (a != (uint32_t)PASS) {
            ggrp = gid;
            const uint64_t c0 = keep64(p == 0, c), c1 = keep64(p == 1, c), c2 = keep64(p == 2, c);
            h0 -= c0; h1 -= c1; h2 -= c2;
            q0 += c0; q1 += c1; q2 += c2;
            const uint64_t left = hand(p);
            greater = p;
            gplay = a;
            if (left == 0) winner = p;
        }
        cur = p == 2 ? 0u : p + 1;
    }
};

// the ids a player may play now: leading -> every combo; following -> [c_lo, c_lo + c_len) (same type, greater
// weight), the bombs unless the last play is a bomb, the rocket; nothing after a rocket (utils.py:590-621)
struct Cand {
    uint32_t c_lo, c_len, b_lo, b_len, r_lo, r_len;
    bool leading;
    __device__ __forceinline__ bool ok(uint32_t x) const
    {
        return (x - c_lo < c_len) | (x - b_lo < b_len) | (x - r_lo < r_len);
    }
    // does any candidate range meet the ids [lo, hi)?
    __device__ __forceinline__ bool meets(uint32_t lo, uint32_t hi) const
    {
        return (c_len && c_lo < hi && c_lo + c_len > lo) | (b_len && b_lo < hi && b_lo + b_len > lo) |
               (r_len && r_lo < hi && r_lo + r_len > lo);
    }
};
__device__ __forceinline__ Cand cand_at(uint32_t greater, uint32_t cur, uint32_t ggrp, const Tab& tb, const TabLds& T)
{
    Cand c;
    c.leading = greater == NONE || greater == cur;   // player.py:60-86 available_actions
    if (c.leading) {
        c.c_lo = 0; c.c_len = PASS; c.b_lo = 0; c.b_len = 0; c.r_lo = 0; c.r_len = 0;
        return c;
    }
    const uint4 q = T.grp[ggrp];
    const uint32_t z = q.z, y = q.w;
    const uint32_t gend = z >> 16, tend = y & 0xFFFFu, type = (y >> 16) & 0xFFu;
    if (type == (uint32_t)TYPE_ROCKET) {
        c.c_lo = 0; c.c_len = 0; c.b_lo = 0; c.b_len = 0; c.r_lo = 0; c.r_len = 0;
        return c;
    }
    c.c_lo = gend;
    c.c_len = tend - gend;
    c.b_lo = (uint32_t)tb.bomb_lo;
    c.b_len = type == (uint32_t)TYPE_BOMB ? 0u : (uint32_t)(tb.bomb_hi - tb.bomb_lo);
    c.r_lo = (uint32_t)tb.rocket;
    c.r_len = 1;
    return c;
}
__device__ __forceinline__ Cand cand_of(const Env& e, const Tab& tb, const TabLds& T)
{
    return cand_at(e.greater, e.cur, e.ggrp, tb, T);
}

// single-id legality + the fallback for an id outside the legal set (cs_step only; the reference has no decode
// fallback for doudizhu -- an illegal id corrupts its hands -- so the ABI defines one: lowest solo when leading,
// pass when following)
__device__ __forceinline__ uint32_t decode_action(int32_t a, const Env& e, const Cand& c, const Tab& tb)
{
    const uint64_t h = e.hand(e.cur);
    bool ok;
    if (a < 0 || a >= NA) ok = false;
    else if (a == PASS) ok = !c.leading;
    else ok = contains(h, tb.cnt[a]) && c.ok((uint32_t)a);
    if (ok) return (uint32_t)a;
    if (!c.leading) return (uint32_t)PASS;
    const uint64_t nz = (h | (h >> 1) | (h >> 2)) & 0x0111111111111111ull;
    return (uint32_t)(__builtin_ctzll(nz) >> 2);   // solo id = rank (checked by the table builder)
}

// ---- MT19937 stream of this env, read by the whole wave --------------------------------------------------------
// Philox mode (cs_config.rng_mode = CS_RNG_PHILOX, ctl bit 18; not the reference's deals): draw k is byte k % 16 of
// Philox4x32-10(key = the env's init_by_array key, counter = (k / 624, (k % 624) / 16)) -- the lane-per-env games'
// Philox byte stream (cs_ring.h), so every rule and the oracle's restatement (oracle/or_rng.c) are shared. The draws
// only use the low 6 bits (interval(i <= 53)). The env's word buffer then holds the key (words 0, 1) and the absolute
// draw count (word 2); `pos` still counts draws modulo 1 248 (the host's rng_position).
// The mode is a template parameter (the kernels are instantiated for both), so the MT19937 path carries no Philox code.
constexpr uint32_t CTL_PHX = 1u << 18;
template <bool PHX>
struct WaveMt {
    uint32_t* base;
    uint32_t pos, stale;
    uint32_t dabs;   // Philox mode: the absolute draw count
    uint64_t key;
    // 64 tempered words from pos (lane k: word pos + k); twists the next block first if the window reaches it or
    // ends exactly at its start: advance() never moves past the window, so a later crossing into the next block
    // always finds it twisted (with `>` a window ending on the block edge left the next block stale -- the first
    // deal after such a crossing read the block consumed 1 248 draws earlier; tests/test_gpu_refill.py)
    __device__ __forceinline__ uint32_t window(int lane)
    {
        if constexpr (PHX) {
            const uint32_t k = dabs + (uint32_t)lane, b = k % 16u;
            uint32_t w[4];
            philox4(key, (uint64_t)(k / (uint32_t)MT_N), (uint64_t)((k % (uint32_t)MT_N) / 16u), w);
            const uint32_t q = b >> 2, word = q == 0 ? w[0] : (q == 1 ? w[1] : (q == 2 ? w[2] : w[3]));
            return (word >> (8u * (b & 3u))) & 255u;
        }
        const uint32_t end = pos < (uint32_t)MT_N ? (uint32_t)MT_N : (uint32_t)MT_WORDS;
        if (stale && pos + WAVE >= end) {
            const uint32_t cur = pos < (uint32_t)MT_N ? 0u : (uint32_t)MT_N;
            mt_twist_wave(base + cur, base + (MT_N - cur), lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            stale = 0;
        }
        uint32_t idx = pos + (uint32_t)lane;
        if (idx >= (uint32_t)MT_WORDS) idx -= MT_WORDS;
        return mt_temper(base[idx]);
    }
    __device__ __forceinline__ void advance(uint32_t k)
    {
        if constexpr (PHX) dabs += k;
        uint32_t np = pos + k;
        const bool crossed = pos < (uint32_t)MT_N ? np >= (uint32_t)MT_N : np >= (uint32_t)MT_WORDS;
        if (np >= (uint32_t)MT_WORDS) np -= MT_WORDS;
        if (crossed) stale = 1;
        pos = np;
    }
    // the stream position back to ctl (and the Philox draw count to the word buffer); one lane
    __device__ __forceinline__ void save(uint32_t* ctl, int64_t env) const
    {
        ctl[env] = pos | (stale << 16) | (PHX ? CTL_PHX : 0u);
        if constexpr (PHX) base[2] = dabs;
    }
};

// Dealer.shuffle + deal_cards + landlord's 3 cards (dealer.py:12-76; game.py:23-53): np.random.shuffle of the
// sorted 54-card deck (position k holds rank k / 4, 52 = black joker, 53 = red joker), hands deck[0:17] (landlord),
// [17:34], [34:51], landlord + deck[51:54]
template <class M>
__device__ __forceinline__ void deal(Env& e, M& m, int lane)
{
    uint32_t deck = (uint32_t)lane;
    uint32_t win = m.window(lane);
    uint32_t wi = 0;
    for (int i = 53; i >= 1; i--) {
        uint32_t mask = (uint32_t)i;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        uint32_t u;
        do {
            if (wi == (uint32_t)WAVE) {
                m.advance(WAVE);
                win = m.window(lane);
                wi = 0;
            }
            u = rl(win, (int)wi) & mask;
            wi++;
        } while (u > (uint32_t)i);
        const uint32_t vi = rl(deck, i), vu = rl(deck, (int)u);
        deck = lane == i ? vu : (lane == (int)u ? vi : deck);
    }
    m.advance(wi);
    const uint32_t rank = deck < 52u ? deck >> 2 : deck - 39u;
    const uint64_t own0 = 0x003800000001FFFFull, own1 = 0x00000003FFFE0000ull, own2 = 0x0007FFFC00000000ull;
    uint64_t h0 = 0, h1 = 0, h2 = 0;
#pragma unroll
    for (int r = 0; r < 15; r++) {
        const uint64_t b = __ballot(lane < 54 && rank == (uint32_t)r);
        h0 |= (uint64_t)__popcll(b & own0) << (4 * r);
        h1 |= (uint64_t)__popcll(b & own1) << (4 * r);
        h2 |= (uint64_t)__popcll(b & own2) << (4 * r);
    }
    e.h0 = h0; e.h1 = h1; e.h2 = h2;
    e.deck = deck;
    e.q0 = e.q1 = e.q2 = 0;
    e.hw0 = e.hw1 = e.hw2 = e.hw3 = e.hw4 = 0xFFFFFFFFu;
    e.ggrp = 0;
    e.hcnt = 0;
    e.ntrace = 0;
    e.greater = NONE;
    e.gplay = 0;
    e.cur = 0;
    e.winner = NONE;
}

// ---- legal mask ------------------------------------------------------------------------------------------------
struct Legal {
    uint32_t total;   // legal combos (pass not included)
    uint32_t nl;      // mask dwords pass c tests (listed in L.lst); > LIST_CAP: more, not all listed
};

__device__ __forceinline__ void zero_mask(WaveLds& L, int lane)
{
    uint4* z = (uint4*)L.mask;
#pragma unroll
    for (int j = 0; j < (MASK_WORDS / 4 + WAVE - 1) / WAVE; j++) {
        const int q = j * WAVE + lane;
        if (q < MASK_WORDS / 4) z[q] = make_uint4(0, 0, 0, 0);
    }
}

// pass c for 2 x PAIRS listed dwords from list entry t0 on (entries >= nl are empty): lanes 0..31 take the even entry
// of a pair, 32..63 the odd one; all the id loads are issued before the first test
constexpr int PAIRS = 4;
__device__ __forceinline__ void test_listed(uint32_t t0, uint32_t nl, uint64_t h, const Cand& c, const Tab& tb,
                                            WaveLds& L, int lane, Legal& r)
{
    uint64_t cnt[PAIRS];
    uint32_t id[PAIRS], dw[PAIRS];
    bool live[PAIRS], ent[PAIRS];
#pragma unroll
    for (int q = 0; q < PAIRS; q++) {
        const uint32_t e = t0 + 2u * (uint32_t)q + (lane < 32 ? 0u : 1u);
        ent[q] = e < nl;
        dw[q] = ent[q] ? L.lst[e & (LIST_RING - 1)] : 0u;
        id[q] = dw[q] * 32u + (uint32_t)(lane & 31);
        live[q] = ent[q] && id[q] < (uint32_t)PASS;
        cnt[q] = live[q] ? tb.cnt[id[q]] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < PAIRS; q++) {
        const uint64_t m = __ballot(live[q] && contains(h, cnt[q]) && c.ok(id[q]));
        if ((lane & 31) == 0 && ent[q]) L.mask[MASK_PAD + dw[q]] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
        r.total += (uint32_t)__popcll(m);
    }
}

// mask image must be zero on entry
__device__ __forceinline__ Legal build_legal(const Env& e, const Cand& c, const Tab& tb, const TabLds& T, WaveLds& L,
                                             int lane)
{
    Legal r;
    r.total = 0;
    r.nl = 0;
    if (e.over()) return r;                                        // game.py:110-128: no actions once over
    const uint64_t h = e.hand(e.cur);
    // a. groups
    uint32_t base = 0;
#pragma unroll
    for (int k = 0; k < MAX_GROUPS / WAVE; k++) {
        const int g = k * WAVE + lane;
        bool pass = false;
        if (g < tb.ng) {
            const uint4 q = T.grp[g];
            pass = contains(h, (uint64_t)q.x | ((uint64_t)q.y << 32)) && c.ok(q.z & 0xFFFFu);
        }
        const uint64_t b = __ballot(pass);
        if (g <= tb.ng) L.pre[g] = (uint16_t)(base + mbcnt(b));
        base += (uint32_t)__popcll(b);
    }
    if (base == 0) return r;
    wave_sync_lds();
    // b. dwords that any passing group overlaps, appended to the list in ascending order (a ring of LIST_RING: at most
    // 7 + 64 entries wait for their test); c. their ids, 2 x PAIRS listed dwords per batch
    // chunks of 64 dwords that any passing group reaches (lane k tests chunk k): the others are skipped whole
    bool chunk_pass = false;
    if (lane < (ND + WAVE - 1) / WAVE) {
        const int last = lane * WAVE + WAVE - 1 < ND ? lane * WAVE + WAVE - 1 : ND - 1;
        const uint32_t lo = T.drange[lane * WAVE] & 0xFFFFu, hi = T.drange[last] >> 16;
        chunk_pass = L.pre[hi + 1] > L.pre[lo];
    }
    uint64_t chunks = __ballot(chunk_pass);
    uint32_t tested = 0;
    while (chunks) {
        const int k = __builtin_ctzll(chunks);
        chunks &= chunks - 1;
        const int d = k * WAVE + lane;
        bool pass = false;
        if (d < ND) {
            const uint32_t dr = T.drange[d];
            pass = L.pre[(dr >> 16) + 1] > L.pre[dr & 0xFFFFu];
        }
        const uint64_t bits = __ballot(pass);
        if (pass) L.lst[(r.nl + mbcnt(bits)) & (LIST_RING - 1)] = (uint16_t)d;
        r.nl += (uint32_t)__popcll(bits);
        for (; r.nl - tested >= 2u * PAIRS; tested += 2u * PAIRS) test_listed(tested, r.nl, h, c, tb, L, lane, r);
    }
    if (tested < r.nl) test_listed(tested, r.nl, h, c, tb, L, lane, r);
    return r;
}

// the k-th set bit of `word` (k < popcount): lane l < 32 holds bit l, mbcnt counts the set bits below it
__device__ __forceinline__ uint32_t kth_bit(uint32_t word, uint32_t k, int lane)
{
    const bool hit = lane < 32 && ((word >> (lane & 31)) & 1u) && __builtin_amdgcn_mbcnt_lo(word, 0u) == k;
    return (uint32_t)__builtin_ctzll(__ballot(hit));
}

// the k-th legal id in ascending order (k < total + !leading; pass is the largest id). Listed dwords (the usual
// case): lane l holds listed dword l, one wave prefix scan over their popcounts finds it. Else (list overflow) lane l
// counts the legal bits of mask dwords [16 l, 16 l + 16), a wave prefix scan finds the lane, 16 lanes then the dword.
__device__ __forceinline__ uint32_t kth_legal(uint32_t k, const Legal& r, const WaveLds& L, int lane)
{
    if (k >= r.total) return (uint32_t)PASS;
    if (r.nl <= (uint32_t)LIST_CAP) {
        const uint32_t d = (uint32_t)lane < r.nl ? L.lst[lane] : 0u;
        const uint32_t w = (uint32_t)lane < r.nl ? L.mask[MASK_PAD + d] : 0u;
        const uint32_t pc = (uint32_t)__popc(w);
        uint32_t inc = pc;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= o) inc += y;
        }
        const int j = __builtin_ctzll(__ballot(inc > k));
        const uint32_t kk = k - (rl(inc, j) - rl(pc, j));
        return rl(d, j) * 32u + kth_bit(rl(w, j), kk, lane);
    }
    uint32_t pc = 0;
    if (lane < KTH_LANES) {
        const uint4* w = (const uint4*)(L.mask + MASK_PAD) + lane * (KTH_WORDS / 4);
#pragma unroll
        for (int j = 0; j < KTH_WORDS / 4; j++) {
            const uint4 x = w[j];
            pc += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        }
    }
    uint32_t inc = pc;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += y;
    }
    const int j = __builtin_ctzll(__ballot(inc > k));
    k -= rl(inc, j) - rl(pc, j);
    // second level: the 16 dwords of lane j
    const uint32_t w = lane < KTH_WORDS ? L.mask[MASK_PAD + j * KTH_WORDS + lane] : 0u;
    const uint32_t p2 = (uint32_t)__popc(w);
    uint32_t inc2 = p2;
#pragma unroll
    for (int o = 1; o < KTH_WORDS; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc2, o);
        if (lane >= o) inc2 += y;
    }
    const int q = __builtin_ctzll(__ballot(lane < KTH_WORDS && inc2 > k));
    const uint32_t kk = k - (rl(inc2, q) - rl(p2, q));
    return (uint32_t)(j * KTH_WORDS + q) * 32u + kth_bit(rl(w, q), kk, lane);
}

// ---- obs -------------------------------------------------------------------------------------------------------
// _extract_state (envs/doudizhu.py:26-134) of player `self` as bits in L.bv. Blocks of 54 bits:
//   0 hand, 1 others' cards, 2 last non-pass action, 3..11 the last 9 actions ('' padded in front), then
//   landlord: 12 / 13 cards played by players 2 / 1, one-hots of their hand sizes at 756 / 773 (17 wide);
//   peasant:  12 / 13 cards played by the landlord / teammate, 14 / 15 their last actions, one-hots of their hand
//             sizes at 864 (20 wide) / 884 (17 wide).
__device__ __forceinline__ void build_obs(const Env& e, uint32_t self, WaveLds& L, int lane)
{
    const uint32_t nt = e.ntrace;
    const uint32_t h8 = e.hw4 & 0xFFFFu;
    const uint32_t mate = 3u - self;
    const uint64_t last_c = rl64(e.hcnt, h8 == (uint32_t)PASS ? 10 : 11);   // last non-pass action (h8, else h7)
    uint64_t ll_c = 0, lt_c = 0;                                               // landlord's / teammate's last action
    if (self != 0) {
        if (nt >= 1u) ll_c = rl64(e.hcnt, 11 - (int)((nt - 1u) % 3u));
        if (nt > mate) lt_c = rl64(e.hcnt, 11 - (int)((nt - 1u - mate) % 3u));
    }
    // the block of lane s, selected without branches (the candidates are wave-uniform)
    const int s = lane;
    const uint64_t u1 = e.hand(self == 0 ? 1u : 0u) + e.hand(self == 2 ? 1u : 2u);
    const uint64_t u12 = self == 0 ? e.q2 : e.q0, u13 = self == 0 ? e.q1 : e.played(mate);
    const uint64_t direct = keep64(s == 0, e.hand(self)) | keep64(s == 1, u1) | keep64(s == 2, last_c) |
                            keep64(s >= 3 && s <= 11, e.hcnt) | keep64(s == 12, u12) | keep64(s == 13, u13) |
                            keep64(s == 14, ll_c) | keep64(s == 15, lt_c);
    if (s < NSEG) L.segv[s] = cards_bits(direct);
    uint32_t p1, p2;
    if (self == 0) {
        const uint32_t n2 = num_cards(e.h2), n1 = num_cards(e.h1);
        p1 = 756u + (n2 >= 1u ? n2 - 1u : 16u);
        p2 = 773u + (n1 >= 1u ? n1 - 1u : 16u);
    } else {
        const uint32_t n0 = num_cards(e.h0), nm = num_cards(e.hand(mate));
        p1 = 864u + (n0 >= 1u ? n0 - 1u : 19u);
        p2 = 884u + (nm >= 1u ? nm - 1u : 16u);
    }
    wave_sync_lds();
    if (lane < BV_WORDS) {
        const int x0 = lane == 0 ? 0 : 32 * lane - 16;             // first obs bit of this dword (lane 0: see below)
        const int sg = x0 / 54, off = x0 - 54 * sg;
        uint32_t v = (uint32_t)((L.segv[sg] >> off) | (L.segv[sg + 1] << (54 - off)));
        const uint32_t d1 = p1 - (uint32_t)x0, d2 = p2 - (uint32_t)x0;   // the one-hots are past dword 0
        L.bv[lane] = lane == 0 ? v << 16                                  // dword 0 = 16 pad bits + obs bits 0..15
                               : v | keep32(d1 < 32u, 1u << (d1 & 31u)) | keep32(d2 < 32u, 1u << (d2 & 31u));
    }
}

// ---- row writers: 16-B stores for the chunks fully inside a row; its two end chunks in one pass for both rows --
__device__ __forceinline__ uint4 expand_bits16(uint32_t x)   // 16 bits -> 16 bytes of 0/1
{
    uint4 o;
    o.x = ((x & 15u) * 0x00204081u) & 0x01010101u;
    o.y = (((x >> 4) & 15u) * 0x00204081u) & 0x01010101u;
    o.z = (((x >> 8) & 15u) * 0x00204081u) & 0x01010101u;
    o.w = (((x >> 12) & 15u) * 0x00204081u) & 0x01010101u;
    return o;
}

// (default-policy stores: nontemporal ones, a win for the lane-per-env games' full-line spans, measured 4.8 -> 6.0 ms
// per launch here, where every row boundary splits a line between two waves)

// chunk q of a row misaligned by mis (its first byte is row byte 16 q - mis; bytes before the row are don't-care)
__device__ __forceinline__ uint4 obs_chunk(const uint32_t* bv, int q, int mis)
{
    const int bp = 16 * q - mis + 16;                               // bit of bv, >= 1
    const uint64_t two = (uint64_t)bv[bp >> 5] | ((uint64_t)bv[(bp >> 5) + 1] << 32);
    return expand_bits16((uint32_t)(two >> (bp & 31)) & 0xFFFFu);
}
__device__ __forceinline__ uint4 legal_chunk(const uint32_t* mask, int q, int mis)
{
    const int sb = 4 * MASK_PAD + 16 * q - mis;                     // byte of the mask image, >= 1
    const uint32_t* w = mask + (sb >> 2);
    const int sh = sb & 3;                                          // alignbyte(x, y, 0) = y
    return make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], sh), __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                      __builtin_amdgcn_alignbyte(w[3], w[2], sh), __builtin_amdgcn_alignbyte(w[4], w[3], sh));
}

// the obs row (OBS bytes) and / or the legal row (LB bytes); null rows are skipped
__device__ __forceinline__ void write_rows(const WaveLds& L, uint8_t* orow, uint8_t* lrow, int lane)
{
    if (orow) {
        const int mis = (int)((uintptr_t)orow & 15u), nchunks = (mis + OBS + 15) >> 4;   // <= 58
        if (lane >= 1 && lane < nchunks - 1) *(uint4*)(orow - mis + 16 * lane) = obs_chunk(L.bv, lane, mis);
    }
    if (lrow) {
        const int mis = (int)((uintptr_t)lrow & 15u), nchunks = (mis + LB + 15) >> 4;    // <= 216
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int q = j * WAVE + lane;
            if (q >= 1 && q < nchunks - 1) *(uint4*)(lrow - mis + 16 * q) = legal_chunk(L.mask, q, mis);
        }
    }
    // the two end chunks of both rows, one byte per lane in one store: lanes 0..15 / 16..31 the obs row's first / last
    // chunk, 32..47 / 48..63 the legal row's
    const bool is_obs = lane < 32;
    uint8_t* row = is_obs ? orow : lrow;
    if (row) {
        const int nbytes = is_obs ? OBS : LB;
        const int mis = (int)((uintptr_t)row & 15u), nchunks = (mis + nbytes + 15) >> 4;
        const int q = (lane & 16) ? nchunks - 1 : 0, o = 16 * q - mis + (lane & 15);   // row byte
        if (o >= 0 && o < nbytes) {
            const uint32_t x = 16u + (uint32_t)o;   // obs: bit of L.bv; legal: byte of L.mask (MASK_PAD = 4)
            const uint32_t v = is_obs ? (L.bv[x >> 5] >> (x & 31u)) & 1u : ((const uint8_t*)L.mask)[x];
            row[o] = (uint8_t)v;
        }
    }
}

struct Ctx {
    int lane, wid;
    int64_t env;
    bool valid;
};
__device__ __forceinline__ Ctx ctx_of(int64_t n)
{
    Ctx c;
    c.lane = (int)(threadIdx.x & (WAVE - 1));
    c.wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    c.env = (int64_t)blockIdx.x * WPB + c.wid;
    c.valid = c.env < n;
    return c;
}

template <bool PHX>
__device__ __forceinline__ WaveMt<PHX> wave_mt(uint32_t* mt, const uint32_t* ctl, int64_t env)
{
    WaveMt<PHX> m;
    m.base = mt + env * MT_WORDS;
    const uint32_t w = ctl[env];
    m.pos = w & 0x7FFu;
    m.stale = (w >> 16) & 1u;
    m.dabs = 0;
    m.key = 0;
    if constexpr (PHX) {
        m.key = (uint64_t)m.base[0] | (uint64_t)m.base[1] << 32;
        m.dabs = m.base[2];
    }
    return m;
}

// obs / legal / player / done of the current state, for `self` (observe) or the current player
__device__ __forceinline__ void emit_state(const Env& e, uint32_t self, const Tab& tb, const TabLds& T, WaveLds& L,
                                           int lane, int64_t row, const cs_step_out& out)
{
    zero_mask(L, lane);
    wave_sync_lds();
    const Cand cd = cand_of(e, tb, T);
    build_legal(e, cd, tb, T, L, lane);
    if (!e.over() && !cd.leading && lane == 0) L.mask[MASK_PAD + PASS / 32] |= 1u << (PASS & 31);
    build_obs(e, self, L, lane);
    wave_sync_lds();
    write_rows(L, out.obs ? (uint8_t*)out.obs + row * OBS : nullptr,
               out.legal ? (uint8_t*)out.legal + row * LB : nullptr, lane);
    if (lane == 0) {
        if (out.player) ((uint8_t*)out.player)[row] = (uint8_t)e.cur;
        if (out.done) ((uint8_t*)out.done)[row] = (uint8_t)e.over();
    }
}

__device__ __forceinline__ void payoffs(uint32_t winner, float* r)   // judger.py:350-359
{
    r[0] = winner == 0 ? 1.f : 0.f;
    r[1] = winner == 0 ? 0.f : 1.f;
    r[2] = r[1];
}
__device__ __forceinline__ void payoffs(const Env& e, float* r) { payoffs(e.winner, r); }

template <bool PHX>
__global__ __launch_bounds__(BLOCK) void k_reset(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                  cs_step_out out, Tab tb, StepRecord rec)
{
    __shared__ WaveLds lds[WPB];
    __shared__ TabLds tl;
    load_tab(tl, tb);                 // every thread of the block, before any wave leaves
    const Ctx c = ctx_of(n);
    if (!c.valid) return;
    WaveLds& L = lds[c.wid];
    Env e;
    auto m = wave_mt<PHX>(mt, ctl, c.env);
    deal(e, m, c.lane);
    emit_state(e, e.cur, tb, tl, L, c.lane, c.env, out);
    if (c.lane == 0 && out.reward) {
        float* r = (float*)out.reward + c.env * P;
        r[0] = r[1] = r[2] = 0.f;
    }
    e.store(st, c.env, c.lane);
    if (c.lane == 0) m.save(ctl, c.env);
    if (rec.seq != nullptr && c.env == rec.env) {   // StepRecord (cs_engine.h): state words, fence, sequence number
        e.store(rec.words, 0, c.lane);
        __threadfence_system();
        if (c.lane == 0) __hip_atomic_store(rec.seq, rec.seqv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool PHX>
__global__ __launch_bounds__(BLOCK) void k_step(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                 const int32_t* actions, cs_step_out out, Tab tb, StepRecord rec)
{
    __shared__ WaveLds lds[WPB];
    __shared__ TabLds tl;
    load_tab(tl, tb);                 // every thread of the block, before any wave leaves
    const Ctx c = ctx_of(n);
    if (!c.valid) return;
    WaveLds& L = lds[c.wid];
    Env e;
    e.load(st, c.env, c.lane, tb);
    auto m = wave_mt<PHX>(mt, ctl, c.env);
    float r[3] = {0.f, 0.f, 0.f};
    bool done = false;
    if (e.over()) {
        deal(e, m, c.lane);
    } else {
        const Cand cd = cand_of(e, tb, tl);
        e.apply(decode_action(actions[c.env], e, cd, tb), tb, c.lane);
        done = e.over();
        if (done) payoffs(e, r);
    }
    emit_state(e, e.cur, tb, tl, L, c.lane, c.env, out);
    if (c.lane == 0) {
        if (out.reward) {
            float* o = (float*)out.reward + c.env * P;
            o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
        }
        if (out.done) ((uint8_t*)out.done)[c.env] = (uint8_t)done;
    }
    e.store(st, c.env, c.lane);
    if (c.lane == 0) m.save(ctl, c.env);
    if (rec.seq != nullptr && c.env == rec.env) {   // StepRecord (cs_engine.h): state words, fence, sequence number
        e.store(rec.words, 0, c.lane);
        __threadfence_system();
        if (c.lane == 0) __hip_atomic_store(rec.seq, rec.seqv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(BLOCK) void k_observe(const uint32_t* st, int64_t n, int player, cs_step_out out, Tab tb,
                                                    StepRecord rec)
{
    __shared__ WaveLds lds[WPB];
    __shared__ TabLds tl;
    load_tab(tl, tb);                 // every thread of the block, before any wave leaves
    const Ctx c = ctx_of(n);
    if (!c.valid) return;
    Env e;
    e.load(st, c.env, c.lane, tb);
    emit_state(e, (uint32_t)player, tb, tl, lds[c.wid], c.lane, c.env, out);
    if (rec.seq != nullptr && c.env == rec.env) {   // StepRecord (cs_engine.h): state words, fence, sequence number
        e.store(rec.words, 0, c.lane);
        __threadfence_system();
        if (c.lane == 0) __hip_atomic_store(rec.seq, rec.seqv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- the rollout: TWO envs per wave, legal rows without a mask image ------------------------------------------------
// Lanes 0..31 play one env and lanes 32..63 the next: every step below runs for both envs in the same instructions
// (each half-wave is one env's 32 lanes), so the game logic that the one-env kernels run as wave-uniform scalar code
// -- the scalar unit is their busiest pipe -- becomes vector code shared by two envs, and the two envs' dependency
// chains (LDS round trips, table loads) overlap inside one wave. Same functions of the same state, same outputs:
// the per-env values are simply held per lane (uniform within a half). The deal (rare: once per game) still runs with
// the whole wave for one env at a time, through the one-env `deal`.
//
// The legal row is 27 472 bits of which a random-play step sets ~6 (1.8 nonzero mask dwords on average, at most 46 in
// 409 600 steps of random play, `tools/ddz_sparsity.py`). So the step keeps no 3.4 KB mask image: the legal scan
// appends each nonzero mask dword (index, value) to a list in ascending order (NZ_CAP entries, a bitmap of the listed
// dwords and its prefix ranks), the policy pick scans the list's popcounts, and the row's 16-B chunks are zeros except
// where the bitmap says a listed dword falls -- those few are gathered from the list. Per env 1.6 KB of LDS instead of
// 4.4 KB, no per-step zeroing or cleaning of an image. A step whose list overflows (more than NZ_CAP nonzero dwords:
// none seen in random play, but a 20-card hand can have hundreds) runs the legal scan a second time with a row cursor
// that writes the row in ascending order straight to HBM (zeros between the nonzero dwords) and finds the picked id on
// the way; kernel flag bit 1 forces that path for every step (tests/test_gpu_engine.py runs it against the oracle).
#ifndef CS_DDZ_PAIR_WAVES
#define CS_DDZ_PAIR_WAVES 4   // waves per block (the group table in LDS is shared by 2 x this many envs)
#endif
#ifndef CS_DDZ_PAIR_MINW
#define CS_DDZ_PAIR_MINW 6    // waves per SIMD the registers must allow (80 VGPRs; 5: +1 %, 4: +13 %, EXPERIMENTS R6-1)
#endif
constexpr int HW = WAVE / 2;                         // lanes per env
constexpr int PWPB = CS_DDZ_PAIR_WAVES, PBLOCK = PWPB * WAVE;
constexpr int NCH = (ND + HW - 1) / HW;              // 27 chunks of 32 mask dwords (pass b of the legal scan)
constexpr int NZ_CAP = 64;                           // nonzero mask dwords an env's list holds
constexpr int TRING = 64;                            // pass c's ring of dwords waiting for their test (<= 3 + 32)
constexpr int NZBM = 28;                             // bitmap words over the 859 mask dwords, + 1 zero word
constexpr int LROW_IT = (LB + 15 + 15) / 16 / HW + 1;   // 32-lane iterations over a legal row's <= 216 16-B chunks
struct alignas(16) PairLds {
    uint32_t val[NZ_CAP];            // the step's nonzero mask dwords in ascending order: values
    uint32_t nzbm[NZBM];             // bit d: mask dword d is in the list
    uint16_t idx[NZ_CAP];            //   ... their indices
    uint16_t tst[TRING];             // pass c's ring of dwords to test / the following fast path's OR scratch
    uint16_t pre[MAX_GROUPS + 8];    // pass a's group prefix counts
    uint8_t npre[32];                // listed dwords before bitmap word w
    uint64_t segv[NSEG];             // the obs image: 54-bit blocks
    uint32_t bv[BV_WORDS];           //   ... and its bits (obs bit x at bit 16 + x)
    uint64_t q[3];                   // the env's played cards (Round.played_cards): read by the obs, added to by a play
    // cold env state, touched at a deal and at the end of the launch only
    uint64_t mkey;                   // the stream (WaveMt fields): Philox key,
    uint32_t mpos, mdabs;            //   position | stale << 16, Philox draw count
    uint8_t deck[64];                // the dealt deck (state words W_DECK..)
};
static_assert(MAX_GROUPS % HW == 0 && NSEG <= HW && BV_WORDS == HW && NCH <= HW && NZBM <= HW && NZ_CAP <= 2 * HW &&
              (ND + 31) / 32 < NZBM && 2 * TRING >= 4 * HW, "pair layout");

__device__ __forceinline__ uint32_t half32(uint64_t b, int lane) { return lane < HW ? (uint32_t)b : (uint32_t)(b >> 32); }
__device__ __forceinline__ uint32_t below32(uint32_t m, int hl) { return (uint32_t)__popc(m & ((1u << hl) - 1u)); }
// v at lane k of this lane's half (k may differ per lane)
__device__ __forceinline__ uint32_t hshfl(uint32_t v, int lane, uint32_t k)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((uint32_t)(lane & HW) + (k & (HW - 1))) << 2), (int)v);
}
__device__ __forceinline__ uint64_t hshfl64(uint64_t v, int lane, uint32_t k)
{
    return (uint64_t)hshfl((uint32_t)v, lane, k) | ((uint64_t)hshfl((uint32_t)(v >> 32), lane, k) << 32);
}

// An env held by a half-wave: every field uniform within the half (per lane), the small fields packed, the trace's
// last 9 entries distributed over lanes 3..11 (like Env::hcnt) -- the registers the step loop keeps live
struct PEnv {
    uint64_t h0, h1, h2;   // hands (the played cards are in the env's LDS, PairLds::q)
    uint64_t hcnt;         // lane s = 3..11: packed counts of trace entry s - 3 of the last 9 (0: pass / none)
    uint32_t hid;          // lane s = 3..11: its action id (NO_ACTION: none)
    uint32_t gw;           // greater player's last play id | its (type, weight) group << 16
    uint32_t sw;           // ntrace | greater << 16 | cur << 20 | winner << 24 (players and NONE fit 2 bits)
    __device__ __forceinline__ uint32_t ntrace() const { return sw & 0xFFFFu; }
    __device__ __forceinline__ uint32_t greater() const { return (sw >> 16) & 3u; }
    __device__ __forceinline__ uint32_t cur() const { return (sw >> 20) & 3u; }
    __device__ __forceinline__ uint32_t winner() const { return (sw >> 24) & 3u; }
    __device__ __forceinline__ uint32_t ggrp() const { return gw >> 16; }
    __device__ __forceinline__ bool over() const { return winner() != NONE; }
    __device__ __forceinline__ uint64_t hand(uint32_t p) const
    {
        return keep64(p == 0, h0) | keep64(p == 1, h1) | keep64(p == 2, h2);
    }
    // Env::apply_with for the half's env (lane: the caller's lane id, hl: lane in the half; q: its played cards)
    __device__ __forceinline__ void apply_with(uint32_t a, uint64_t c, uint32_t gid, int lane, int hl, uint64_t* q)
    {
        const uint32_t p = cur();
        // the trace shifted down one lane (lanes 3..10 read their upper neighbour, inside the half)
        const int src = ((lane & HW) + ((hl + 1) & (HW - 1))) << 2;
        const uint64_t down = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)hcnt) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(hcnt >> 32)) << 32);
        const uint32_t hdown = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)hid);
        const bool mid = hl >= 3 && hl < 11;
        hcnt = hl == 11 ? c : (mid ? down : 0ull);
        hid = hl == 11 ? a : (mid ? hdown : NO_ACTION);
        uint32_t s = sw + 1u;   // ntrace++
        if (a != (uint32_t)PASS) {
            const uint64_t c0 = keep64(p == 0, c), c1 = keep64(p == 1, c), c2 = keep64(p == 2, c);
            h0 -= c0; h1 -= c1; h2 -= c2;
            if (hl == 0) q[p] += c;
            gw = a | gid << 16;
            s = (s & ~(3u << 16)) | p << 16;
            if (hand(p) == 0) s = (s & ~(3u << 24)) | p << 24;
        }
        s &= ~(3u << 20);
        sw = s | (p == 2 ? 0u : p + 1u) << 20;
    }
};

// cand_of for a half's env: the same type's greater weights [c_lo, c_lo + c_len) (leading: every id), the bombs and
// the rocket as flags over the table's ranges (scalars)
struct PCand {
    uint32_t c_lo, c_len;
    uint32_t fl;              // bit 0: the bombs, bit 1: the rocket, bit 2: leading
    uint32_t b_lo, b_n, r_lo; // the table's bomb range and rocket id
    __device__ __forceinline__ bool leading() const { return (fl & 4u) != 0u; }
    __device__ __forceinline__ uint32_t nb() const { return (fl & 1u) ? b_n : 0u; }
    __device__ __forceinline__ uint32_t nr() const { return (fl >> 1) & 1u; }
    __device__ __forceinline__ bool ok(uint32_t x) const
    {
        return (x - c_lo < c_len) | ((fl & 1u) && x - b_lo < b_n) | ((fl & 2u) && x == r_lo);
    }
    __device__ __forceinline__ bool meets(uint32_t lo, uint32_t hi) const   // does a candidate lie in [lo, hi)?
    {
        return (c_len && c_lo < hi && c_lo + c_len > lo) | ((fl & 1u) && b_lo < hi && b_lo + b_n > lo) |
               ((fl & 2u) && r_lo < hi && r_lo >= lo);
    }
};
__device__ __forceinline__ PCand pcand(const PEnv& e, const Tab& tb, const TabLds& T)
{
    const Cand c = cand_at(e.greater(), e.cur(), e.ggrp(), tb, T);
    PCand p;
    p.c_lo = c.c_lo;
    p.c_len = c.c_len;
    p.fl = (c.b_len ? 1u : 0u) | (c.r_len ? 2u : 0u) | (c.leading ? 4u : 0u);
    p.b_lo = (uint32_t)tb.bomb_lo;
    p.b_n = (uint32_t)(tb.bomb_hi - tb.bomb_lo);
    p.r_lo = (uint32_t)tb.rocket;
    return p;
}

// inclusive prefix sum within each half-wave, with DPP (no LDS): row_shr 1, 2, 4, 8 inside the 16-lane rows, then
// row_bcast:15 adds the last lane of rows 0 / 2 to rows 1 / 3 (row mask 0xA: rows 0 and 2 take 0)
__device__ __forceinline__ uint32_t scan32(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    return x;
}

// the k-th set bit of each half's `m` (k < popcount(m), per half)
__device__ __forceinline__ uint32_t kth_bit32(uint32_t m, uint32_t k, int lane)
{
    const int hl = lane & (HW - 1);
    const uint32_t bm = half32(__ballot(((m >> hl) & 1u) && below32(m, hl) == k), lane);
    return bm ? (uint32_t)__builtin_ctz(bm) : 0u;
}

// ---- the sinks of the legal scan: where each tested mask dword's value goes (in ascending dword order) -------------
// the list (the usual path): nonzero dwords appended with their bitmap bit; n counts past NZ_CAP (overflow)
struct NzSink {
    PairLds* L;
    uint32_t n;   // per half
    __device__ __forceinline__ void operator()(bool ent, uint32_t dw, uint32_t m, int lane)
    {
        const bool put = ent && m != 0u;
        if (put && (lane & (HW - 1)) == 0 && n < (uint32_t)NZ_CAP) {
            L->val[n] = m;
            L->idx[n] = (uint16_t)dw;
            atomicOr(&L->nzbm[dw >> 5], 1u << (dw & 31u));
        }
        n += put ? 1u : 0u;
    }
};
// the overflow path: the row written in ascending order straight to HBM (u16 stores: rows start at even addresses),
// zeros between the nonzero dwords, and the k-th legal id found on the way
struct RowCursor {
    uint8_t* row;      // per half; null: the half is not on this path
    uint32_t w;        // row bytes written
    uint32_t k, run;   // the pick: the k-th legal id (k < the legal count), legal ids seen so far
    uint32_t found;
    bool pass;         // the pass bit goes into dword ND - 1 (its bit PASS % 32)
    __device__ __forceinline__ void fill(uint32_t to, int lane)   // zeros over [w, to), both even
    {
        uint32_t o = w + 2u * (uint32_t)(lane & (HW - 1));
        while (__ballot(row != nullptr && o < to)) {
            if (row != nullptr && o < to) *(uint16_t*)(row + o) = 0;
            o += 2u * HW;
        }
        if (row != nullptr) w = to > w ? to : w;
    }
    __device__ __forceinline__ void put(bool ent, uint32_t dw, uint32_t m, int lane)
    {
        const bool on = row != nullptr && ent && (m != 0u || (pass && dw == (uint32_t)(ND - 1)));
        const uint32_t c = (uint32_t)__popc(m);
        const uint32_t kb = kth_bit32(m, k - run, lane);
        if (on && k >= run && k < run + c) found = dw * 32u + kb;
        run += on ? c : 0u;
        const uint32_t v = m | (pass && dw == (uint32_t)(ND - 1) ? 1u << (PASS & 31) : 0u);
        fill(on ? 4u * dw : 0u, lane);
        if (on && (lane & (HW - 1)) == 0) {
            *(uint16_t*)(row + 4u * dw) = (uint16_t)v;
            if (4u * dw + 2u < (uint32_t)LB) *(uint16_t*)(row + 4u * dw + 2u) = (uint16_t)(v >> 16);
        }
        if (on) w = 4u * dw + 4u < (uint32_t)LB ? 4u * dw + 4u : (uint32_t)LB;
    }
    __device__ __forceinline__ void operator()(bool ent, uint32_t dw, uint32_t m, int lane) { put(ent, dw, m, lane); }
    __device__ __forceinline__ void finish(int lane)   // the pass dword if no tested dword carried it, the zero tail
    {
        put(pass && w <= 4u * (uint32_t)(ND - 1), (uint32_t)(ND - 1), 0u, lane);
        fill((uint32_t)LB, lane);
    }
};

// pass c (see build_legal) for the listed dwords [t0, lim) of each half's env, up to 4 per env
template <class Sink>
__device__ __forceinline__ void test_listed2(uint32_t t0, uint32_t lim, uint64_t h, const PCand& c, const Tab& tb,
                                             const PairLds& L, int lane, Legal& r, Sink& sink)
{
    const int hl = lane & (HW - 1);
    uint64_t cnt[4];
    uint32_t id[4], dw[4];
    bool live[4], ent[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t e = t0 + (uint32_t)q;
        ent[q] = e < lim;
        dw[q] = ent[q] ? L.tst[e & (TRING - 1)] : 0u;
        id[q] = dw[q] * 32u + (uint32_t)hl;
        live[q] = ent[q] && id[q] < (uint32_t)PASS;
        cnt[q] = live[q] ? tb.cnt[id[q]] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t m = half32(__ballot(live[q] && contains(h, cnt[q]) && c.ok(id[q])), lane);
        sink(ent[q], dw[q], m, lane);
        r.total += (uint32_t)__popc(m);
    }
}

// Following a play the candidates are at most three id ranges (cand_of: the same type's greater weights, the bombs, the
// rocket). In random play they number <= 32 in ~93 % of the following steps (~70 % of all steps; the same-type range
// has median 5 ids, p90 14), and then the half's 32 lanes test one candidate each -- no group pass, no chunk pass, no
// listed-dword batches. Lane k takes the k-th candidate in id order (the table's bomb and rocket types are its last
// ids, so the ranges come in the order same type < bombs < rocket); the dwords holding a legal id go to the list in
// order, their bits OR-ed together through 32 scratch dwords. Two parts: fast_issue loads the candidates' packed counts
// from the table in HBM / L2 at the start of the step, fast_finish tests them after the group pass (other half) and
// build_obs2, which hide the load latency (issued and tested back to back the path measured slower than the group pass
// it replaces). The solo / pair / trio / bomb / rocket candidates (~95 % of these steps have no other) take their
// counts from simple_cnt: no load. Kernel flag bit 0 turns the path off (the group pass for every step: same outputs).
struct Fast {
    bool fast, cand, load;   // load: a candidate that is not a simple id (its counts come from the table)
    uint32_t id;
    uint64_t cnt;
};
__device__ __forceinline__ Fast fast_issue(const PEnv& e, const PCand& c, const Tab& tb, PairLds& L, int lane, bool act)
{
    const uint32_t hl = (uint32_t)(lane & (HW - 1));
    Fast f;
    f.fast = act && !e.over() && !c.leading() && c.c_len + c.nb() + c.nr() <= (uint32_t)HW;
    const uint32_t n0 = c.c_len, n1 = n0 + c.nb(), n2 = n1 + c.nr();
    f.cand = f.fast && hl < n2;
    f.id = hl < n0 ? c.c_lo + hl : (hl < n1 ? c.b_lo + (hl - n0) : c.r_lo + (hl - n1));
    const bool simple = simple_id(f.id, (uint32_t)tb.bomb_lo);
    f.load = f.cand && !simple;
    f.cnt = f.cand && simple ? simple_cnt(f.id, (uint32_t)tb.bomb_lo) : ~0ull;
    if (f.fast) ((uint32_t*)L.tst)[hl] = 0u;   // the OR scratch
    return f;
}
__device__ __forceinline__ void fast_finish(const Fast& f, uint64_t h, const Tab& tb, PairLds& L, int lane, Legal& r,
                                            NzSink& z)
{
    const uint32_t hl = (uint32_t)(lane & (HW - 1));
    uint32_t* scr = (uint32_t*)L.tst;
    uint64_t cnt = f.cnt;
    // table loads only where a candidate is not simple (~5 % of these steps), waited for inside this branch: on gfx950
    // a load's wait also waits for every earlier store (vmcnt counts both), here the previous step's row stores
    if (__ballot(f.load)) cnt = f.load ? tb.cnt[f.id] : cnt;
    const bool pass = f.cand && contains(h, cnt);
    const uint32_t m = half32(__ballot(pass), lane);
    const uint32_t dw = f.id >> 5;
    const uint32_t below = m & ((1u << hl) - 1u);                   // legal candidates before this lane's
    const uint32_t pdw = hshfl(dw, lane, below ? 31u - (uint32_t)__builtin_clz(below) : hl);
    const bool first = pass && (below == 0u || pdw != dw);           // the first legal id of its dword
    const uint32_t fm = half32(__ballot(first), lane);
    const uint32_t k = (uint32_t)__popc(fm & ((2u << hl) - 1u)) - 1u;   // its dword's rank in the list
    wave_sync_lds();
    if (pass) atomicOr(scr + k, 1u << (f.id & 31u));
    wave_sync_lds();
    if (first) {
        L.val[k] = scr[k];
        L.idx[k] = (uint16_t)dw;
        atomicOr(&L.nzbm[dw >> 5], 1u << (dw & 31u));
    }
    if (f.fast) {
        r.total = (uint32_t)__popc(m);
        z.n = (uint32_t)__popc(fm);
    }
}

// build_legal for each half's env (act: the half holds a live env on this path), in two parts: groups2 (pass a,
// the group prefix counts in L.pre; returns whether the half has any playable group) and scan2 (passes b and c over
// them; the sink takes every tested mask dword in ascending order)
__device__ __forceinline__ bool groups2(const PEnv& e, const PCand& c, const Tab& tb, const TabLds& T, PairLds& L,
                                        int lane, bool act)
{
    const int hl = lane & (HW - 1);
    const bool own = act;   // only the halves on this path write their prefix counts (the other half's may be live)
    act = act && !e.over();
    const uint64_t h = e.hand(e.cur());
    // a. groups, 32 per pass and env; a pass whose groups no candidate range of either env meets only writes the
    // prefix counts (following a play: the same type's greater weights, the bombs, the rocket)
    uint32_t base = 0;
#pragma unroll 2
    for (int k = 0; k < MAX_GROUPS / HW; k++) {
        const int g = k * HW + hl;
        const bool may = act && c.meets((uint32_t)tb.kfirst[k], (uint32_t)tb.kfirst[k + 1]);
        if (__ballot(may)) {
            bool pass = false;
            if (may && g < tb.ng) {
                const uint4 q = T.grp[g];
                pass = contains(h, (uint64_t)q.x | ((uint64_t)q.y << 32)) && c.ok(q.z & 0xFFFFu);
            }
            const uint32_t m = half32(__ballot(pass), lane);
            if (own && g <= tb.ng) L.pre[g] = (uint16_t)(base + below32(m, hl));
            base += (uint32_t)__popc(m);
        } else if (own && g <= tb.ng) {
            L.pre[g] = (uint16_t)base;
        }
    }
    return act && base != 0;
}
template <class Sink>
__device__ __forceinline__ Legal scan2(const PEnv& e, const PCand& c, const Tab& tb, const TabLds& T, PairLds& L,
                                       int lane, bool act, Sink& sink)
{
    const int hl = lane & (HW - 1);
    Legal r;
    r.total = 0;
    r.nl = 0;
    if (!__ballot(act)) return r;
    const uint64_t h = e.hand(e.cur());
    wave_sync_lds();
    // b. chunks of 32 dwords that any passing group reaches (lane k of a half: chunk k), their dwords queued in order;
    // c. 4 queued dwords per env and batch
    bool chp = false;
    if (act && hl < NCH) {
        const int last = hl * HW + HW - 1 < ND ? hl * HW + HW - 1 : ND - 1;
        const uint32_t lo = T.drange[hl * HW] & 0xFFFFu, hi = T.drange[last] >> 16;
        chp = L.pre[hi + 1] > L.pre[lo];
    }
    uint32_t chunks = half32(__ballot(chp), lane);
    uint32_t tested = 0;
    while (__ballot(chunks != 0u)) {
        const bool has = chunks != 0u;
        const int k = has ? __builtin_ctz(chunks) : 0;
        chunks &= chunks - 1u;
        const int d = k * HW + hl;
        bool pass = false;
        if (has && d < ND) {
            const uint32_t dr = T.drange[d];
            pass = L.pre[(dr >> 16) + 1] > L.pre[dr & 0xFFFFu];
        }
        const uint32_t m = half32(__ballot(pass), lane);
        if (pass) L.tst[(r.nl + below32(m, hl)) & (TRING - 1)] = (uint16_t)d;
        r.nl += (uint32_t)__popc(m);
        while (__ballot(r.nl - tested >= 4u)) {
            const bool full = r.nl - tested >= 4u;
            test_listed2(tested, full ? tested + 4u : tested, h, c, tb, L, lane, r, sink);
            tested += full ? 4u : 0u;
        }
    }
    if (__ballot(tested < r.nl)) test_listed2(tested, r.nl, h, c, tb, L, lane, r, sink);
    return r;
}

// the k-th legal id of each half's env from its list (k < the env's legal count, n <= NZ_CAP entries): lane l of a half
// holds entries l and 32 + l, a prefix scan of their popcounts finds the entry (the pass bit, merged into dword
// ND - 1, is the largest id and never reached)
__device__ __forceinline__ uint32_t kth_listed(uint32_t k, uint32_t n, const PairLds& L, int lane)
{
    const uint32_t hl = (uint32_t)(lane & (HW - 1));
    uint32_t v = hl < n ? L.val[hl] : 0u;
    uint32_t pc = (uint32_t)__popc(v);
    uint32_t inc = scan32(pc);
    const uint32_t tot = hshfl(inc, lane, HW - 1);
    uint32_t off = 0;
    const bool hi = k >= tot;   // only with more than 32 entries
    if (__ballot(hi)) {
        const uint32_t v2 = hl + HW < n ? L.val[hl + HW] : 0u;
        const uint32_t pc2 = (uint32_t)__popc(v2);
        const uint32_t inc2 = scan32(pc2);
        if (hi) {
            v = v2;
            pc = pc2;
            inc = inc2;
            k -= tot;
            off = HW;
        }
    }
    const uint32_t jm = half32(__ballot(inc > k), lane);
    const uint32_t j = jm ? (uint32_t)__builtin_ctz(jm) : 0u;
    const uint32_t incj = hshfl(inc, lane, j), pcj = hshfl(pc, lane, j), wj = hshfl(v, lane, j);
    const uint32_t dj = L.idx[(off + j) & (NZ_CAP - 1)];
    return dj * 32u + kth_bit32(wj, k - (incj - pcj), lane);
}

// mask dword d of the env's legal row from its list (0 when not listed)
__device__ __forceinline__ uint32_t listed_dword(const PairLds& L, uint32_t d)
{
    const uint32_t wb = L.nzbm[d >> 5], b = d & 31u;
    const uint32_t r = (uint32_t)L.npre[d >> 5] + (uint32_t)__popc(wb & ((1u << b) - 1u));
    return ((wb >> b) & 1u) ? L.val[r & (NZ_CAP - 1)] : 0u;
}

// build_obs for each half's env, observed by `self` (per half)
__device__ __forceinline__ void build_obs2(const PEnv& e, uint32_t self, PairLds& L, int lane)   // (L.q: played)
{
    const int hl = lane & (HW - 1);
    const uint32_t nt = e.ntrace();
    const uint32_t mate = 3u - self;
    // last non-pass action: the last trace entry unless it is a pass (or none: both give zero counts)
    const uint64_t l11 = hshfl64(e.hcnt, lane, 11u), l10 = hshfl64(e.hcnt, lane, 10u);
    const uint64_t last_c = l11 != 0ull ? l11 : l10;
    const uint64_t llv = hshfl64(e.hcnt, lane, 11u - (nt - 1u) % 3u);                 // landlord's last action
    const uint64_t ltv = hshfl64(e.hcnt, lane, 11u - (nt - 1u - mate) % 3u);          // teammate's last action
    const uint64_t ll_c = (self != 0u && nt >= 1u) ? llv : 0ull, lt_c = (self != 0u && nt > mate) ? ltv : 0ull;
    const int s = hl;
    const uint64_t u1 = e.hand(self == 0 ? 1u : 0u) + e.hand(self == 2 ? 1u : 2u);
    const uint64_t u12 = L.q[self == 0 ? 2 : 0], u13 = L.q[self == 0 ? 1 : mate];
    const uint64_t direct = keep64(s == 0, e.hand(self)) | keep64(s == 1, u1) | keep64(s == 2, last_c) |
                            keep64(s >= 3 && s <= 11, e.hcnt) | keep64(s == 12, u12) | keep64(s == 13, u13) |
                            keep64(s == 14, ll_c) | keep64(s == 15, lt_c);
    if (s < NSEG) L.segv[s] = cards_bits(direct);
    uint32_t p1, p2;
    if (self == 0) {
        const uint32_t n2 = num_cards(e.h2), n1 = num_cards(e.h1);
        p1 = 756u + (n2 >= 1u ? n2 - 1u : 16u);
        p2 = 773u + (n1 >= 1u ? n1 - 1u : 16u);
    } else {
        const uint32_t n0 = num_cards(e.h0), nm = num_cards(e.hand(mate));
        p1 = 864u + (n0 >= 1u ? n0 - 1u : 19u);
        p2 = 884u + (nm >= 1u ? nm - 1u : 16u);
    }
    wave_sync_lds();
    const int x0 = hl == 0 ? 0 : 32 * hl - 16;
    const int sg = x0 / 54, off = x0 - 54 * sg;
    const uint32_t v = (uint32_t)((L.segv[sg] >> off) | (L.segv[sg + 1] << (54 - off)));
    const uint32_t d1 = p1 - (uint32_t)x0, d2 = p2 - (uint32_t)x0;
    L.bv[hl] = hl == 0 ? v << 16 : v | keep32(d1 < 32u, 1u << (d1 & 31u)) | keep32(d2 < 32u, 1u << (d2 & 31u));
}

// the obs row and (lrow non-null) the legal row of each half's env, 16-B stores for the chunks inside a row and one
// byte per lane for its two end chunks. The legal row's chunks are zero unless a listed dword falls into them (zw: the
// half's nonzero bitmap words; a 32-chunk iteration j spans words 4 j - 1 .. 4 j + 4)
__device__ __forceinline__ void write_rows2(const PairLds& L, uint8_t* orow, uint8_t* lrow, uint32_t zw, int lane)
{
    const int hl = lane & (HW - 1);
    if (orow) {
        const int mis = (int)((uintptr_t)orow & 15u), nchunks = (mis + OBS + 15) >> 4;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int q = j * HW + hl;
            if (q >= 1 && q < nchunks - 1) *(uint4*)(orow - mis + 16 * q) = obs_chunk(L.bv, q, mis);
        }
    }
    if (lrow) {
        const int mis = (int)((uintptr_t)lrow & 15u), nchunks = (mis + LB + 15) >> 4;
#pragma unroll
        for (int j = 0; j < LROW_IT; j++) {
            const int q = j * HW + hl;
            const bool touched = ((zw >> (j ? 4 * j - 1 : 0)) & 0x3Fu) != 0u;
            if (q >= 1 && q < nchunks - 1) {
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (touched) {   // rare: gather the chunk's five mask dwords (row bytes 16 q - mis .. + 15)
                    const uint32_t s = (uint32_t)(16 * q - mis), d = s >> 2, sh = s & 3u;
                    const uint32_t w0 = listed_dword(L, d), w1 = listed_dword(L, d + 1), w2 = listed_dword(L, d + 2),
                                   w3 = listed_dword(L, d + 3), w4 = listed_dword(L, d + 4);
                    v = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                   __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
                }
                *(uint4*)(lrow - mis + 16 * q) = v;
            }
        }
    }
    // the rows' end chunks, a byte per lane: lanes 0..15 / 16..31 of a half the first / last chunk
#pragma unroll
    for (int rr = 0; rr < 2; rr++) {
        uint8_t* row = rr ? lrow : orow;
        if (row) {
            const int nbytes = rr ? LB : OBS;
            const int mis = (int)((uintptr_t)row & 15u), nchunks = (mis + nbytes + 15) >> 4;
            const int q = (hl & 16) ? nchunks - 1 : 0, o = 16 * q - mis + (hl & 15);
            if (o >= 0 && o < nbytes) {
                const uint32_t x = 16u + (uint32_t)o;
                row[o] = (uint8_t)(rr ? listed_dword(L, (uint32_t)o >> 2) >> (8 * (o & 3)) : (L.bv[x >> 5] >> (x & 31u)) & 1u);
            }
        }
    }
}

// deal a new game to half j's env with the whole wave (the one-env `deal`; its stream fields and the dealt deck in
// that env's LDS), then hand it to the half
template <bool PHX>
__device__ __forceinline__ void deal_half(int j, PEnv& e, PairLds& Lj, uint32_t* mt, int64_t env_h, int lane)
{
    WaveMt<PHX> m;
    const int64_t ej = (int64_t)rl((uint32_t)env_h, HW * j) | ((int64_t)rl((uint32_t)((uint64_t)env_h >> 32), HW * j) << 32);
    m.base = mt + ej * MT_WORDS;
    const uint32_t mp = Lj.mpos;
    m.pos = mp & 0xFFFFu;
    m.stale = mp >> 16;
    m.dabs = Lj.mdabs;
    m.key = Lj.mkey;
    Env es;
    deal(es, m, lane);
    Lj.deck[lane] = (uint8_t)(lane < 54 ? es.deck : 0u);
    if (lane < 3) Lj.q[lane] = 0ull;
    if (lane == 0) {
        Lj.mpos = m.pos | m.stale << 16;
        Lj.mdabs = m.dabs;
    }
    if ((lane >> 5) == j) {
        e.h0 = es.h0; e.h1 = es.h1; e.h2 = es.h2;
        e.hcnt = 0;
        e.hid = NO_ACTION;
        e.gw = 0;
        e.sw = NONE << 16 | 0u << 20 | NONE << 24;   // ntrace 0, no greater player, landlord to play, not over
    }
    wave_sync_lds();
}

// k_rollout2's arguments, one struct: the kernel reads them from the kernarg segment through a pointer that every step
// makes opaque again (PairArgsK), so a field is a scalar load where the step uses it. Taken as separate arguments
// (the table alone 24 SGPRs, the outputs 14) they stayed live in SGPRs for the whole kernel, were spilled to VGPR
// lanes and restored with v_readlane -- a VALU instruction -- at every use (153 spilled SGPRs, 417 restores in the
// step loop).
struct PairArgs {
    uint32_t* mt;
    uint32_t* ctl;
    uint32_t* st;
    int64_t n;
    uint64_t seed, t0, env_base;
    cs_traj_out out;
    Tab tb;
    int32_t T, kfl;
};
typedef const __attribute__((address_space(4))) PairArgs* PairArgsK;
// read back through __builtin_amdgcn_kernarg_segment_ptr() (RolloutArgs, cs_skeleton.h): PairArgs must stay
// k_rollout2's ONLY explicit parameter; any new argument goes inside the struct
static_assert(std::is_standard_layout<PairArgs>::value && std::is_trivially_copyable<PairArgs>::value,
              "PairArgs is copied into the kernarg segment bytewise");
static_assert(offsetof(PairArgs, mt) == 0 && alignof(PairArgs) == 8 && sizeof(PairArgs) % 8 == 0,
              "PairArgs: first kernarg at offset 0, 8-byte aligned");

template <bool PHX>
__global__ __launch_bounds__(PBLOCK) __attribute__((amdgpu_waves_per_eu(CS_DDZ_PAIR_MINW)))
void k_rollout2(PairArgs args)
{
    PairArgsK ak = (PairArgsK)__builtin_amdgcn_kernarg_segment_ptr();
    auto arg = [&]() -> const PairArgs& {
        asm volatile("" : "+s"(ak));
        return *(const PairArgs*)ak;
    };
    uint32_t* const mt = args.mt;
    uint32_t* const ctl = args.ctl;
    uint32_t* const st = args.st;
    const int64_t n = args.n;
    const int T = args.T, kfl = args.kfl;
    __shared__ PairLds lds[PWPB][2];
    __shared__ TabLds tl;
    load_tab(tl, args.tb);            // every thread of the block, before any wave leaves
    const int lane = (int)(threadIdx.x & (WAVE - 1)), hl = lane & (HW - 1), hf = lane >> 5;
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const uint32_t bx = xcd_block(blockIdx.x, gridDim.x);   // rows shared by neighbouring blocks meet in one L2
    const int64_t env = (int64_t)bx * (2 * PWPB) + 2 * wid + hf;
    const bool valid = env < n;
    if (!__ballot(valid)) return;
    PairLds& L = lds[wid][hf];
    PEnv e;
    {   // the env's state words (lanes 0..31 of its half: words 0..31, the deck bytes) and stream position
        const uint32_t* srow = st + (valid ? env : 0) * WORDS;
        const uint32_t wlo = valid ? srow[hl] : 0u;
        auto F = [&](uint32_t w) { return hshfl(wlo, lane, w); };
        e.h0 = (uint64_t)F(0) | ((uint64_t)F(1) << 32);
        e.h1 = (uint64_t)F(2) | ((uint64_t)F(3) << 32);
        e.h2 = (uint64_t)F(4) | ((uint64_t)F(5) << 32);
        const uint64_t qv = (uint64_t)F(6 + 2 * (hl % 3)) | ((uint64_t)F(7 + 2 * (hl % 3)) << 32);
        if (hl < 3) L.q[hl] = qv;
        const uint32_t k = (uint32_t)(hl >= 3 ? hl - 3 : 0);   // lanes 3..11: trace entry hl - 3 of the last 9
        const uint32_t hw = F(W_HIST + (k >> 1));
        e.hid = hl >= 3 && hl <= 11 ? (hw >> (16 * (k & 1))) & 0xFFFFu : NO_ACTION;
        e.hcnt = e.hid < (uint32_t)PASS ? args.tb.cnt[e.hid] : 0ull;
        const uint32_t g = F(W_GREATER), c = F(W_CUR);
        e.gw = (g >> 16) | (F(W_HIST + 4) & 0xFFFF0000u);
        const uint32_t winner = valid ? (c >> 8) & 0xFFu : 0u;   // a missing env stays "over" and is never dealt
        e.sw = F(W_NTRACE) | (g & 3u) << 16 | (c & 3u) << 20 | winner << 24;
        const uint8_t* dk = (const uint8_t*)(srow + W_DECK);
        L.deck[hl] = valid ? dk[hl] : 0u;
        L.deck[HW + hl] = valid && hl < 54 - HW ? dk[HW + hl] : 0u;
        if (hl == 0) {
            L.mpos = valid ? ctl[env] & 0x1FFFFu : 0u;   // position | stale << 16
            L.mdabs = 0;
            L.mkey = 0;
            if constexpr (PHX) {
                const uint32_t* b = mt + (valid ? env : 0) * MT_WORDS;
                L.mkey = valid ? (uint64_t)b[0] | (uint64_t)b[1] << 32 : 0ull;
                L.mdabs = valid ? b[2] : 0u;
            }
        }
        wave_sync_lds();
    }
    {
        const uint64_t need = __ballot(valid && e.over());
#pragma unroll 1
        for (int j = 0; j < 2; j++)
            if ((need >> (HW * j)) & 1u) deal_half<PHX>(j, e, lds[wid][j], mt, env, lane);
    }
    uint32_t rr_lane = 0;
    for (int t = 0; t < T; t++) {
        // the lane id made opaque at each step: lane-derived values (LDS and row offsets) are recomputed where they are
        // used instead of hoisted out of the loop -- held, they were spilled, and a spill reload waits on vmcnt, i.e.
        // on every row store the wave has in flight
        int lane_o = lane;
        asm volatile("" : "+v"(lane_o));
        const int lane = lane_o, hl = lane & (HW - 1);
        PairLds& L = lds[wid][lane >> 5];   // (from the opaque lane: its member addresses are not held across steps)
        const PairArgs& A = arg();
        const Tab& tb = A.tb;
        const cs_traj_out& out = A.out;
        const int64_t row = (int64_t)t * n + env;
        uint8_t* const lrow = (uint8_t*)out.legal + row * LB;
        wave_sync_lds();                  // the previous step's row writer has read the list
        if (hl < NZBM) L.nzbm[hl] = 0u;
        wave_sync_lds();
        const PCand cd = pcand(e, tb, tl);
        const Fast fst = fast_issue(e, cd, tb, L, lane, valid && (kfl & 1) == 0);   // kernel flag bit 0: off
        NzSink z{&L, 0u};
        const bool gact = groups2(e, cd, tb, tl, L, lane, valid && !fst.fast);
        Legal lg = scan2(e, cd, tb, tl, L, lane, gact, z);
        build_obs2(e, e.cur(), L, lane);
        if (__ballot(fst.fast)) fast_finish(fst, e.hand(e.cur()), tb, L, lane, lg, z);
        wave_sync_lds();
        // the pass bit (following a play): OR-ed into the list's last dword when that is dword ND - 1, else appended
        const bool pass = valid && !e.over() && !cd.leading();
        if (__ballot(pass)) {
            const uint32_t lastd = z.n > 0u && z.n <= (uint32_t)NZ_CAP ? L.idx[z.n - 1u] : 0xFFFFu;
            const bool merge = lastd == (uint32_t)(ND - 1);
            if (pass && hl == 0) {
                if (merge) L.val[z.n - 1u] |= 1u << (PASS & 31);
                else if (z.n < (uint32_t)NZ_CAP) {
                    L.val[z.n] = 1u << (PASS & 31);
                    L.idx[z.n] = (uint16_t)(ND - 1);
                    atomicOr(&L.nzbm[(ND - 1) >> 5], 1u << ((ND - 1) & 31));
                }
            }
            z.n += pass && !merge ? 1u : 0u;
        }
        const bool ovf = valid && (z.n > (uint32_t)NZ_CAP || (kfl & 2) != 0);   // kernel flag bit 1: every step
        wave_sync_lds();
        // the bitmap's prefix ranks and nonzero words
        const uint32_t bw = hl < NZBM ? L.nzbm[hl] : 0u;
        const uint32_t bpc = (uint32_t)__popc(bw);
        if (hl < NZBM) L.npre[hl] = (uint8_t)(scan32(bpc) - bpc);
        const uint32_t zw = half32(__ballot(bw != 0u), lane);
        // the policy pick: the k-th legal id, k uniform from Philox (pass = the last when following)
        const uint32_t count = lg.total + (cd.leading() ? 0u : 1u);
        if ((t & (HW - 1)) == 0) rr_lane = philox_u32(A.seed, A.env_base + (uint64_t)env, A.t0 + (uint64_t)(t + hl));
        const uint32_t rr = hshfl(rr_lane, lane, (uint32_t)(t & (HW - 1)));
        const uint32_t k = (uint32_t)(((uint64_t)rr * count) >> 32);
        uint32_t a = (uint32_t)PASS;
        if (__ballot(k < lg.total && !ovf)) {
            const uint32_t ka = kth_listed(k, z.n, L, lane);
            if (k < lg.total && !ovf) a = ka;
        }
        if (__ballot(ovf)) {   // the overflow path: the legal scan again, the row straight to HBM
            RowCursor rc{ovf ? lrow : nullptr, 0u, k, 0u, (uint32_t)PASS, pass};
            if (__ballot(ovf && !gact)) groups2(e, cd, tb, tl, L, lane, ovf && !gact);   // kernel flag 2 on fast steps
            scan2(e, cd, tb, tl, L, lane, ovf, rc);
            rc.finish(lane);
            if (ovf && k < lg.total) a = rc.found;
        }
        // the action's table entries, loaded now so that their latency hides behind the row writes
        const bool play = valid && a != (uint32_t)PASS;
        const uint64_t ca = play ? tb.cnt[a] : 0ull;
        const uint32_t ga = play ? (uint32_t)tb.gid[a] : 0u;
        wave_sync_lds();
        write_rows2(L, valid && !(CS_PROF_DDZ & 2) ? (uint8_t*)out.obs + row * OBS : nullptr,
                    valid && !ovf && !(CS_PROF_DDZ & 1) ? lrow : nullptr, zw, lane);
        const uint32_t p = e.cur();
        if (valid) e.apply_with(a, ca, ga, lane, hl, L.q);
        const bool done = valid && e.over();
        if (valid && hl == 0) {
            ((uint8_t*)out.player)[row] = (uint8_t)p;
            ((int16_t*)out.action)[row] = (int16_t)a;
            float r[3] = {0.f, 0.f, 0.f};
            if (done) payoffs(e.winner(), r);
            float* o = (float*)out.reward + row * P;
            o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
            ((uint8_t*)out.done)[row] = (uint8_t)done;
        }
        const uint64_t fin = __ballot(done);
        if (fin) {
            if (out.final_obs) {   // Env.run's final state of every player (envs/env.py:161-164)
                for (uint32_t q = 0; q < (uint32_t)P; q++) {
                    wave_sync_lds();
                    build_obs2(e, q, L, lane);
                    wave_sync_lds();
                    write_rows2(L, done ? (uint8_t*)out.final_obs + (row * P + q) * OBS : nullptr, nullptr, 0u, lane);
                }
            }
#pragma unroll 1
            for (int j = 0; j < 2; j++)
                if ((fin >> (HW * j)) & 1u) deal_half<PHX>(j, e, lds[wid][j], mt, env, lane);
        }
    }
    // the state back: words 0..19 (lanes 0..4 of the half, 16 B each), the deck bytes, the stream position
    const uint32_t h01 = hshfl(e.hid, lane, 3u + 2u * (uint32_t)(hl - 3)) | hshfl(e.hid, lane, 4u + 2u * (uint32_t)(hl - 3)) << 16;
    const uint32_t hw0 = hshfl(h01, lane, 3u), hw1 = hshfl(h01, lane, 4u), hw2 = hshfl(h01, lane, 5u),
                   hw3 = hshfl(h01, lane, 6u), hw4 = hshfl(h01, lane, 7u);
    if (valid) {
        if (hl == 0) {
            uint4* o = (uint4*)(st + env * WORDS);
            o[0] = make_uint4((uint32_t)e.h0, (uint32_t)(e.h0 >> 32), (uint32_t)e.h1, (uint32_t)(e.h1 >> 32));
            const uint64_t q0 = L.q[0], q1 = L.q[1], q2 = L.q[2];
            o[1] = make_uint4((uint32_t)e.h2, (uint32_t)(e.h2 >> 32), (uint32_t)q0, (uint32_t)(q0 >> 32));
            o[2] = make_uint4((uint32_t)q1, (uint32_t)(q1 >> 32), (uint32_t)q2, (uint32_t)(q2 >> 32));
            o[3] = make_uint4(hw0, hw1, hw2, hw3);
            o[4] = make_uint4((hw4 & 0xFFFFu) | (e.gw & 0xFFFF0000u), e.ntrace(),
                              e.greater() | (e.gw & 0xFFFFu) << 16, e.cur() | e.winner() << 8);
            ctl[env] = L.mpos | (PHX ? CTL_PHX : 0u);
            if constexpr (PHX) mt[env * MT_WORDS + 2] = L.mdabs;
        }
        uint8_t* db = (uint8_t*)(st + env * WORDS + W_DECK);
        db[hl] = L.deck[hl];
        db[HW + hl] = L.deck[HW + hl];
    }
}

// Test hook (cs_debug_ddz_legal): the legal set of player 0 holding `counts` -- leading when prev < 0, else following
// another player's play `prev` -- through the same cand_of / build_legal the step and rollout kernels run (reference:
// Judger.playable_cards_from_hand, judger.py:124-258, and get_gt_cards, utils.py:225-262, pass included)
__global__ __launch_bounds__(BLOCK) void k_debug_legal(const uint8_t* __restrict__ counts, const int32_t* __restrict__ prev,
                                                       int64_t n, uint8_t* legal, Tab tb)
{
    __shared__ WaveLds lds[WPB];
    __shared__ TabLds tl;
    load_tab(tl, tb);
    const Ctx c = ctx_of(n);
    if (!c.valid) return;
    const uint32_t k = c.lane < 15 ? counts[c.env * 15 + c.lane] : 0u;
    uint64_t h = 0;
#pragma unroll
    for (int r = 0; r < 15; r++) h |= (uint64_t)(rl(k, r) & 15u) << (4 * r);
    const int32_t pv = prev[c.env];
    Env e;
    e.h0 = h; e.h1 = 0; e.h2 = 0; e.q0 = 0; e.q1 = 0; e.q2 = 0;
    e.hw0 = e.hw1 = e.hw2 = e.hw3 = e.hw4 = 0xFFFFFFFFu;
    e.ntrace = 0;
    e.hcnt = 0;
    e.deck = 0;
    e.cur = 0;
    e.winner = NONE;
    const bool lead = pv < 0 || pv >= PASS;
    e.greater = lead ? NONE : 1u;
    e.gplay = lead ? 0u : (uint32_t)pv;
    e.ggrp = lead ? 0u : (uint32_t)tb.gid[pv];
    cs_step_out o{nullptr, legal, nullptr, nullptr, nullptr};
    emit_state(e, 0u, tb, tl, lds[c.wid], c.lane, c.env, o);
}

// _cards2array of action ids (envs/doudizhu.py:136-142 get_action_feature; pass and invalid ids -> zeros), one
// thread per id, 27 two-byte stores per 54-byte row
__global__ __launch_bounds__(BLOCK) void k_features(const int32_t* __restrict__ ids, int64_t count, uint8_t* out, Tab tb)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= count) return;
    const int32_t id = ids[i];
    const uint64_t bits = cards_bits(id >= 0 && id < PASS ? tb.cnt[id] : 0ull);
    uint16_t* o = (uint16_t*)(out + i * 54);
#pragma unroll
    for (int k = 0; k < 27; k++) o[k] = (uint16_t)(((bits >> (2 * k)) & 1u) | (((bits >> (2 * k + 1)) & 1u) << 8));
}

static inline dim3 grid_of(int64_t n) { return dim3((unsigned)((n + WPB - 1) / WPB)); }

hipError_t launch_features(const Buffers& b, const int32_t* ids, int64_t count, uint8_t* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_features, dim3((unsigned)((count + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, ids, count, out,
                       *(const Tab*)b.table);
    return hipGetLastError();
}

hipError_t launch_debug_legal(const Buffers& b, const uint8_t* counts, const int32_t* prev, int64_t n,
                              uint8_t* legal, hipStream_t s)
{
    hipLaunchKernelGGL(k_debug_legal, grid_of(n), dim3(BLOCK), 0, s, counts, prev, n, legal, *(const Tab*)b.table);
    return hipGetLastError();
}

hipError_t launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
    if (b.rng_mode == CS_RNG_PHILOX)
        hipLaunchKernelGGL(k_reset<true>, grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, o, *(const Tab*)b.table,
                           b.rec);
    else
        hipLaunchKernelGGL(k_reset<false>, grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, o, *(const Tab*)b.table,
                           b.rec);
    return hipGetLastError();
}
hipError_t launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
    if (b.rng_mode == CS_RNG_PHILOX)
        hipLaunchKernelGGL(k_step<true>, grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, a, o,
                           *(const Tab*)b.table, b.rec);
    else
        hipLaunchKernelGGL(k_step<false>, grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, a, o,
                           *(const Tab*)b.table, b.rec);
    return hipGetLastError();
}
hipError_t launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(k_observe, grid_of(b.n), dim3(BLOCK), 0, s, b.state, b.n, p, o, *(const Tab*)b.table, b.rec);
    return hipGetLastError();
}
hipError_t launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                          const cs_traj_out& o, hipStream_t s)
{
    const dim3 g((unsigned)((b.n + 2 * PWPB - 1) / (2 * PWPB)));
    const PairArgs a{b.mt, b.ctl, b.state, b.n, seed, t0, env_base, o, *(const Tab*)b.table, T, b.serial_refill};
    if (b.rng_mode == CS_RNG_PHILOX) hipLaunchKernelGGL(k_rollout2<true>, g, dim3(PBLOCK), 0, s, a);
    else hipLaunchKernelGGL(k_rollout2<false>, g, dim3(PBLOCK), 0, s, a);
    return hipGetLastError();
}

}  // namespace ddz
}  // namespace cs
