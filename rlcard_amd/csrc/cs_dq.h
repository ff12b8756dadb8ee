// cs_dq.h -- the deal queue of the lane-per-env games whose deal depends only on the env's stream (heads-up hold'em,
// cs_limit.h, cs_nolimit.h): deals drawn ahead, in stream order, popped by the game resets. Shared by the rollout
// skeleton (cs_skeleton.h) and the CFR kernel (cs_cfr.hip), which resets through the same queue.
#pragma once
#include <type_traits>
#include "cs_device.h"

namespace cs {

// ---- the deal queue: q = the env's queue words, `stride` apart (state in HBM: n; LDS copy: 1) ------
template <class G, class = void>
struct DqOf {
    static constexpr int value = 0, words = 0, cb = 0, xb = 0;
};
template <class G>
struct DqOf<G, std::void_t<decltype(G::DQ)>> {
    static constexpr int value = G::DQ, words = G::DQ > 0 ? 1 + 2 * G::DQ : 0;
    // header fields (cs_limit.h): count bits, then head bits (cb - 1), from bit xb the dealer bits and draws[8:7]
    static constexpr int cb = G::DQ == 8 ? 4 : G::DQ == 4 ? 3 : 2, xb = 2 * cb - 1;
};

// the queue words of one env, `stride` apart (state in HBM: n; the rollout's LDS copy: 1)
struct DqMem {
    uint32_t* p;
    int64_t stride;
    __device__ __forceinline__ uint32_t get(uint32_t i) const { return p[i * stride]; }
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) { p[i * stride] = v; }
};

// draw the env's next deal into its queue (the caller checks for room)
template <class G, class Rng, class Q>
__device__ __forceinline__ void dq_push(const G& g, Rng& rng, Q& q)
{
    constexpr int CB = DqOf<G>::cb, XB = DqOf<G>::xb;
    constexpr uint32_t CM = (1u << CB) - 1u, HM = (uint32_t)G::DQ - 1u;
    uint32_t hdr = q.get(0);
    const uint32_t cnt = hdr & CM, head = (hdr >> CB) & HM, p0 = rng.pos;
    uint32_t e0, e1;
    g.make_deal(rng, hdr, e0, e1);
    uint32_t d = rng.pos >= p0 ? rng.pos - p0 : rng.pos + (uint32_t)RING - p0;
    d = d < 511u ? d : 511u;
    const uint32_t slot = (head + cnt) & HM, hi = (uint32_t)XB + 2u + 2u * slot;
    q.set(1 + 2 * slot, e0 | (d & 127u) << 25);
    q.set(2 + 2 * slot, e1);
    q.set(0, (hdr & ~CM & ~(3u << hi)) | (d >> 7) << hi | (cnt + 1u));
}

// Game.init_game: the oldest queued deal, or a deal drawn now when the queue is empty
template <class G, class Rng, class Q>
__device__ __forceinline__ void dq_reset(G& g, Rng& rng, Q& q)
{
    constexpr int CB = DqOf<G>::cb, XB = DqOf<G>::xb;
    constexpr uint32_t CM = (1u << CB) - 1u, HM = (uint32_t)G::DQ - 1u;
    uint32_t hdr = q.get(0), e0, e1;
    const uint32_t cnt = hdr & CM, head = (hdr >> CB) & HM;
    if (cnt) {
        e0 = q.get(1 + 2 * head);
        e1 = q.get(2 + 2 * head);
        hdr = (hdr & ~((1u << XB) - 1u)) | (cnt - 1u) | ((head + 1u) & HM) << CB;
    } else {
        g.make_deal(rng, hdr, e0, e1);
    }
    q.set(0, hdr);
    g.reset_from(e0, e1);
}


// Game.init_game through the env's queue in HBM (its words after the game words, `n` apart) where the game has one
template <class G, class Rng>
__device__ __forceinline__ void game_reset_hbm(G& g, Rng& rng, uint32_t* st, int64_t n, int64_t env)
{
    if constexpr (DqOf<G>::value > 0) {
        DqMem q{st + (int64_t)G::GW * n + env, n};
        dq_reset(g, rng, q);
    } else {
        g.reset(rng);
    }
}

}  // namespace cs
