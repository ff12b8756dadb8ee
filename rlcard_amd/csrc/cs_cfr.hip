// cs_cfr.hip -- chance-sampling CFR on Leduc Hold'em (rlcard/agents/cfr_agent.py) over a handle's envs.
//
// One lane per env. Per iteration (reference train(), :30-43), for each player: the env deals a new game from its
// own MT19937 stream (Env.reset, the same draws as cs_reset) and the lane walks the whole betting tree under that
// deal depth-first with an explicit stack of saved game states -- the reference's env.step / env.step_back recursion
// (traverse_tree, :45-98) -- then a second kernel applies regret matching to every infoset with regrets (update_policy,
// :100-123). The betting tree's shape does not depend on the cards, so the lanes of a wave walk it in lockstep.
// Tables (fp64, device, [CFR_NI][4]): policy, average_policy, regrets, indexed by the Leduc observation the
// reference keys its dicts with (envs/leducholdem.py:41-71):
//   ((hand * 4 + public + 1 (0 = none)) * 15 + my chips) * 15 + others' chips
// flags[CFR_NI] u32: bit 0 = key present in policy, bit 1 = key present in regrets / average_policy.
// Every fp64 operation follows the reference's order and nothing is contracted into FMAs, so one env (one deal per
// player per iteration, the reference agent) is bit-exact.
// Batched mode (n envs, one deal each per player per iteration; oracle/or_cfr.c): the table sums must come out in one
// fixed order -- per iteration, player 0's pass then player 1's, envs ascending, each deal's nodes in traversal
// (post-)order, as the oracle adds them. Each lane writes its deal's contributions as records (infoset | legal bits
// key, regret and average-policy terms) at (pass, env, node) slots; a stable radix sort on the 12-bit infoset groups
// them per infoset keeping that order, and one thread per (infoset, action) adds its segment sequentially. Same
// bits every run, equal to the oracle's at any iteration count.
#include <hipcub/hipcub.hpp>
#include "cs_device.h"
#include "cs_ring.h"
#include "cs_engine.h"
#include "cs_leduc.h"
#include "cs_dq.h"

#pragma clang fp contract(off)

namespace cs {

namespace {

constexpr int NA = 4;
constexpr int MAXD = 12;   // deepest Leduc betting line: 8 actions (two raises per round) + root
// records per (pass, env): the traversing player's decision nodes of one deal's betting tree -- 18 for either seat
// (the tree's shape does not depend on the cards); slots past the node count hold REC_NONE keys
constexpr int REC_CAP = 24;
constexpr uint32_t REC_NONE = 0xFFFu;   // sorts after every infoset (< 2700)

// batched-mode record buffers: key u16 (infoset | legal << 12), the regret and average-policy terms of the 4 actions
struct Recs {
    uint16_t* key;
    double* val;      // [slot][8]: regret[4], avg[4]
    int64_t n;        // envs
    int pass;
};

struct Frame {
    uint32_t w[2];        // packed Leduc state (Leduc::store with n = 1)
    uint32_t cp, legal, next, idx;
    double pr0, pr1;      // reach probabilities (probs)
    double su0, su1;      // state utility accumulated over the children visited so far
    double au[NA];        // action utilities of the acting player
    double ap[NA];        // action probabilities after remove_illegal
};

__device__ __forceinline__ int leduc_infoset(const Leduc& g, int p)
{
    const int hand = (p ? g.h1 : g.h0) >> 1, pub = g.rc >= 1 ? (g.pub >> 1) + 1 : 0;
    const int my = p ? g.in1 : g.in0, op = g.in0 + g.in1 - my;
    return ((hand * 4 + pub) * 15 + my) * 15 + op;
}

// traverse_tree entry for a non-terminal node: acting player, infoset, legal ids, remove_illegal(policy row)
__device__ __forceinline__ void enter(Frame& f, const Leduc& g, double pr0, double pr1, const CfrTables& t)
{
    uint32_t w[2];
    g.store(w, 1, 0);
    f.w[0] = w[0];
    f.w[1] = w[1];
    f.cp = (uint32_t)g.current();
    f.legal = g.legal();
    f.next = 0;
    f.idx = (uint32_t)leduc_infoset(g, (int)f.cp);
    f.pr0 = pr0;
    f.pr1 = pr1;
    f.su0 = 0.0;
    f.su1 = 0.0;
    // action_probs (cfr_agent.py:125-146): unseen keys read the uniform row the host initialised and are inserted
    if (!(t.flags[f.idx] & 1u)) atomicOr(&t.flags[f.idx], 1u);
    double p[NA];
    int nl = 0;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        const bool l = (f.legal >> a) & 1u;
        p[a] = l ? t.policy[f.idx * NA + a] : 0.0;
        nl += l;
        f.au[a] = 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < NA; a++) s = s + p[a];
#pragma unroll
    for (int a = 0; a < NA; a++) {   // utils.py:181-198 remove_illegal
        if (s == 0.0) f.ap[a] = ((f.legal >> a) & 1u) ? 1.0 / (double)nl : 0.0;
        else f.ap[a] = p[a] / s;
    }
}

__device__ __forceinline__ void deliver(Frame& f, int a, double u0, double u1)
{
    f.su0 = f.su0 + f.ap[a] * u0;
    f.su1 = f.su1 + f.ap[a] * u1;
    f.au[a] = f.cp ? u1 : u0;
}

// cfr_agent.py:84-97: regrets and average policy at the traversing player's node; batched mode writes the terms as
// the lane's next record instead of adding them
__device__ __forceinline__ void record(const Frame& f, double iteration, const CfrTables& t, const Recs& rc,
                                       bool batched, int64_t slot)
{
    const double pp = f.cp ? f.pr1 : f.pr0;
    const double cf = f.cp == 0 ? 1.0 * f.pr1 : f.pr0 * 1.0;
    const double us = f.cp ? f.su1 : f.su0;
    if (!(t.flags[f.idx] & 2u)) atomicOr(&t.flags[f.idx], 2u);
    if (batched) {
        double* v = rc.val + slot * 8;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            const bool l = (f.legal >> a) & 1u;
            v[a] = l ? cf * (f.au[a] - us) : 0.0;
            v[NA + a] = l ? (iteration * pp) * f.ap[a] : 0.0;
        }
        rc.key[slot] = (uint16_t)(f.idx | (f.legal << 12));
        return;
    }
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (!((f.legal >> a) & 1u)) continue;
        const double regret = cf * (f.au[a] - us);
        t.regrets[f.idx * NA + a] = t.regrets[f.idx * NA + a] + regret;
        t.avg[f.idx * NA + a] = t.avg[f.idx * NA + a] + (iteration * pp) * f.ap[a];
    }
}

// the whole tree under the lane's current deal, for traversing player `player` (rc: batched mode, the lane's
// records start at slot0)
__device__ void traverse(const Leduc& root, int player, double iteration, const CfrTables& t, const Recs& rc,
                         bool batched, int64_t slot0)
{
    Frame S[MAXD];
    int d = 0;
    int nrec = 0;
    enter(S[0], root, 1.0, 1.0, t);
    RingLane<> none;   // Leduc::step draws nothing
    none.init(nullptr, CTL_IDLE);
    while (true) {
        Frame& f = S[d];
        const uint32_t rem = f.legal & ~((1u << f.next) - 1u);
        if (rem) {
            const int a = __builtin_ctz(rem);
            f.next = (uint32_t)a + 1u;
            Leduc c;
            c.load(f.w, 1, 0);
            c.step(a, none);
            double p0 = f.pr0, p1 = f.pr1;
            if (f.cp == 0) p0 = p0 * f.ap[a];
            else p1 = p1 * f.ap[a];
            if (c.is_over()) {
                float r[2];
                c.payoffs(r);
                deliver(f, a, (double)r[0], (double)r[1]);
            } else {
                d++;
                enter(S[d], c, p0, p1, t);
            }
        } else {
            if ((int)f.cp == player && nrec < REC_CAP) record(f, iteration, t, rc, batched, slot0 + nrec++);
            const double u0 = f.su0, u1 = f.su1;
            if (d == 0) break;
            d--;
            deliver(S[d], (int)S[d].next - 1, u0, u1);
        }
    }
    if (batched)
        for (int k = nrec; k < REC_CAP; k++) rc.key[slot0 + k] = (uint16_t)REC_NONE;
}

__global__ __launch_bounds__(256) void k_cfr_iteration(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                       CfrTables t, double iteration, Recs recs)
{
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = env < n;
    const bool batched = n > 1;
    RingLane<> m;
    if (valid) m.init(mt + env * RING_ENV_WORDS, ctl[env]);
    else m.init(mt, CTL_IDLE);   // never needs a refill
    Leduc g;
    g.blank();
    if (valid) g.load(st, n, env);
    for (int p = 0; p < 2; p++) {
        if (valid) game_reset_hbm(g, m, st, n, env);   // env.reset(): the next deal of the env's stream (its deal
                                                        // queue first, cs_dq.h)
        ring_refill_wave(m, lane);      // all 64 lanes
        if (valid) traverse(g, p, iteration, t, recs, batched, ((int64_t)p * n + env) * REC_CAP);
    }
    if (valid) {
        g.store(st, n, env);            // the env is left at the last deal's root (every step stepped back)
        ctl[env] = m.ctl_word();
    }
}

// update_policy (cfr_agent.py:100-123): regret matching for every key of regrets
__global__ void k_cfr_update(CfrTables t)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= CFR_NI || !(t.flags[i] & 2u)) return;
    double r[NA], pos = 0.0;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        r[a] = t.regrets[i * NA + a];
        if (r[a] > 0) pos = pos + r[a];
    }
#pragma unroll
    for (int a = 0; a < NA; a++) {
        double x = 1.0 / NA;
        if (pos > 0) {
            x = r[a] / pos;
            x = x > 0.0 ? x : 0.0;
        }
        t.policy[i * NA + a] = x;
    }
    t.flags[i] |= 1u;
}

__global__ void k_iota(uint32_t* v, int64_t m)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) v[i] = (uint32_t)i;
}

// segment [seg[2 k], seg[2 k + 1]) of the sorted keys holds infoset k's records (empty segments stay 0, 0)
__global__ void k_cfr_segments(const uint16_t* __restrict__ key, int64_t m, int32_t* seg)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t k = key[i] & 0xFFFu, kp = i > 0 ? key[i - 1] & 0xFFFu : 0xFFFFu;
    const uint32_t kn = i + 1 < m ? key[i + 1] & 0xFFFu : 0xFFFFu;
    if (k >= (uint32_t)CFR_NI) return;
    if (k != kp) seg[2 * k] = (int32_t)i;
    if (k != kn) seg[2 * k + 1] = (int32_t)i + 1;
}

// one thread per (infoset, action): its records in (pass, env, node) order, added one by one as the oracle does
__global__ void k_cfr_reduce(const uint16_t* __restrict__ key, const uint32_t* __restrict__ slot,
                             const double* __restrict__ val, const int32_t* __restrict__ seg, CfrTables t)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= CFR_NI * NA) return;
    const int idx = i / NA, a = i % NA;
    const int32_t lo = seg[2 * idx], hi = seg[2 * idx + 1];
    if (lo >= hi) return;
    double r = t.regrets[i], v = t.avg[i];
    for (int32_t j = lo; j < hi; j++) {
        if (!((key[j] >> (12 + a)) & 1u)) continue;
        const double* x = val + (int64_t)slot[j] * 8;
        r = r + x[a];
        v = v + x[NA + a];
    }
    t.regrets[i] = r;
    t.avg[i] = v;
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

hipError_t launch_cfr(const Buffers& b, int32_t iterations, int64_t iteration0, const CfrTables& t, CfrScratch* sc,
                      hipStream_t s)
{
    const dim3 grid((unsigned)((b.n + 255) / 256)), ugrid((CFR_NI + 255) / 256);
    Recs recs{nullptr, nullptr, b.n, 0};
    uint16_t *key_out = nullptr;
    uint32_t *slot_in = nullptr, *slot_out = nullptr;
    int32_t* seg = nullptr;
    void* sort_tmp = nullptr;
    size_t sort_bytes = 0;
    const int64_t m = 2 * b.n * REC_CAP;   // records per iteration
    hipError_t e;
    if (b.n > 1) {
        if (m > (int64_t)INT32_MAX) return hipErrorInvalidValue;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint16_t*)nullptr, (uint16_t*)nullptr,
                                               (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)m, 0, 12, s);
        if (e != hipSuccess) return e;
        const size_t o_val = 0, o_key = al256(o_val + (size_t)m * 64), o_kout = al256(o_key + (size_t)m * 2),
                     o_sin = al256(o_kout + (size_t)m * 2), o_sout = al256(o_sin + (size_t)m * 4),
                     o_seg = al256(o_sout + (size_t)m * 4), o_tmp = al256(o_seg + (size_t)CFR_NI * 8),
                     total = o_tmp + sort_bytes;
        const bool fresh = sc->bytes < total;
        if (fresh) {
            if (sc->mem) (void)hipFree(sc->mem);
            sc->mem = nullptr;
            sc->bytes = 0;
            if ((e = hipMalloc(&sc->mem, total)) != hipSuccess) return e;
            sc->bytes = total;
        }
        uint8_t* base = (uint8_t*)sc->mem;
        recs.val = (double*)(base + o_val);
        recs.key = (uint16_t*)(base + o_key);
        key_out = (uint16_t*)(base + o_kout);
        slot_in = (uint32_t*)(base + o_sin);
        slot_out = (uint32_t*)(base + o_sout);
        seg = (int32_t*)(base + o_seg);
        sort_tmp = base + o_tmp;
        hipLaunchKernelGGL(k_iota, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, slot_in, m);
    }
    for (int32_t it = 0; it < iterations; it++) {
        hipLaunchKernelGGL(k_cfr_iteration, grid, dim3(256), 0, s, b.mt, b.ctl, b.state, b.n, t,
                           (double)(iteration0 + it + 1), recs);
        if (b.n > 1) {
            if ((e = hipMemsetAsync(seg, 0, (size_t)CFR_NI * 8, s)) != hipSuccess) return e;
            size_t tb = sort_bytes;
            e = hipcub::DeviceRadixSort::SortPairs(sort_tmp, tb, (const uint16_t*)recs.key, key_out,
                                                   (const uint32_t*)slot_in, slot_out, (int)m, 0, 12, s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k_cfr_segments, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, key_out, m, seg);
            hipLaunchKernelGGL(k_cfr_reduce, dim3((CFR_NI * NA + 63) / 64), dim3(64), 0, s, key_out, slot_out,
                               recs.val, seg, t);
        }
        hipLaunchKernelGGL(k_cfr_update, ugrid, dim3(256), 0, s, t);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace cs
