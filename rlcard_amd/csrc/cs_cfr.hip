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
// player per iteration, the reference agent) is bit-exact; with more envs the table updates are fp64 atomics
// (summation order varies run to run).
#include "cs_device.h"
#include "cs_ring.h"
#include "cs_engine.h"
#include "cs_leduc.h"

#pragma clang fp contract(off)

namespace cs {

namespace {

constexpr int NA = 4;
constexpr int MAXD = 12;   // deepest Leduc betting line: 8 actions (two raises per round) + root

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

__device__ __forceinline__ void add_f64(double* p, double v, bool atomic)
{
    if (atomic) atomicAdd(p, v);
    else *p = *p + v;
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

// cfr_agent.py:84-97: regrets and average policy at the traversing player's node
__device__ __forceinline__ void record(const Frame& f, double iteration, const CfrTables& t, bool atomic)
{
    const double pp = f.cp ? f.pr1 : f.pr0;
    const double cf = f.cp == 0 ? 1.0 * f.pr1 : f.pr0 * 1.0;
    const double us = f.cp ? f.su1 : f.su0;
    if (!(t.flags[f.idx] & 2u)) atomicOr(&t.flags[f.idx], 2u);
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (!((f.legal >> a) & 1u)) continue;
        const double regret = cf * (f.au[a] - us);
        add_f64(&t.regrets[f.idx * NA + a], regret, atomic);
        add_f64(&t.avg[f.idx * NA + a], (iteration * pp) * f.ap[a], atomic);
    }
}

// the whole tree under the lane's current deal, for traversing player `player`
__device__ void traverse(const Leduc& root, int player, double iteration, const CfrTables& t, bool atomic)
{
    Frame S[MAXD];
    int d = 0;
    enter(S[0], root, 1.0, 1.0, t);
    RingLane<> none;   // Leduc::step draws nothing
    none.init(nullptr, 2u << 12);
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
            if ((int)f.cp == player) record(f, iteration, t, atomic);
            const double u0 = f.su0, u1 = f.su1;
            if (d == 0) break;
            d--;
            deliver(S[d], (int)S[d].next - 1, u0, u1);
        }
    }
}

__global__ __launch_bounds__(256) void k_cfr_iteration(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                       CfrTables t, double iteration)
{
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t env = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = env < n;
    const bool atomic = n > 1;
    RingLane<> m;
    if (valid) m.init(mt + env * RING_ENV_WORDS, ctl[env]);
    else m.init(mt, 2u << 12);   // never needs a refill
    Leduc g;
    g.blank();
    if (valid) g.load(st, n, env);
    for (int p = 0; p < 2; p++) {
        if (valid) g.reset(m);          // env.reset(): a new deal from the env's own stream
        ring_refill_wave(m, lane);      // all 64 lanes
        if (valid) traverse(g, p, iteration, t, atomic);
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

}  // namespace

hipError_t launch_cfr(const Buffers& b, int32_t iterations, int64_t iteration0, const CfrTables& t, hipStream_t s)
{
    const dim3 grid((unsigned)((b.n + 255) / 256)), ugrid((CFR_NI + 255) / 256);
    for (int32_t it = 0; it < iterations; it++) {
        hipLaunchKernelGGL(k_cfr_iteration, grid, dim3(256), 0, s, b.mt, b.ctl, b.state, b.n, t,
                           (double)(iteration0 + it + 1));
        hipLaunchKernelGGL(k_cfr_update, ugrid, dim3(256), 0, s, t);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace cs
