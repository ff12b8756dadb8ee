// cs_dmc.hip -- the DMC learner's side of the rollout, on the device:
//
//   actor buffers  rlcard/agents/dmc_agent/utils.py:97-163 (act): every (env, player) keeps its stream of
//                  transitions -- state = the obs the player acted on (int8), action = Env.get_action_feature of its
//                  action (int8), target = the player's payoff of that game on every one of its rows, done / episode
//                  return on its last row of the game -- and hands out T-row chunks once more than T rows of finished
//                  games are queued (`while size[p] > T`). Here each (env, player) stream lives in a ring of `slots`
//                  chunks in HBM; k_dmc_index assigns ring rows to a trajectory's rows (one lane per env, in time
//                  order: the stream order) and back-fills the targets when a game ends, k_dmc_rows copies the obs
//                  rows and writes the action features (one thread per 4 bytes / per row: coalesced), and the newly
//                  ready chunks are listed in stream order (count pass + prefix sum + fill).
//   get_batch      utils.py:33-46: chunks of one player stacked along dim 1 -> [T][B][...] (k_dmc_gather).
//   Q scoring      dmc_agent/model.py:21-43,91-110 (DMCNet over [obs, action feature] for every legal action): the
//                  first layer splits into W_obs . obs (one GEMM per state, torch / hipBLASLt) + W_act . feature
//                  (per legal action); k_dmc_layer1 fuses the gather of the state's projection, the action part (a
//                  sum of the weight rows of the feature's set bits: one-hot ids or DouDizhu's 54-bit card code),
//                  bias and ReLU. The 512-wide hidden layers are plain GEMMs (torch, hipBLASLt). k_dmc_select is the
//                  per-state argmax (np.argmax: first maximum) with the epsilon-greedy branch of DMCAgent.step.
// All streaming integer / fp32 work, HBM-bound: no MFMA in these kernels (the GEMMs between them are hipBLASLt's).
#include <hipcub/hipcub.hpp>
#include "cs_device.h"
#include "cs_engine.h"
#include "cs_doudizhu.h"

namespace cs {

constexpr int DBLOCK = 256;

// ring row of stream index w of (env, player) stream s: chunk w / Tc in slot (w / Tc) % R
__device__ __forceinline__ int64_t ring_row(int64_t s, int64_t w, int Tc, int R)
{
    const int64_t k = w / Tc;
    return (s * R + k % R) * Tc + (w - k * Tc);
}

// One lane per env, rows in time order. player >= P marks a row that is not a transition (skipped).
__global__ __launch_bounds__(DBLOCK) void k_dmc_index(const uint8_t* __restrict__ player,
                                                      const uint8_t* __restrict__ done,
                                                      const float* __restrict__ reward, int T, int64_t n, int P,
                                                      int Tc, int R, int64_t* ctr, int64_t* gstart,
                                                      const int64_t* __restrict__ emitted, int64_t* dst, float* tgt,
                                                      float* ret, uint8_t* dne, int32_t* counts, uint32_t* flag)
{
    const int64_t e = (int64_t)blockIdx.x * DBLOCK + threadIdx.x;
    if (e >= n) return;
    const float nan = __builtin_nanf("");
    for (int t = 0; t < T; t++) {
        const int64_t row = (int64_t)t * n + e;
        const int p = player[row];
        if (p >= P) {
            dst[row] = -1;
            continue;
        }
        const int64_t s = e * P + p, w = ctr[s];
        if (w - emitted[s] * Tc >= (int64_t)R * Tc) {
            // would overwrite a chunk not yet handed out: the row is dropped and not counted (ctr stays), so no chunk
            // holding it is ever listed as ready; the stream is broken from here on and the host raises (flag bit 0)
            dst[row] = -1;
            atomicOr(flag, 1u);
        } else {
            const int64_t r = ring_row(s, w, Tc, R);
            dst[row] = r;
            tgt[r] = nan;   // filled when the game ends
            ret[r] = 0.f;
            dne[r] = 0;
            ctr[s] = w + 1;
        }
        if (done[row]) {   // the game's rows of every player get its payoff (utils.py:121-128)
            for (int q = 0; q < P; q++) {
                const int64_t sq = e * P + q, end = ctr[sq];
                const float pay = reward[row * P + q];
                for (int64_t i = gstart[sq]; i < end; i++) {   // rows [gstart, ctr) are all in the ring
                    const int64_t r = ring_row(sq, i, Tc, R);
                    tgt[r] = pay;
                    if (i == end - 1) {
                        dne[r] = 1;
                        ret[r] = pay;
                    }
                }
                gstart[sq] = end;
            }
        }
    }
    for (int q = 0; q < P; q++) {   // chunks ready: the reference emits while the finished rows exceed T
        const int64_t sq = e * P + q, fin = gstart[sq];
        const int64_t ready = fin > 0 ? (fin - 1) / Tc : 0;
        counts[sq] = (int32_t)(ready - emitted[sq]);
    }
}

// ready chunk ids (stream s, chunk k -> s * R + k % R) in (env, player, chunk) order; emitted advances by the ids
// actually listed: chunks past `cap` stay queued for the next fill (flag bit 1)
__global__ __launch_bounds__(DBLOCK) void k_dmc_ready(const int32_t* __restrict__ counts,
                                                      const int64_t* __restrict__ offsets, int64_t streams, int R,
                                                      int64_t* emitted, int64_t* ready, int64_t cap, int64_t* nready,
                                                      uint32_t* flag)
{
    const int64_t s = (int64_t)blockIdx.x * DBLOCK + threadIdx.x;
    if (s == 0) {
        const int64_t total = offsets[streams];
        *nready = total < cap ? total : cap;
        if (total > cap) atomicOr(flag, 2u);
    }
    if (s >= streams) return;
    const int64_t o = offsets[s];
    const int64_t room = cap - o;
    const int c = room <= 0 ? 0 : (counts[s] < room ? counts[s] : (int)room);
    const int64_t k0 = emitted[s];
    for (int i = 0; i < c; i++) ready[o + i] = s * R + (k0 + i) % R;
    emitted[s] = k0 + c;
}

// obs rows -> ring state rows: one thread per 4 bytes of a row (consecutive threads, consecutive bytes)
__global__ __launch_bounds__(DBLOCK) void k_dmc_rows(const uint8_t* __restrict__ obs, const int64_t* __restrict__ dst,
                                                     int64_t rows, int O, int8_t* st)
{
    const int q4 = (O + 3) / 4;
    const int64_t i = (int64_t)blockIdx.x * DBLOCK + threadIdx.x;
    if (i >= rows * q4) return;
    const int64_t row = i / q4;
    const int c = (int)(i - row * q4) * 4;
    const int64_t r = dst[row];
    if (r < 0) return;
    const uint8_t* src = obs + row * O + c;
    int8_t* d = st + r * O + c;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (c + k < O) d[k] = (int8_t)src[k];
}

// Env.get_action_feature of each row's action into its ring row: one-hot of num_actions (envs/env.py:217-226), or
// DouDizhu's _cards2array of the combo (envs/doudizhu.py:136-142; pass -> zeros), one thread per row
__global__ __launch_bounds__(DBLOCK) void k_dmc_features(const void* __restrict__ action, int abytes,
                                                         const int64_t* __restrict__ dst, int64_t rows, int F, int A,
                                                         const uint64_t* __restrict__ ddz_cnt, int8_t* act)
{
    const int64_t row = (int64_t)blockIdx.x * DBLOCK + threadIdx.x;
    if (row >= rows) return;
    const int64_t r = dst[row];
    if (r < 0) return;
    const int a = abytes == 1 ? (int)((const uint8_t*)action)[row] : (int)((const int16_t*)action)[row];
    int8_t* d = act + r * F;
    if (ddz_cnt) {
        const uint64_t bits = ddz::cards_bits(a >= 0 && a < ddz::PASS ? ddz_cnt[a] : 0ull);
        for (int k = 0; k < F; k++) d[k] = (int8_t)((bits >> k) & 1u);
    } else {
        for (int k = 0; k < F; k++) d[k] = (int8_t)(k == a);
    }
}

// get_batch: chunk j of the list -> column j of [Tc][B][...]
__global__ __launch_bounds__(DBLOCK) void k_dmc_gather(const int64_t* __restrict__ chunks, int64_t B, int Tc, int O,
                                                       int SO, int F, const int8_t* __restrict__ st,
                                                       const int8_t* __restrict__ act, const float* __restrict__ tgt,
                                                       const float* __restrict__ ret, const uint8_t* __restrict__ dne,
                                                       int8_t* o_st, int8_t* o_act, float* o_tgt, float* o_ret,
                                                       uint8_t* o_dne)
{
    const int64_t j = blockIdx.x, t = blockIdx.y;   // batch column, chunk row
    const int64_t r = chunks[j] * Tc + t, orow = t * B + j;
    for (int k = threadIdx.x; k < SO; k += DBLOCK)
        if (o_st) o_st[orow * SO + k] = st[r * O + k];
    for (int k = threadIdx.x; k < F; k += DBLOCK)
        if (o_act) o_act[orow * F + k] = act[r * F + k];
    if (threadIdx.x == 0) {
        if (o_tgt) o_tgt[orow] = tgt[r];
        if (o_ret) o_ret[orow] = ret[r];
        if (o_dne) o_dne[orow] = dne[r];
    }
}

hipError_t launch_dmc_fill(const Buffers& b, const DmcRing& d, int32_t T, const cs_traj_out& tr, int64_t* ready,
                           int64_t cap, int64_t* nready, int64_t* dst, void** tmp, size_t* tmp_bytes, hipStream_t s)
{
    const int64_t streams = b.n * b.num_players, rows = (int64_t)T * b.n;
    hipLaunchKernelGGL(k_dmc_index, dim3((unsigned)((b.n + DBLOCK - 1) / DBLOCK)), dim3(DBLOCK), 0, s,
                       (const uint8_t*)tr.player, (const uint8_t*)tr.done, (const float*)tr.reward, T, b.n,
                       b.num_players, d.T, d.slots, d.ctr, d.gstart, d.emitted, dst, d.tgt, d.ret, d.dne, d.counts,
                       d.flag);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t need = 0;
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, d.counts, d.offsets, streams + 1, s);
    if (e != hipSuccess) return e;
    if (need > *tmp_bytes) {
        if (*tmp) (void)hipFree(*tmp);
        *tmp = nullptr;
        *tmp_bytes = 0;
        e = hipMalloc(tmp, need);
        if (e != hipSuccess) return e;
        *tmp_bytes = need;
    }
    // counts[streams] is kept 0, so offsets[streams] is the total
    e = hipcub::DeviceScan::ExclusiveSum(*tmp, need, d.counts, d.offsets, streams + 1, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dmc_ready, dim3((unsigned)((streams + DBLOCK - 1) / DBLOCK)), dim3(DBLOCK), 0, s, d.counts,
                       d.offsets, streams, d.slots, d.emitted, ready, cap, nready, d.flag);
    if (tr.obs) {
        const int64_t work = rows * ((b.obs_dim + 3) / 4);
        hipLaunchKernelGGL(k_dmc_rows, dim3((unsigned)((work + DBLOCK - 1) / DBLOCK)), dim3(DBLOCK), 0, s,
                           (const uint8_t*)tr.obs, dst, rows, b.obs_dim, d.st);
    }
    if (tr.action) {
        const uint64_t* cnt = b.game == CS_GAME_DOUDIZHU ? ((const ddz::Tab*)b.table)->cnt : nullptr;
        hipLaunchKernelGGL(k_dmc_features, dim3((unsigned)((rows + DBLOCK - 1) / DBLOCK)), dim3(DBLOCK), 0, s,
                           tr.action, b.action_bytes, dst, rows, d.F, b.num_actions, cnt, d.act);
    }
    return hipGetLastError();
}

hipError_t launch_dmc_gather(const DmcRing& d, int32_t state_dim, int32_t obs_dim, const int64_t* chunks,
                             int64_t count, const cs_dmc_batch& o, hipStream_t s)
{
    dim3 grid((unsigned)count, (unsigned)d.T);
    hipLaunchKernelGGL(k_dmc_gather, grid, dim3(DBLOCK), 0, s, chunks, count, d.T, obs_dim, state_dim, d.F, d.st,
                       d.act, d.tgt, d.ret, d.dne, (int8_t*)o.state, (int8_t*)o.action, (float*)o.target,
                       (float*)o.episode_return, (uint8_t*)o.done);
    return hipGetLastError();
}

// ---- Q scoring ----------------------------------------------------------------------------------------------------
// h1[i][:] = relu(X[state[i]][:] + b1 + sum over the set bits k of feature(id[i]) of Wa[k][:]) (one entry per block;
// four consecutive hidden units per thread per pass, float4 loads / stores; H a multiple of 4)
__global__ __launch_bounds__(128) void k_dmc_layer1(const float* __restrict__ X, const int32_t* __restrict__ state_of,
                                                    const int32_t* __restrict__ ids, int64_t E, int H,
                                                    const float* __restrict__ Wa, const float* __restrict__ b1, int F,
                                                    const uint64_t* __restrict__ ddz_cnt, float* h1)
{
    const int64_t i = blockIdx.x;
    if (i >= E) return;
    const int a = ids[i];
    for (int j = threadIdx.x * 4; j < H; j += 4 * (int)blockDim.x) {
    const float4 x = *(const float4*)(X + (int64_t)state_of[i] * H + j);
    const float4 bb = *(const float4*)(b1 + j);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ddz_cnt) {
        uint64_t bits = ddz::cards_bits(a >= 0 && a < ddz::PASS ? ddz_cnt[a] : 0ull);
        while (bits) {   // ascending feature index, as a dot product over the feature vector would run
            const int k = __builtin_ctzll(bits);
            bits &= bits - 1;
            const float4 w = *(const float4*)(Wa + (int64_t)k * H + j);
            acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
        }
    } else if (a >= 0 && a < F) {
        acc = *(const float4*)(Wa + (int64_t)a * H + j);
    }
    float4 h;
    h.x = fmaxf(x.x + acc.x + bb.x, 0.f);
    h.y = fmaxf(x.y + acc.y + bb.y, 0.f);
    h.z = fmaxf(x.z + acc.z + bb.z, 0.f);
    h.w = fmaxf(x.w + acc.w + bb.w, 0.f);
    *(float4*)(h1 + i * H + j) = h;
    }
}

// per state: the legal id with the largest value (first maximum, np.argmax); with probability eps a uniform legal id
// instead (DMCAgent.step, model.py:58-67; Philox4x32-10 keyed by seed on (global state index, t) replaces np.random)
__global__ __launch_bounds__(DBLOCK) void k_dmc_select(const float* __restrict__ values,
                                                       const int32_t* __restrict__ counts,
                                                       const int64_t* __restrict__ offsets,
                                                       const int32_t* __restrict__ ids, int64_t S, float eps,
                                                       uint64_t seed, uint64_t t, uint64_t base, int32_t* actions)
{
    const int64_t si = (int64_t)blockIdx.x * DBLOCK + threadIdx.x;
    if (si >= S) return;
    const int c = counts[si];
    const int64_t o = offsets[si];
    if (c <= 0) {
        actions[si] = -1;
        return;
    }
    int best = 0;
    float bv = values[o];
    for (int k = 1; k < c; k++) {
        const float v = values[o + k];
        if (v > bv) { bv = v; best = k; }
    }
    if (eps > 0.f) {
        uint32_t r[4];
        philox4(seed, base + (uint64_t)si, t, r);
        const float u = (float)(r[0] >> 8) * (1.0f / 16777216.0f);
        if (u < eps) best = (int)(((uint64_t)r[1] * (uint64_t)c) >> 32);
    }
    actions[si] = ids[o + best];
}

hipError_t launch_dmc_layer1(const float* X, const int32_t* state_of, const int32_t* ids, int64_t E, int32_t H,
                             const float* Wa, const float* b1, int32_t F, const Buffers& b, float* h1, hipStream_t s)
{
    const uint64_t* cnt = b.game == CS_GAME_DOUDIZHU ? ((const ddz::Tab*)b.table)->cnt : nullptr;
    hipLaunchKernelGGL(k_dmc_layer1, dim3((unsigned)E), dim3(128), 0, s, X, state_of, ids, E, H, Wa, b1, F, cnt, h1);
    return hipGetLastError();
}

hipError_t launch_dmc_select(const float* values, const int32_t* counts, const int64_t* offsets, const int32_t* ids,
                             int64_t S, float eps, uint64_t seed, uint64_t t, uint64_t base, int32_t* actions,
                             hipStream_t s)
{
    hipLaunchKernelGGL(k_dmc_select, dim3((unsigned)((S + DBLOCK - 1) / DBLOCK)), dim3(DBLOCK), 0, s, values, counts,
                       offsets, ids, S, eps, seed, t, base, actions);
    return hipGetLastError();
}

}  // namespace cs
