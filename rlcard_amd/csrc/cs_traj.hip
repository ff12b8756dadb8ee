// cs_traj.hip -- the steps right after the rollout, on the device:
//   k_transitions                  rlcard's reorganize (rlcard/utils/utils.py:153-179) + the DMC return target
//                                  (rlcard/agents/dmc_agent/utils.py:97-163) for every (step, env) of a trajectory
//   k_legal_count / k_legal_fill   legal-action id lists from the bitmask rows (wavefront compaction), the form the
//                                  agents consume (state['legal_actions'] keys, envs/env.py _extract_state)
// All HBM-bound streaming: a few bytes per row in and out.
#include <hipcub/hipcub.hpp>
#include "cs_device.h"
#include "cs_engine.h"

namespace cs {

constexpr int TBLOCK = 256;
constexpr int MAXP = 10;   // players per env (3..10-player hold'em, cs_holdem_n.h)

// One lane per env, scanning its T rows backwards. Row (t, e) is a transition of the player who acted at t:
//   next_t  its next turn in the same game, -1 = the game ended first (next state = final_obs at row end_t), -2 = the
//           game goes on past the window (the caller carries it into the next chunk)
//   end_t   row where this row's game ends, -1 = past the window
//   reward  the player's payoff on its last transition of the game, else 0 (reorganize: payoffs[player], done True)
//   done    1 on that last transition
//   ret     the player's payoff of the game (the DMC target for every step it took); NaN if it ends past the window
__global__ __launch_bounds__(TBLOCK) void k_transitions(const uint8_t* __restrict__ player,
                                                        const uint8_t* __restrict__ done,
                                                        const float* __restrict__ reward, int T, int64_t n, int P,
                                                        int32_t* next_t, int32_t* end_t, float* r_out, uint8_t* d_out,
                                                        float* ret)
{
    const int64_t e = (int64_t)blockIdx.x * TBLOCK + threadIdx.x;
    if (e >= n) return;
    const float nan = __builtin_nanf("");
    int32_t nxt[MAXP];
    float pay[MAXP];
#pragma unroll
    for (int q = 0; q < MAXP; q++) {
        nxt[q] = -2;
        pay[q] = nan;
    }
    int32_t end = -1;
    for (int t = T - 1; t >= 0; t--) {
        const int64_t row = (int64_t)t * n + e;
        if (done[row]) {   // a game ends at t: rows t, t-1, ... back to the previous end belong to it
            end = t;
#pragma unroll
            for (int q = 0; q < MAXP; q++) {
                nxt[q] = -1;
                pay[q] = q < P ? reward[row * P + q] : 0.f;
            }
        }
        const int p = player[row];
        int32_t np = -2;
        float pp = nan;
#pragma unroll
        for (int q = 0; q < MAXP; q++) {
            if (q == p) {
                np = nxt[q];
                pp = pay[q];
                nxt[q] = t;
            }
        }
        if (next_t) next_t[row] = np;
        if (end_t) end_t[row] = end;
        if (r_out) r_out[row] = np == -1 ? pp : 0.f;
        if (d_out) d_out[row] = np == -1 ? 1 : 0;
        if (ret) ret[row] = end >= 0 ? pp : nan;
    }
}

// ---- legal lists ------------------------------------------------------------------------------------------------
// short rows (<= 16 bytes: leduc / limit / blackjack): one lane per row
__global__ __launch_bounds__(TBLOCK) void k_legal_count_small(const uint8_t* __restrict__ legal, int64_t rows, int lb,
                                                              int32_t* counts)
{
    const int64_t r = (int64_t)blockIdx.x * TBLOCK + threadIdx.x;
    if (r >= rows) return;
    int c = 0;
    for (int k = 0; k < lb; k++) c += __popc(legal[r * lb + k]);
    counts[r] = c;
}

__global__ __launch_bounds__(TBLOCK) void k_legal_fill_small(const uint8_t* __restrict__ legal, int64_t rows, int lb,
                                                             const int64_t* __restrict__ offsets, int32_t* ids)
{
    const int64_t r = (int64_t)blockIdx.x * TBLOCK + threadIdx.x;
    if (r >= rows) return;
    int64_t o = offsets[r];
    for (int k = 0; k < lb; k++) {
        uint32_t b = legal[r * lb + k];
        while (b) {
            ids[o++] = 8 * k + __builtin_ctz(b);
            b &= b - 1;
        }
    }
}

// long rows (doudizhu: 3 434 bytes): one wave per row, read as the 16-B aligned chunks that cover it (lane q takes
// chunk q of a 64-chunk round: every load instruction moves 1 KB contiguous); bytes of the neighbouring rows are masked
// off, and the chunk that would run past the row's end is read bytewise (it may be the buffer's end). The fill pass
// turns each round's popcounts into write positions with a wave prefix scan, so the ids come out ascending.
__device__ __forceinline__ uint4 row_chunk(uintptr_t cs, uintptr_t a, uintptr_t e)
{
    uint4 v;
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const v4u g4;   // global, not flat (see cs_device.h to_global)
    typedef __attribute__((address_space(1))) const uint8_t g1;
    if (cs + 16 <= e) {
        const v4u t = *(g4*)cs;
        v = make_uint4(t.x, t.y, t.z, t.w);
    } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int k = 0; k < 16 && cs + k < e; k++) w[k >> 2] |= (uint32_t)(*(g1*)(cs + k)) << (8 * (k & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (cs < a) {   // first chunk: drop the previous row's bytes
        const int h = (int)(a - cs);
        uint32_t* w = (uint32_t*)&v;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int lo = 4 * k;
            w[k] &= lo + 4 <= h ? 0u : (lo >= h ? 0xFFFFFFFFu : (0xFFFFFFFFu << (8 * (h - lo))));
        }
    }
    return v;
}

template <bool FILL>
__global__ __launch_bounds__(TBLOCK) void k_legal_wave(const uint8_t* __restrict__ legal, int64_t rows, int lb,
                                                       int32_t* counts, const int64_t* __restrict__ offsets,
                                                       int32_t* ids)
{
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t r = (int64_t)blockIdx.x * (TBLOCK / WAVE) + threadIdx.x / WAVE;
    if (r >= rows) return;
    const uintptr_t a = (uintptr_t)(legal + r * lb), a0 = a & ~(uintptr_t)15, e = a + (uintptr_t)lb;
    const int nq = (int)((e - a0 + 15) >> 4);
    if constexpr (!FILL) {
        int c = 0;
        for (int q = lane; q < nq; q += WAVE) {
            const uint4 v = row_chunk(a0 + 16 * (uintptr_t)q, a, e);
            c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        }
        for (int o = WAVE / 2; o; o >>= 1) c += __shfl_xor(c, o);
        if (lane == 0) counts[r] = c;
    } else {
        int64_t base = offsets[r];
        for (int q0 = 0; q0 < nq; q0 += WAVE) {
            const int q = q0 + lane;
            const uintptr_t cs = a0 + 16 * (uintptr_t)q;
            const uint4 v = q < nq ? row_chunk(cs, a, e) : make_uint4(0, 0, 0, 0);
            const int c = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
            if (!__ballot(c != 0)) continue;   // legal ids are sparse in a 27 472-bit row: most rounds are empty
            int inc = c;
#pragma unroll
            for (int o = 1; o < WAVE; o <<= 1) {
                const int y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            int64_t w = base + (inc - c);
            const int bit0 = 8 * (int)((intptr_t)cs - (intptr_t)a);   // id of the chunk's first bit (may be < 0)
            const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t b = ws[k];
                while (b) {
                    ids[w++] = bit0 + 32 * k + __builtin_ctz(b);
                    b &= b - 1;
                }
            }
            base += __shfl(inc, WAVE - 1);
        }
    }
}

// Trajectory placement probe (cs_traj_probe): zeros written into every output tensor of a T-step trajectory in the
// rollout's order -- per step, each wave's span of EPW consecutive envs' rows of each tensor -- with no game logic.
// Its time tells how fast this allocation takes the rollout's writes (the rollout's time follows it: DESIGN 7); the
// host keeps the fastest of a few candidate allocations (VecEnv.new_traj_out(select=k)). 16-B nontemporal stores for
// the span's whole chunks, single bytes for its ends: nothing outside a tensor is written.
struct ProbeSpan {
    uint8_t* base;
    int32_t row;   // bytes per env row
};
__device__ __forceinline__ void probe_span(uint8_t* p, int64_t begin, int64_t end, int lane)
{
    const int64_t b16 = (begin + 15) & ~(int64_t)15, e16 = end & ~(int64_t)15;
    if (b16 >= e16) {   // a span inside one chunk: bytes
        for (int64_t k = begin + lane; k < end; k += WAVE) p[k] = 0;
        return;
    }
    const u32x4_t z = {0u, 0u, 0u, 0u};
    for (int64_t q = b16 + 16 * (int64_t)lane; q < e16; q += 16 * WAVE) __builtin_nontemporal_store(z, (u32x4_t*)(p + q));
    if (lane < 16 && begin + lane < b16) p[begin + lane] = 0;
    if (lane >= 16 && lane < 32 && e16 + (lane - 16) < end) p[e16 + (lane - 16)] = 0;
}
__global__ __launch_bounds__(TBLOCK) void k_traj_probe(ProbeSpan o0, ProbeSpan o1, ProbeSpan o2, ProbeSpan o3,
                                                       ProbeSpan o4, ProbeSpan o5, int T, int64_t n, int epw)
{
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t wave = (int64_t)blockIdx.x * (TBLOCK / WAVE) + __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int64_t e0 = wave * epw;
    if (e0 >= n) return;
    const int64_t e1 = e0 + epw < n ? e0 + epw : n;
    const ProbeSpan sp[6] = {o0, o1, o2, o3, o4, o5};
    for (int t = 0; t < T; t++) {
        const int64_t r0 = (int64_t)t * n;
#pragma unroll
        for (int k = 0; k < 6; k++)
            if (sp[k].base) probe_span(sp[k].base, (r0 + e0) * sp[k].row, (r0 + e1) * sp[k].row, lane);
    }
}

hipError_t launch_traj_probe(const Buffers& b, int32_t T, const cs_traj_out& tr, int32_t obs_dim, int32_t legal_bytes,
                             int32_t action_bytes, int32_t epw, hipStream_t s)
{
    const ProbeSpan o0{(uint8_t*)tr.obs, obs_dim}, o1{(uint8_t*)tr.legal, legal_bytes}, o2{(uint8_t*)tr.player, 1},
        o3{(uint8_t*)tr.action, action_bytes}, o4{(uint8_t*)tr.reward, 4 * b.num_players}, o5{(uint8_t*)tr.done, 1};
    const int64_t waves = (b.n + epw - 1) / epw;
    const dim3 grid((unsigned)((waves + TBLOCK / WAVE - 1) / (TBLOCK / WAVE)));
    hipLaunchKernelGGL(k_traj_probe, grid, dim3(TBLOCK), 0, s, o0, o1, o2, o3, o4, o5, T, b.n, epw);
    return hipGetLastError();
}

hipError_t launch_transitions(const Buffers& b, int32_t T, const cs_traj_out& tr, const cs_trans_out& o,
                              hipStream_t s)
{
    hipLaunchKernelGGL(k_transitions, dim3((unsigned)((b.n + TBLOCK - 1) / TBLOCK)), dim3(TBLOCK), 0, s,
                       (const uint8_t*)tr.player, (const uint8_t*)tr.done, (const float*)tr.reward, T, b.n,
                       b.num_players, (int32_t*)o.next_t, (int32_t*)o.end_t, (float*)o.reward, (uint8_t*)o.done,
                       (float*)o.ret);
    return hipGetLastError();
}

hipError_t launch_legal_lists(const Buffers& b, int32_t lb, const uint8_t* legal, int64_t rows, int32_t* counts,
                              int64_t* offsets, int32_t* ids, void** tmp, size_t* tmp_bytes, hipStream_t s)
{
    hipError_t e;
    const bool wave = lb > 16;
    const dim3 g_lane((unsigned)((rows + TBLOCK - 1) / TBLOCK)), g_wave((unsigned)((rows + 3) / 4));
    if (wave) hipLaunchKernelGGL(k_legal_wave<false>, g_wave, dim3(TBLOCK), 0, s, legal, rows, lb, counts, nullptr,
                                 nullptr);
    else hipLaunchKernelGGL(k_legal_count_small, g_lane, dim3(TBLOCK), 0, s, legal, rows, lb, counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // offsets[0] = 0, offsets[1..rows] = inclusive prefix sum of the counts
    if ((e = hipMemsetAsync(offsets, 0, sizeof(int64_t), s)) != hipSuccess) return e;
    size_t need = 0;
    if ((e = hipcub::DeviceScan::InclusiveSum(nullptr, need, counts, offsets + 1, rows, s)) != hipSuccess) return e;
    if (need > *tmp_bytes) {
        if (*tmp) (void)hipFree(*tmp);
        *tmp = nullptr;
        *tmp_bytes = 0;
        if ((e = hipMalloc(tmp, need)) != hipSuccess) return e;
        *tmp_bytes = need;
    }
    if ((e = hipcub::DeviceScan::InclusiveSum(*tmp, need, counts, offsets + 1, rows, s)) != hipSuccess) return e;
    if (ids) {
        if (wave) hipLaunchKernelGGL(k_legal_wave<true>, g_wave, dim3(TBLOCK), 0, s, legal, rows, lb, nullptr, offsets,
                                     ids);
        else hipLaunchKernelGGL(k_legal_fill_small, g_lane, dim3(TBLOCK), 0, s, legal, rows, lb, offsets, ids);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

// one-hot action features (envs/env.py get_action_feature) for games without a card-combo feature
__global__ __launch_bounds__(TBLOCK) void k_onehot(const int32_t* __restrict__ ids, int64_t count, int na,
                                                   uint8_t* out)
{
    const int64_t i = (int64_t)blockIdx.x * TBLOCK + threadIdx.x;
    if (i >= count * na) return;
    const int64_t r = i / na;
    out[i] = ids[r] == (int32_t)(i - r * na) ? 1 : 0;
}

// one env's packed state words (word-major [sw][n] or env-major [n][sw]) into dst: cs_copy_env_state
__global__ void k_copy_state(const uint32_t* __restrict__ st, int64_t n, int64_t env, int sw, int env_major,
                             uint32_t* dst)
{
    const int w = (int)threadIdx.x;
    if (w < sw) dst[w] = env_major ? st[env * sw + w] : st[(int64_t)w * n + env];
}

hipError_t launch_copy_state(const Buffers& b, int64_t env, int32_t sw, uint32_t* dst, hipStream_t s)
{
    hipLaunchKernelGGL(k_copy_state, dim3(1), dim3(64), 0, s, b.state, b.n, env, sw, state_env_major(b.game) ? 1 : 0,
                       dst);
    return hipGetLastError();
}

// one env's RNG stream (cs_copy_env_rng / cs_load_env_rng): buf = ctl word, then the env's mt words (env-major at
// mt + env * mtw, or a column mt[k * n + env] for the Blackjack shoe). load = 1 writes the env from buf; clear_mask
// then drops ctl bits (the rollout's "staged rows valid" bit: the restored position restages from the ring).
__global__ __launch_bounds__(TBLOCK) void k_rng_copy(uint32_t* __restrict__ mt, uint32_t* __restrict__ ctl, int64_t n,
                                                     int64_t env, int mtw, int column, uint32_t clear_mask,
                                                     uint32_t* __restrict__ buf, int load)
{
    for (int k = (int)threadIdx.x; k <= mtw; k += TBLOCK) {
        if (k == 0) {
            if (load) ctl[env] = buf[0] & ~clear_mask;
            else buf[0] = ctl[env];
            continue;
        }
        uint32_t* w = column ? mt + (int64_t)(k - 1) * n + env : mt + env * mtw + (k - 1);
        if (load) *w = buf[k];
        else buf[k] = *w;
    }
}

hipError_t launch_rng_copy(const Buffers& b, int64_t env, int32_t mtw, int32_t column, uint32_t clear_mask,
                           uint32_t* buf, int32_t load, hipStream_t s)
{
    hipLaunchKernelGGL(k_rng_copy, dim3(1), dim3(TBLOCK), 0, s, b.mt, b.ctl, b.n, env, mtw, column, clear_mask, buf,
                       load);
    return hipGetLastError();
}

hipError_t launch_onehot(const int32_t* ids, int64_t count, int32_t na, uint8_t* out, hipStream_t s)
{
    const int64_t total = count * na;
    hipLaunchKernelGGL(k_onehot, dim3((unsigned)((total + TBLOCK - 1) / TBLOCK)), dim3(TBLOCK), 0, s, ids, count, na,
                       out);
    return hipGetLastError();
}

}  // namespace cs
