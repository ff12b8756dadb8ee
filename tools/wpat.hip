// wpat.hip -- synthetic trajectory-write probe (round 5): the rollout's output write pattern with
// no game logic, so trajectory layouts can be compared on the same HBM placement (one allocation, every layout) and on
// physically contiguous allocations (hipDeviceMallocContiguous: the slowest placement, deterministic).
// One wave = 64 envs; per step a wave spins `work` dependent VALU ops (the game's compute), then writes its rows:
//   mode 0 split       obs [T][ts][36] + legal/player/action/done [T][ts] u8 + reward [T][ts][2] f32 (the r04 layout)
//   mode 1 packed      rec [T][ts][48], the wave's 3 072-B span as coalesced 16-B stores (3 per lane)
//   mode 2 wavemajor   rec [n/64][T][64*48]: each wave's steps consecutive
//   mode 3 packedlane  rec [T][ts][48], lane l stores its own three 16-B chunks (48-B lane stride)
//   mode 4 blockmajor  rec [n/256][T][256*48]: a block's four waves write adjacent spans, steps consecutive
//   mode 5 obsonly     obs [T][ts][36] only
//   mode 6 split_nt0   mode 0 with default-policy stores
//   mode 7 work        no rows (the work's time alone)
//   mode 8 grouped     rec [n/64/R][T][R*64*48]: groups of R waves, time-major inside a group (R = n/64: packed,
//                      R = 1: wavemajor, R = 4: blockmajor)
//   mode 9 packed_nt0  mode 1 with default-policy stores
//   mode 12 planes     rec [T][3][ts][16]: the 48-B record as three 16-B planes (each wave store 1 KB contiguous)
//   mode 13 ddz        DouDizhu's two row tensors (legal 3 434 B at off_legal, obs 901 B), 2 envs per wave; 14: nt
//   mode 11 chunks     one sweep of the buffer, wave w writes R consecutive 1-KB pieces (a block: 4 R KB); T = 1
// ts = rows per step (n + pad). Built by hand: hipcc -O3 -shared -fPIC --offload-arch=gfx950 -o tools/libwpat.so tools/wpat.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, class T>
__device__ __forceinline__ void st(T* p, T v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

struct WArgs {
    uint8_t* base;      // one buffer; split layouts carve obs / bytes / reward from it at the given offsets
    int64_t off_legal, off_player, off_action, off_done, off_reward;
    int64_t n, ts;
    int32_t T, work, mode, R;   // R: waves per group (mode 8)
    int32_t dm, xcd;            // data: 0 = varying (x, x+1, ..), 1 = zeros, 2 = one constant, 3 = per-env constant
                                // xcd: 1 = block b handles env block (b % 8) * (B / 8) + b / 8 (XCD x owns 1/8 of the envs)
};

template <int MODE>
__global__ __launch_bounds__(256) void k_wpat(WArgs a)
{
    extern __shared__ uint32_t dyn[];   // occupancy control only
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t nb = gridDim.x;
    const int64_t bx = a.xcd ? (int64_t)(blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : (int64_t)blockIdx.x;
    const int64_t wave = bx * 4 + wid, wf = wave * 64, env = wf + lane;
    if (wf >= a.n) return;
    uint32_t x = (uint32_t)env * 2654435761u;
    if (a.work < 0) dyn[threadIdx.x] = x;
    for (int t = 0; t < a.T; t++) {
        for (int k = 0; k < a.work; k++) x = x * 1664525u + 1013904223u;
        asm volatile("" : "+v"(x));
        u32x4 v = {x, x + 1u, x + 2u, x + 3u};
        if (a.dm == 1) v = u32x4{0u, 0u, 0u, 0u};
        else if (a.dm == 2) v = u32x4{0x3F9E0419u, 0x3F9E0419u, 0x3F9E0419u, 0x3F9E0419u};
        else if (a.dm == 3) v = u32x4{(uint32_t)env, (uint32_t)env, 7u, 9u};
        if constexpr (MODE == 0 || MODE == 5 || MODE == 6) {
            constexpr bool NT = MODE != 6;
            const int64_t row0 = (int64_t)t * a.ts + wf;
            u32x4* o = (u32x4*)(a.base + row0 * 36);
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const int q = j * 64 + lane;
                if (q < 144) st<NT>(o + q, v);
            }
            if constexpr (MODE != 5) {
                const int64_t row = row0 + lane;
                st<NT>(a.base + a.off_legal + row, (uint8_t)x);
                st<NT>(a.base + a.off_player + row, (uint8_t)(x >> 8));
                st<NT>(a.base + a.off_action + row, (uint8_t)(x >> 16));
                st<NT>((uint64_t*)(a.base + a.off_reward) + row, (uint64_t)x * 3u);
                st<NT>(a.base + a.off_done + row, (uint8_t)(x >> 24));
            }
        } else if constexpr (MODE == 13 || MODE == 14) {   // DouDizhu rows: 2 envs per wave, 3 434 + 901 B each
            // (13: default-policy stores, 14: nontemporal); spans rounded out to 16-B chunks (neighbours overlap)
            constexpr bool NT = MODE == 14;
            const int64_t e0 = (int64_t)t * a.ts + 2 * wave;
            const int64_t lb = e0 * 3434, ob = e0 * 901;
            uint8_t* lrow = a.base + a.off_legal + (lb & ~15ll);
            uint8_t* orow = a.base + (ob & ~15ll);
            const int lq = (int)(((lb & 15) + 6868 + 15) >> 4), oq = (int)(((ob & 15) + 1802 + 15) >> 4);
            for (int q = lane; q < lq; q += 64) st<NT>((u32x4*)lrow + q, v);
            for (int q = lane; q < oq; q += 64) st<NT>((u32x4*)orow + q, v);
        } else if constexpr (MODE == 12) {   // planes: rec [T][3][ts][16], each store one 1-KB piece of a plane
#pragma unroll
            for (int j = 0; j < 3; j++) st<true>((u32x4*)(a.base + (((int64_t)t * 3 + j) * a.ts + env) * 16), v);
        } else if constexpr (MODE == 11) {   // one sweep: wave w writes R consecutive 1-KB pieces at w * R KB
            u32x4* o = (u32x4*)(a.base + wave * a.R * 1024);
            for (int j = 0; j < a.R; j++) st<true>(o + j * 64 + lane, v);
        } else if constexpr (MODE == 9) {   // packed, default-policy stores
            u32x4* o = (u32x4*)(a.base + ((int64_t)t * a.ts + wf) * 48);
#pragma unroll
            for (int j = 0; j < 3; j++) st<false>(o + j * 64 + lane, v);
        } else if constexpr (MODE == 1 || MODE == 2 || MODE == 4 || MODE == 8) {
            int64_t span;
            if constexpr (MODE == 8) span = (((wave / a.R) * a.T + t) * a.R + wave % a.R) * (64 * 48);
            else if constexpr (MODE == 1) span = ((int64_t)t * a.ts + wf) * 48;
            else if constexpr (MODE == 2) span = (wave * a.T + t) * (64 * 48);
            else span = ((bx * a.T + t) * 4 + wid) * (64 * 48);
            u32x4* o = (u32x4*)(a.base + span);
#pragma unroll
            for (int j = 0; j < 3; j++) st<true>(o + j * 64 + lane, v);
        } else if constexpr (MODE == 3) {
            u32x4* o = (u32x4*)(a.base + ((int64_t)t * a.ts + env) * 48);
#pragma unroll
            for (int j = 0; j < 3; j++) st<true>(o + j, v);
        }
    }
    if constexpr (MODE == 7) st<true>((uint32_t*)a.base + env, x);   // work only (calibration): one store per lane
}

extern "C" int wpat_run(const WArgs* a, int lds_bytes, void* stream)
{
    const dim3 grid((unsigned)((a->n + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
    switch (a->mode) {
    case 0: hipLaunchKernelGGL(k_wpat<0>, grid, dim3(256), lds_bytes, s, *a); break;
    case 1: hipLaunchKernelGGL(k_wpat<1>, grid, dim3(256), lds_bytes, s, *a); break;
    case 2: hipLaunchKernelGGL(k_wpat<2>, grid, dim3(256), lds_bytes, s, *a); break;
    case 3: hipLaunchKernelGGL(k_wpat<3>, grid, dim3(256), lds_bytes, s, *a); break;
    case 4: hipLaunchKernelGGL(k_wpat<4>, grid, dim3(256), lds_bytes, s, *a); break;
    case 5: hipLaunchKernelGGL(k_wpat<5>, grid, dim3(256), lds_bytes, s, *a); break;
    case 6: hipLaunchKernelGGL(k_wpat<6>, grid, dim3(256), lds_bytes, s, *a); break;
    case 7: hipLaunchKernelGGL(k_wpat<7>, grid, dim3(256), lds_bytes, s, *a); break;
    case 8: hipLaunchKernelGGL(k_wpat<8>, grid, dim3(256), lds_bytes, s, *a); break;
    case 9: hipLaunchKernelGGL(k_wpat<9>, grid, dim3(256), lds_bytes, s, *a); break;
    case 13: hipLaunchKernelGGL(k_wpat<13>, grid, dim3(256), lds_bytes, s, *a); break;
    case 14: hipLaunchKernelGGL(k_wpat<14>, grid, dim3(256), lds_bytes, s, *a); break;
    case 12: hipLaunchKernelGGL(k_wpat<12>, grid, dim3(256), lds_bytes, s, *a); break;
    case 11: hipLaunchKernelGGL(k_wpat<11>, grid, dim3(256), lds_bytes, s, *a); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
