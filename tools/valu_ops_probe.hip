// VALU issue rate per SIMD for the integer instructions the lane-game kernels are made of (v_bfe_u32, v_xor_b32,
// v_add_u32, v_ffbh_u32, v_cmp + v_subbrev) against v_fma_f32, at 1, 2, 4 and 8 waves per SIMD: is a kernel that
// issues one wave64 integer VALU instruction every ~4 cycles per SIMD at the VALU roof, or latency-bound?
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_ops_probe tools/valu_ops_probe.hip && tools/valu_ops_probe
// Each lane runs 8 independent chains of ITER x 16 instructions; cycles per wave from s_memtime (core clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k_probe(uint32_t* out, unsigned long long* cyc, int iters, uint32_t s)
// cyc per wave: [core-clock cycles, realtime start, realtime end] (s_memtime; s_memrealtime at 100 MHz)
{
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x * 2654435761u + (uint32_t)k * s;
    const uint32_t b = s ^ threadIdx.x;
    const uint64_t sm = 0x5555555555555555ull ^ s;
    if constexpr (OP == 29) asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 2; r++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 1) asm volatile("v_bfe_u32 %0, %0, %1, 9" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 3) asm volatile("v_ffbh_u32 %0, %0" : "+v"(a[k]));
                if constexpr (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 5) asm volatile("v_cmp_le_u32 vcc, %0, %1\n\tv_subbrev_co_u32 %0, vcc, 0, %0, vcc"
                                                    : "+v"(a[k]) : "v"(b) : "vcc");
                if constexpr (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 7) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 8) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 9) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 10) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 11) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 12) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 13) asm volatile("v_mov_b32 %0, %1" : "=v"(a[k]) : "v"(b));
                if constexpr (OP == 15) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 16) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 17) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 18) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 19) asm volatile("v_cmp_le_u32 vcc, %0, %1" : : "v"(a[k]), "v"(b) : "vcc");
                if constexpr (OP == 20) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "s"(sm));
                if constexpr (OP == 21) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 22) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 23) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 24) asm volatile("v_subbrev_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a[k]) : : "vcc");
                if constexpr (OP == 25) asm volatile("v_add_u32 %0, %0, 7" : "+v"(a[k]));
                if constexpr (OP == 26) asm volatile("v_and_b32 %0, 63, %0" : "+v"(a[k]));
                if constexpr (OP == 27) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
                if constexpr (OP == 28) asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a[k]) : "v"(b) : "s40", "s41");
                if constexpr (OP == 29) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == 30) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_subbrev_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
                if constexpr (OP == 31) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
                if constexpr (OP == 32) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
                if constexpr (OP == 33) asm volatile("s_mov_b64 vcc, %1\n\tv_cndmask_b32 %0, %0, %2, vcc" : "+v"(a[k]) : "s"(sm), "v"(b) : "vcc");
                if constexpr (OP == 14) asm volatile("v_and_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(a[k]) : "v"(b));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) x ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) {
        unsigned long long* c = cyc + 3 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
        c[0] = t1 - t0;
        c[1] = r0;
        c[2] = r1;
    }
}

template <int OP>
static int run(const char* name, int cus)
{
    const int iters = 4096, per_iter = (OP == 5 || OP == 27 || OP == 28 || OP == 30 || OP == 33) ? 32 : (OP == 31 || OP == 32) ? 64 : 16;
    for (int wps = 1; wps <= 8; wps *= 8) {
        // 4 waves per block = one per SIMD; wps blocks per CU
        const int blocks = cus * wps, threads = 256;
        uint32_t* out;
        unsigned long long* cyc;
        CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
        CHECK(hipMalloc(&cyc, (size_t)blocks * 4 * 24));
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 64, 12345u);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 12345u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long* h = new unsigned long long[(size_t)blocks * 12];
        CHECK(hipMemcpy(h, cyc, (size_t)blocks * 4 * 24, hipMemcpyDeviceToHost));
        double mean = 0, fsum = 0;
        unsigned long long rmin = ~0ull, rmax = 0;
        for (int i = 0; i < blocks * 4; i++) {
            mean += (double)h[3 * i];
            fsum += (double)h[3 * i] / ((double)(h[3 * i + 2] - h[3 * i + 1]) * 10.0);   // cycles per ns * 1000 = MHz
            rmin = h[3 * i + 1] < rmin ? h[3 * i + 1] : rmin;
            rmax = h[3 * i + 2] > rmax ? h[3 * i + 2] : rmax;
        }
        mean /= blocks * 4;
        const double mhz = fsum / (blocks * 4) * 1000.0, window_us = (double)(rmax - rmin) / 100.0;
        const double insts = (double)iters * per_iter;
        // per SIMD: wps waves share it; cycles per instruction per SIMD = wave cycles / (wps * instructions per wave)
        printf("%-10s waves/SIMD %d: %.3f ms (window %.1f us), clock %.0f MHz, cycles/inst one wave %.2f, "
               "per SIMD over the window %.2f\n", name, wps, ms, window_us, mhz, mean / insts,
               window_us * mhz / (insts * wps));
        delete[] h;
        CHECK(hipFree(out));
        CHECK(hipFree(cyc));
    }
    return 0;
}

int main()
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, cus);
    if (run<31>("cmp+3cnd", cus) || run<32>("cmp+2add+cnd", cus) || run<33>("smov+cnd", cus))
        return 1;
    return 0;
}
