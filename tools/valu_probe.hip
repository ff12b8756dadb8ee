// valu_probe.hip -- measures the vector / scalar instruction issue ceilings of one MI355X, the second roofline of the
// integer rollout kernels (they run out of VALU issue before HBM). Each thread runs K independent integer
// add chains (the compiler cannot fold them: the chains mix in lane data), so a SIMD's VALU pipe is the only limit;
// waves per SIMD come from the launch width. Prints wave-instructions per SIMD per cycle for each configuration.
//   hipcc -O3 --offload-arch=gfx950 -o tools/valu_probe tools/valu_probe.hip && tools/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int K>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t a[K];
#pragma unroll
    for (int k = 0; k < K; k++) a[k] = threadIdx.x * (k + 1) + seed;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % K]));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 3) % K]));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < K; k++) s += a[k];
    if (s == 0x12345678u) out[blockIdx.x] = s;
}

// scalar issue: K x 4 independent s_mov per iteration per wave (wave-uniform work). s_mov / s_mul do not write SCC,
// which the loop's own compare-and-branch uses (an SCC-writing asm op here can turn the loop endless)
template <int K>
__global__ __launch_bounds__(256) void k_salu(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t s0 = seed, s1 = seed * 3u, s2 = seed * 5u, s3 = seed * 7u;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(s1));
            asm volatile("s_mov_b32 %0, %1" : "=s"(s1) : "s"(s2));
            asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s2) : "s"(s3));
            asm volatile("s_mov_b32 %0, %1" : "=s"(s3) : "s"(s0));
        }
    }
    if ((s0 ^ s1 ^ s2 ^ s3) == 0x12345678u) out[blockIdx.x] = s0;
}

// mixed: per iteration K VALU pairs and K SALU quads, independent: do the two pipes overlap?
template <int K>
__global__ __launch_bounds__(256) void k_mixed(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t a[K];
#pragma unroll
    for (int k = 0; k < K; k++) a[k] = threadIdx.x * (k + 1) + seed;
    uint32_t s0 = seed, s1 = seed * 3u, s2 = seed * 5u, s3 = seed * 7u;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % K]));
            asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(s1));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 3) % K]));
            asm volatile("s_mov_b32 %0, %1" : "=s"(s1) : "s"(s2));
        }
    }
    uint32_t s = s0 ^ s1;
#pragma unroll
    for (int k = 0; k < K; k++) s += a[k];
    if (s == 0x12345678u) out[blockIdx.x] = s;
}

int main()
{
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    printf("device %s, %d CUs, clock %d MHz\n", p.name, cus, clk_khz / 1000);
    uint32_t* out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int wps = 1; wps <= 8; wps *= 2) {          // waves per SIMD
        const int blocks = cus * wps;                  // 4 waves per block -> one per SIMD
        for (int kind = 0; kind < 3; kind++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(k_valu<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
                else if (kind == 1) hipLaunchKernelGGL(k_salu<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
                else hipLaunchKernelGGL(k_mixed<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep == 0) continue;
                // wave-instructions per SIMD: waves per SIMD x iters x 16 (VALU) / (SALU 32) / (mixed 16 + 16)
                const double per_simd = (double)wps * iters * (kind == 1 ? 32.0 : 16.0);
                const double cycles = ms * 1e-3 * 2.4e9;   // at the 2.4 GHz max clock
                printf("%-6s waves/SIMD %d: %.3f ms  %.3f %s wave-instr per SIMD-cycle (at 2.4 GHz)%s\n",
                       kind == 0 ? "VALU" : (kind == 1 ? "SALU" : "mixed"), wps, ms, per_simd / cycles,
                       kind == 2 ? "VALU (+ as many SALU)" : "", "");
            }
        }
    }
    hipFree(out);
    return 0;
}
