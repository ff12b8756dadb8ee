// calib.hip -- HBM counter calibration kernels (measurement infrastructure, not the engine).
//
// MI355X_MICROARCH.md (HBM): FETCH_SIZE reads exactly half the bytes of a 16-B-per-lane streaming read on gfx950 and
// WRITE_SIZE is exact for 16-B-per-lane streaming stores; every other access width is uncalibrated. The rollout
// kernels also move bytes in other shapes, so each shape is run here on a known byte count (well past the 256 MiB
// Infinity Cache) and the counters are compared with it (tools/calib.py, tools/gpu_calib.sh):
//   read16   16 B per lane, coalesced                       (control: the guide's calibrated case)
//   read4    4 B per lane, coalesced                        (state words, ring control words)
//   seg64    64-B rows at 4-B-aligned random offsets, 16 lanes per row with dword loads, 4 rows per instruction
//            (ring_restage_wave's restage rows, cs_ring.h)
//   write16  16 B per lane, coalesced, default policy       (control)
//   write16nt 16 B per lane, nontemporal                    (obs rows, RowWriter)
//   write1   1 B per lane, coalesced, default policy        (player / done / action rows)
//   write1nt 1 B per lane, nontemporal                      (the same rows as the rollout stores them)
//   write4nt 4 B per lane, nontemporal                      (reward rows)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

extern "C" {

__global__ __launch_bounds__(256) void k_read16(const uint4* __restrict__ a, int64_t n, uint32_t* out)
{
    uint32_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 v = a[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x9E3779B9u) out[0] = s;   // keeps the loads; never true for the zero-filled input
}

__global__ __launch_bounds__(256) void k_read4(const uint32_t* __restrict__ a, int64_t n, uint32_t* out)
{
    uint32_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s ^= a[i];
    if (s == 0x9E3779B9u) out[0] = s;
}

// rows: 64-B rows, row r starts at byte off[r] (multiple of 4); 16 lanes per row
__global__ __launch_bounds__(256) void k_seg64(const uint8_t* __restrict__ a, const uint32_t* __restrict__ off,
                                               int64_t rows, uint32_t* out)
{
    uint32_t s = 0;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < rows * 16; t += (int64_t)gridDim.x * 256) {
        const int64_t r = t >> 4;
        s ^= *(const uint32_t*)(a + off[r] + 4 * (t & 15));
    }
    if (s == 0x9E3779B9u) out[0] = s;
}

__global__ __launch_bounds__(256) void k_write16(uint4* a, int64_t n, int nt)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const u32x4_t v = {(uint32_t)i, 1u, 2u, 3u};
        if (nt) __builtin_nontemporal_store(v, (u32x4_t*)&a[i]);
        else *(u32x4_t*)&a[i] = v;
    }
}

__global__ __launch_bounds__(256) void k_write1(uint8_t* a, int64_t n, int nt)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if (nt) __builtin_nontemporal_store((uint8_t)i, a + i);
        else a[i] = (uint8_t)i;
    }
}

__global__ __launch_bounds__(256) void k_write4(uint32_t* a, int64_t n, int nt)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if (nt) __builtin_nontemporal_store((uint32_t)i, a + i);
        else a[i] = (uint32_t)i;
    }
}

// host launchers (ctypes): grid 8192 blocks x 256 threads, grid-stride loops
static const dim3 G(8192), B(256);
int calib_read16(const void* a, int64_t bytes, void* out)
{
    hipLaunchKernelGGL(k_read16, G, B, 0, 0, (const uint4*)a, bytes / 16, (uint32_t*)out);
    return (int)hipDeviceSynchronize();
}
int calib_read4(const void* a, int64_t bytes, void* out)
{
    hipLaunchKernelGGL(k_read4, G, B, 0, 0, (const uint32_t*)a, bytes / 4, (uint32_t*)out);
    return (int)hipDeviceSynchronize();
}
int calib_seg64(const void* a, const void* off, int64_t rows, void* out)
{
    hipLaunchKernelGGL(k_seg64, G, B, 0, 0, (const uint8_t*)a, (const uint32_t*)off, rows, (uint32_t*)out);
    return (int)hipDeviceSynchronize();
}
int calib_write16(void* a, int64_t bytes, int nt)
{
    hipLaunchKernelGGL(k_write16, G, B, 0, 0, (uint4*)a, bytes / 16, nt);
    return (int)hipDeviceSynchronize();
}
int calib_write1(void* a, int64_t bytes, int nt)
{
    hipLaunchKernelGGL(k_write1, G, B, 0, 0, (uint8_t*)a, bytes, nt);
    return (int)hipDeviceSynchronize();
}
int calib_write4(void* a, int64_t bytes, int nt)
{
    hipLaunchKernelGGL(k_write4, G, B, 0, 0, (uint32_t*)a, bytes / 4, nt);
    return (int)hipDeviceSynchronize();
}

}  // extern "C"
