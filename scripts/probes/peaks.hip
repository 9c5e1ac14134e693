// Sustained-peak probe ("measure the sustained INT32 peak and
// HBM bandwidth with microbenchmarks on the box"), the denominators next to
// the nominal ones the rooflines in bench.py use.
//
//   int32 VALU: every lane runs 16 independent add/xor chains (one v_add_u32 or
//               v_xor_b32 per op, checked in the ISA), 8 waves per SIMD;
//               ops/s = lanes x iterations x 32 / time.
//   HBM read:   grid-stride 16-byte loads over a 4 GiB buffer, XOR-reduced.
//   HBM copy:   grid-stride 16-byte load + store, 2 GiB -> 2 GiB (bytes = read + write).
//
// Prints one JSON line.  Build: hipcc --offload-arch=gfx950 -O3 peaks.hip -o peaks
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_int32(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = threadIdx.x * (j + 1) + seed;
    const uint32_t b = seed | 1u;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            a[j] += b;                 // v_add_u32
            a[j] ^= a[(j + 1) & 15];   // v_xor_b32 (reads the neighbour's previous value)
            asm volatile("" : "+v"(a[j]));
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) r ^= a[j];
    if (r == 0x9e3779b9u) out[blockIdx.x] = r;   // keeps the chains live
}

__global__ __launch_bounds__(256) void k_read(const uint4 *__restrict__ p, size_t n, uint32_t *out) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345679u) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        d[i] = s[i];
}

__global__ void k_fill(uint4 *p, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        p[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 7), 3u, 5u);
}

template <class F>
static float best_ms(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipEventDestroy(a); hipEventDestroy(b);
    return best;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *out = nullptr;
    CHK(hipMalloc(&out, 1u << 20));

    // int32: 8 waves per SIMD (32 per CU), 4096 iterations x 32 ops per lane
    const uint32_t blocks = (uint32_t)cus * 8u, iters = 4096u;
    const float ms_i = best_ms([&] { hipLaunchKernelGGL(k_int32, dim3(blocks), dim3(256), 0, 0, out, iters, 7u); }, 10);
    const double ops = (double)blocks * 256.0 * iters * 32.0;
    CHK(hipGetLastError());

    // HBM: 4 GiB read; 2 GiB + 2 GiB copy
    const size_t bytes = (size_t)4 << 30;
    uint4 *buf = nullptr;
    CHK(hipMalloc(&buf, bytes));
    const size_t n = bytes / 16;
    hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, buf, n);
    CHK(hipDeviceSynchronize());
    const uint32_t gb = (uint32_t)cus * 16u;
    const float ms_r = best_ms([&] { hipLaunchKernelGGL(k_read, dim3(gb), dim3(256), 0, 0, buf, n, out); }, 10);
    const float ms_c = best_ms([&] { hipLaunchKernelGGL(k_copy, dim3(gb), dim3(256), 0, 0, buf, buf + n / 2, n / 2); }, 10);
    CHK(hipGetLastError());
    CHK(hipFree(buf));
    CHK(hipFree(out));

    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %d, "
           "\"int32_tops\": %.3f, \"int32_ms\": %.4f, "
           "\"hbm_read_gbs\": %.1f, \"hbm_copy_gbs\": %.1f, \"read_ms\": %.4f, \"copy_ms\": %.4f}\n",
           prop.name, cus, prop.clockRate / 1000, ops / (ms_i * 1e-3) / 1e12, ms_i,
           (double)bytes / (ms_r * 1e-3) / 1e9, (double)bytes / (ms_c * 1e-3) / 1e9, ms_r, ms_c);
    return 0;
}
