// Issue-rate probe for the issue-bound floors of kernels 1 and 2 (DESIGN.md
// §3.1, §3.2): how many wave-instructions of each class one CU issues per
// shader clock, by waves per SIMD.
//
//   salu:   16 independent s_add_u32 / s_xor_b32 chains per wave (inline asm)
//   valu:   16 independent v_add_u32 / v_xor_b32 chains per lane (inline asm)
//   mix:    both streams interleaved 1:1 in one wave (do SALU and VALU co-issue?)
//   branch: s_cmp + a never-taken s_cbranch_scc1, 16 per iteration
//
// Rate = wave-instructions / (CUs x clock x time).  Prints one JSON line.
// Build: hipcc --offload-arch=gfx950 -O3 issue_rates.hip -o issue_rates
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

#define S2(a, b) asm volatile("s_add_u32 %0, %0, %2\n\ts_xor_b32 %1, %1, %2" : "+s"(a), "+s"(b) : "s"(k) : "scc");
#define V2(a, b) asm volatile("v_add_u32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2" : "+v"(a), "+v"(b) : "v"(kv));

__global__ __launch_bounds__(256) void k_salu(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t k = __builtin_amdgcn_readfirstlane(seed | 1u);
    uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5, a6 = k + 6, a7 = k + 7;
    uint32_t b0 = k, b1 = k ^ 1, b2 = k ^ 2, b3 = k ^ 3, b4 = k ^ 4, b5 = k ^ 5, b6 = k ^ 6, b7 = k ^ 7;
    for (uint32_t i = 0; i < iters; ++i) {
        S2(a0, b0) S2(a1, b1) S2(a2, b2) S2(a3, b3) S2(a4, b4) S2(a5, b5) S2(a6, b6) S2(a7, b7)
    }
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
    if (r == 0x9e3779b9u) out[blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_valu(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t kv = seed | 1u;
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint32_t b0 = a0 ^ 9, b1 = a0 ^ 1, b2 = a0 ^ 2, b3 = a0 ^ 3, b4 = a0 ^ 4, b5 = a0 ^ 5, b6 = a0 ^ 6, b7 = a0 ^ 7;
    for (uint32_t i = 0; i < iters; ++i) {
        V2(a0, b0) V2(a1, b1) V2(a2, b2) V2(a3, b3) V2(a4, b4) V2(a5, b5) V2(a6, b6) V2(a7, b7)
    }
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
    if (r == 0x9e3779b9u) out[blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mix(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t k = __builtin_amdgcn_readfirstlane(seed | 1u);
    uint32_t kv = seed | 1u;
    uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, b0 = k, b1 = k ^ 1, b2 = k ^ 2, b3 = k ^ 3;
    uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, d0 = c0 ^ 9, d1 = c0 ^ 1, d2 = c0 ^ 2,
             d3 = c0 ^ 3;
    for (uint32_t i = 0; i < iters; ++i) {
        S2(a0, b0) V2(c0, d0) S2(a1, b1) V2(c1, d1) S2(a2, b2) V2(c2, d2) S2(a3, b3) V2(c3, d3)
    }
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3 ^ c0 ^ c1 ^ c2 ^ c3 ^ d0 ^ d1 ^ d2 ^ d3;
    if (r == 0x9e3779b9u) out[blockIdx.x] = r;
}

#define BR() asm volatile("s_cmp_eq_u32 %0, 0\n\ts_cbranch_scc1 1f\n1:" : : "s"(k) : "scc");

__global__ __launch_bounds__(256) void k_branch(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t k = __builtin_amdgcn_readfirstlane(seed | 1u);
    for (uint32_t i = 0; i < iters; ++i) {
        BR() BR() BR() BR() BR() BR() BR() BR()
    }
    if (k == 0x9e3779b9u) out[blockIdx.x] = k;
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
    const double clk = 2.4e9;
    uint32_t *out = nullptr;
    CHK(hipMalloc(&out, 1u << 20));
    const uint32_t iters = 4096u;
    printf("{\"cus\": %d, \"clock_assumed_mhz\": 2400, \"rates\": {", cus);
    const char *names[4] = {"salu", "valu", "mix", "branch"};
    // wave-instructions per wave per iteration (the loop's own s_add / s_cmp /
    // s_cbranch are counted apart: 3 SALU+branch per iteration)
    const double per_iter[4] = {16.0, 16.0, 16.0, 16.0};
    for (int kk = 0; kk < 4; ++kk) {
        printf("%s\"%s\": {", kk ? ", " : "", names[kk]);
        for (int wps = 1; wps <= 8; wps *= 2) {
            // wps blocks of 4 waves per CU: wps waves on each SIMD
            const uint32_t threads = 256u, nblk = (uint32_t)cus * (uint32_t)wps;
            auto launch = [&] {
                if (kk == 0) hipLaunchKernelGGL(k_salu, dim3(nblk), dim3(threads), 0, 0, out, iters, 7u);
                if (kk == 1) hipLaunchKernelGGL(k_valu, dim3(nblk), dim3(threads), 0, 0, out, iters, 7u);
                if (kk == 2) hipLaunchKernelGGL(k_mix, dim3(nblk), dim3(threads), 0, 0, out, iters, 7u);
                if (kk == 3) hipLaunchKernelGGL(k_branch, dim3(nblk), dim3(threads), 0, 0, out, iters, 7u);
            };
            const float ms = best_ms(launch, 8);
            CHK(hipGetLastError());
            const double waves_per_cu = 4.0 * wps;
            const double instr_per_cu = waves_per_cu * iters * per_iter[kk];
            const double per_clk = instr_per_cu / (ms * 1e-3 * clk);
            printf("%s\"%d\": {\"ms\": %.4f, \"wave_instr_per_cu_clk\": %.4f}", wps > 1 ? ", " : "", wps, ms,
                   per_clk);
        }
        printf("}");
    }
    printf("}}\n");
    CHK(hipFree(out));
    return 0;
}
