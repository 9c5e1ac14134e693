// Launch-cost probe: event-timed launches of near-empty kernels with the
// shape of k_lane_step (256 x 256 threads) and, separately, its dynamic LDS
// (134 KiB) and per-lane scratch (672 B), to attribute kernel 1's fixed cost.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(int *out) {
    if (threadIdx.x == 0 && blockIdx.x == 100000) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_lds(int *out) {
    extern __shared__ int dyn[];
    dyn[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (dyn[(threadIdx.x + 1) & 255] == 7 && blockIdx.x == 100000) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_scratch(int *out, int k) {
    volatile int buf[168];
    for (int i = 0; i < 168; ++i) buf[i] = i * k;
    if (buf[(threadIdx.x + k) % 168] == -5) out[0] = 1;
}

template <class F>
static float timeit(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 20; ++r) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best * 1000.f;
}

int main() {
    int *out; hipMalloc(&out, 4);
    const size_t lds = 134 * 1024;
    hipFuncSetAttribute((const void *)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
    printf("empty            %7.1f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, out); }));
    printf("lds 134 KiB      %7.1f us\n", timeit([&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(256), lds, 0, out); }));
    printf("lds 64 KiB       %7.1f us\n", timeit([&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(256), 64 * 1024, 0, out); }));
    printf("scratch 672 B    %7.1f us\n", timeit([&] { hipLaunchKernelGGL(k_scratch, dim3(256), dim3(256), 0, 0, out, 3); }));
    printf("empty 1024 blk   %7.1f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, 0, out); }));
    return 0;
}
