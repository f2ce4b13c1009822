// Inter-kernel gap probe (experiment, not product code): back-to-back launches on one stream of
//   W: 2073600 threads each storing 3 doubles (a C2-sized f64 image, 49.8 MB) with ordinary stores,
//   N: the same with nontemporal stores, Z: the same grid with no stores.
// Run under rocprofv3 --kernel-trace; tools/probes/gap_stats.py reads the gaps.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) store_w(double* out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        out[3 * i] = 1.0 * i;
        out[3 * i + 1] = 2.0 * i;
        out[3 * i + 2] = 3.0 * i;
    }
}
__global__ void __launch_bounds__(256) store_n(double* out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        __builtin_nontemporal_store(1.0 * i, out + 3 * i);
        __builtin_nontemporal_store(2.0 * i, out + 3 * i + 1);
        __builtin_nontemporal_store(3.0 * i, out + 3 * i + 2);
    }
}
__global__ void __launch_bounds__(256) store_z(double* out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == n) out[0] = 0.0;  // never true
}

int main() {
    const int n = 1920 * 1080;
    double* out = nullptr;
    if (hipMalloc(&out, (size_t)n * 3 * sizeof(double)) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 1;
    const dim3 grid((n + 255) / 256), block(256);
    for (int pass = 0; pass < 3; ++pass) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, st);
        for (int k = 0; k < 100; ++k) {
            if (pass == 0) hipLaunchKernelGGL(store_w, grid, block, 0, st, out, n);
            if (pass == 1) hipLaunchKernelGGL(store_n, grid, block, 0, st, out, n);
            if (pass == 2) hipLaunchKernelGGL(store_z, grid, block, 0, st, out, n);
        }
        (void)hipEventRecord(e1, st);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%s: %.2f us per launch (100 back-to-back)\n", pass == 0 ? "ordinary" : pass == 1 ? "nontemporal" : "no stores",
               ms * 10.0f);
    }
    (void)hipFree(out);
    return 0;
}
