// microbenchmark: cost of the canonical draw pieces (Philox4x32-10, log, sincos2pi, sqrt,
// Box–Muller pair) per element on one MI355X. Diagnostics only (tools/).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "wsmc_math.h"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
template <int K>
__global__ __launch_bounds__(256) void kb(double* out, int64_t n, uint64_t seed, uint64_t op) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double r0 = 0, r1 = 0;
    if (K == 0) { wsmc_normal_pair(wsmc_rng_block(seed, op, (uint64_t)i, 0u), &r0, &r1); }
    if (K == 1) { wsmc_u32x4 w = wsmc_rng_block(seed, op, (uint64_t)i, 0u); r0 = (double)(w.v[0] ^ w.v[1] ^ w.v[2] ^ w.v[3]); }
    if (K == 2) { r0 = wsmc_log((double)(i + 1) * 1e-7); }
    if (K == 3) { wsmc_sincos2pi((double)i * 1e-7, &r0, &r1); }
    if (K == 4) { r0 = wsmc_sqrt((double)(i + 1)); }
    if (K == 5) { r0 = wsmc_expw(-(double)i * 1e-6); }
    if (K == 6) { r0 = (double)i; }
    out[i] = r0 + r1;
}
template <int K>
static float run(double* d, int64_t n, hipEvent_t a, hipEvent_t b) {
    dim3 g((unsigned)((n + 255) / 256));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kb<K>, g, dim3(256), 0, 0, d, n, 42ull, 7ull);
    hipEventRecord(a);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kb<K>, g, dim3(256), 0, 0, d, n, 42ull, 7ull);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}
int main() {
    const char* names[] = {"normal_pair", "philox", "log", "sincos2pi", "sqrt", "expw", "store-only"};
    for (int64_t n : {1000000ll, 16000000ll}) {
        double* d; CK(hipMalloc(&d, sizeof(double) * n));
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        float t[7] = {run<0>(d, n, a, b), run<1>(d, n, a, b), run<2>(d, n, a, b), run<3>(d, n, a, b),
                      run<4>(d, n, a, b), run<5>(d, n, a, b), run<6>(d, n, a, b)};
        for (int k = 0; k < 7; ++k) printf("n=%lld %-12s %8.2f us  %.3f ns/elem\n", (long long)n, names[k], t[k] * 1e3, t[k] * 1e6 / n);
        CK(hipFree(d));
    }
    return 0;
}
