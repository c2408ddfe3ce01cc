// microbenchmark: what a dependent phase boundary costs on one MI355X.
//  (a) a HIP graph of R launches of a small streaming kernel (1M doubles read + written),
//      back to back on one stream;
//  (b) one persistent launch doing the same R phases separated by a device-wide barrier
//      (atomic arrive + spin on a generation word, bounded by a 200 ms deadline so a
//      missing block can never hang the GPU: the kernel then reports a timeout);
//  (c) the same persistent launch without barriers (the phases' own cost).
// Diagnostics only (tools/).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_phase(const double* __restrict__ a, double* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i] + 1.0;
}

__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned& my_gen,
                                             int* timeout) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned target = my_gen + 1;
        if (atomicAdd(count, 1u) == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // 200 ms at 100 MHz
                    atomicExch(timeout, 1);
                    ok = false;
                    break;
                }
            }
        }
        my_gen = target;
    }
    __syncthreads();
    return ok && !__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool BAR>
__global__ __launch_bounds__(256) void k_persist(double* a, double* b, int64_t n, int rounds, unsigned* count,
                                                 unsigned* gen, int* timeout) {
    unsigned my_gen = 0;
    if (threadIdx.x == 0) my_gen = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    for (int r = 0; r < rounds; ++r) {
        const double* src = (r & 1) ? b : a;
        double* dst = (r & 1) ? a : b;
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
            dst[i] = src[i] + 1.0;
        if (BAR && !grid_barrier(count, gen, gridDim.x, my_gen, timeout)) return;
    }
}

int main() {
    const int64_t n = 1000000;
    const int R = 300;
    double *a, *b;
    unsigned *count, *gen;
    int* timeout;
    CK(hipMalloc(&a, sizeof(double) * n));
    CK(hipMalloc(&b, sizeof(double) * n));
    CK(hipMalloc(&count, 256));
    CK(hipMalloc(&gen, 256));
    CK(hipMalloc(&timeout, 256));
    CK(hipMemset(a, 0, sizeof(double) * n));
    CK(hipMemset(count, 0, 256));
    CK(hipMemset(gen, 0, 256));
    CK(hipMemset(timeout, 0, 256));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    // (a) graph of R launches (the fused run's grid shape: one thread per element)
    const dim3 g1((unsigned)((n + 255) / 256));
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_phase, g1, dim3(256), 0, s, (r & 1) ? b : a, (r & 1) ? a : b, n);
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(exec, s));
    CK(hipEventRecord(e0, s));
    for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(exec, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph: %d launches of a 1M-element phase: %.2f us per phase\n", R, ms * 1e3 / (5 * R));
    // (b), (c) persistent: one block per CU x k
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    for (int per : {1, 2, 4, 8}) {
        const dim3 g2((unsigned)(ncu * per));
        for (int bar = 0; bar < 2; ++bar) {
            for (int w = 0; w < 2; ++w) {
                if (bar) hipLaunchKernelGGL(k_persist<true>, g2, dim3(256), 0, s, a, b, n, R, count, gen, timeout);
                else hipLaunchKernelGGL(k_persist<false>, g2, dim3(256), 0, s, a, b, n, R, count, gen, timeout);
            }
            CK(hipEventRecord(e0, s));
            for (int w = 0; w < 5; ++w) {
                if (bar) hipLaunchKernelGGL(k_persist<true>, g2, dim3(256), 0, s, a, b, n, R, count, gen, timeout);
                else hipLaunchKernelGGL(k_persist<false>, g2, dim3(256), 0, s, a, b, n, R, count, gen, timeout);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            int to = 0;
            CK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
            printf("persistent %d blocks (%d/CU) %s: %.2f us per phase%s\n", ncu * per, per,
                   bar ? "with grid barrier" : "no barrier     ", ms * 1e3 / (5 * R), to ? "  TIMEOUT" : "");
            if (to) return 2;
        }
    }
    return 0;
}
