// microbenchmark: one grid-wide barrier inside a kernel whose blocks are all co-resident,
// against the same two phases as two dependent launches in a HIP graph (1M and 8M elements).
//   phase 1: read w (f64), write one partial per 1024-element tile
//   phase 2: read w again + every tile partial before it in its group, write a u32 per element
// The barrier: thread 0 of each block fences, adds 1 to a per-launch counter, and polls it
// with s_sleep until all blocks arrived (bounded by a deadline so a missing block reports a
// timeout instead of hanging). The grid is capped at the occupancy-derived resident count and
// loops over tiles, so every block is resident by construction.
// Diagnostics only (tools/).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kB = 256, kTile = 1024;

__device__ __forceinline__ double tile_work(const double* __restrict__ w, int64_t n, int64_t tile) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kTile / kB; ++k) {
        const int64_t i = tile * kTile + k * kB + threadIdx.x;
        if (i < n) s += w[i];
    }
    return s;
}

__global__ __launch_bounds__(kB) void k_p1(const double* __restrict__ w, int64_t n, double* __restrict__ part) {
    __shared__ double red[kB / 64];
    double s = tile_work(w, n, blockIdx.x);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ __launch_bounds__(kB) void k_p2(const double* __restrict__ w, int64_t n, const double* __restrict__ part,
                                           uint32_t* __restrict__ out) {
    const double off = part[blockIdx.x > 0 ? blockIdx.x - 1 : 0];
#pragma unroll
    for (int k = 0; k < kTile / kB; ++k) {
        const int64_t i = (int64_t)blockIdx.x * kTile + k * kB + threadIdx.x;
        if (i < n) out[i] = (uint32_t)(w[i] + off);
    }
}

__device__ __forceinline__ bool gbar(unsigned* ctr, unsigned nblocks, int* timeout) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nblocks) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {   // 100 ms at 100 MHz
                __hip_atomic_store(timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
    return !__hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kB) void k_fused(const double* __restrict__ w, int64_t n, double* __restrict__ part,
                                              uint32_t* __restrict__ out, unsigned* ctr, int* timeout) {
    __shared__ double red[kB / 64];
    const int64_t ntiles = (n + kTile - 1) / kTile;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        double s = tile_work(w, n, t);
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) part[t] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
    if (!gbar(ctr, gridDim.x, timeout)) return;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const double off = part[t > 0 ? t - 1 : 0];
#pragma unroll
        for (int k = 0; k < kTile / kB; ++k) {
            const int64_t i = t * kTile + k * kB + threadIdx.x;
            if (i < n) out[i] = (uint32_t)(w[i] + off);
        }
    }
}

int main() {
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused, kB, 0));
    printf("CUs %d, resident blocks/CU for the fused kernel %d\n", ncu, occ);
    const int R = 200;
    for (int64_t n : {1000000ll, 8000000ll}) {
        const int64_t ntiles = (n + kTile - 1) / kTile;
        double *w, *part;
        uint32_t* out;
        unsigned* ctr;
        int* timeout;
        CK(hipMalloc(&w, sizeof(double) * n));
        CK(hipMalloc(&part, sizeof(double) * ntiles));
        CK(hipMalloc(&out, sizeof(uint32_t) * n));
        CK(hipMalloc(&ctr, sizeof(unsigned) * 64 * R));
        CK(hipMalloc(&timeout, 64));
        CK(hipMemset(w, 0, sizeof(double) * n));
        CK(hipMemset(timeout, 0, 64));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float ms;
        for (int variant = 0; variant < 3; ++variant) {
            const unsigned grid = variant == 0 ? 0u
                                  : (unsigned)(ntiles < (int64_t)ncu * occ ? ntiles : (int64_t)ncu * occ) /
                                        (variant == 2 ? 2u : 1u);
            hipGraph_t graph;
            hipGraphExec_t exec;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            CK(hipMemsetAsync(ctr, 0, sizeof(unsigned) * 64 * R, s));
            for (int r = 0; r < R; ++r) {
                if (variant == 0) {
                    hipLaunchKernelGGL(k_p1, dim3((unsigned)ntiles), dim3(kB), 0, s, w, n, part);
                    hipLaunchKernelGGL(k_p2, dim3((unsigned)ntiles), dim3(kB), 0, s, w, n, part, out);
                } else {
                    hipLaunchKernelGGL(k_fused, dim3(grid), dim3(kB), 0, s, w, n, part, out, ctr + 64 * r, timeout);
                }
            }
            CK(hipStreamEndCapture(s, &graph));
            CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
            CK(hipGraphLaunch(exec, s));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int w2 = 0; w2 < 3; ++w2) CK(hipGraphLaunch(exec, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            int to = 0;
            CK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
            printf("n=%lld %s grid %u: %.2f us per two-phase step%s\n", (long long)n,
                   variant == 0 ? "two launches      " : "one launch+barrier", variant == 0 ? (unsigned)ntiles : grid,
                   ms * 1e3 / (3 * R), to ? "  TIMEOUT" : "");
            CK(hipGraphExecDestroy(exec));
            CK(hipGraphDestroy(graph));
            if (to) return 2;
        }
        CK(hipFree(w)); CK(hipFree(part)); CK(hipFree(out)); CK(hipFree(ctr)); CK(hipFree(timeout));
    }
    return 0;
}
