// microbenchmark (round 3): a properly built device-wide barrier against a
// kernel boundary, for the C2 resample leg's two phases (statistics -> fill).
//   phase 1: read w (f64), write one partial per 1024-element tile
//   phase 2: read w again + the tile partial before it, write a u32 per element
// Barrier (placement-independent; the b % 8 grouping only makes the groups likely to share an
// XCD): every block's lane 0, after its stores drained and one agent-scope release fence,
// adds to its group's counter (8 groups, one 128-B line each, blocks b with b % 8 == g). The
// last arriver of a group adds to the top counter; the last of those bumps the generation
// word. Everyone polls the generation with relaxed agent loads + s_sleep, then one agent
// acquire fence. Counters are per launch (zeroed by a memset node); every spin is bounded
// (a timeout flag instead of a hang). Grids are 1 / 2 / 4 blocks per CU, all resident.
// Diagnostics only (tools/); results in DESIGN.md §3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kB = 256, kTile = 1024, kGroups = 8, kLine = 32;   // 32 u32 = one 128-B line

__device__ __forceinline__ double tile_sum(const double* __restrict__ w, int64_t n, int64_t tile) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kTile / kB; ++k) {
        const int64_t i = tile * kTile + k * kB + threadIdx.x;
        if (i < n) s += w[i];
    }
    return s;
}
__device__ __forceinline__ void block_partial(double s, double* red, double* dst) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *dst = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
}

__global__ __launch_bounds__(kB) void k_p1(const double* __restrict__ w, int64_t n, double* __restrict__ part) {
    __shared__ double red[kB / 64];
    block_partial(tile_sum(w, n, blockIdx.x), red, part + blockIdx.x);
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
__global__ void k_empty() {}

// ctr: [kGroups + 2][kLine] u32 — group counters, the top counter, the generation word
__device__ __forceinline__ bool xbar(uint32_t* ctr, int* timeout) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned G = gridDim.x, g = blockIdx.x % kGroups;
        const unsigned members = G / kGroups + (g < G % kGroups ? 1u : 0u);
        const unsigned ngroups = G < (unsigned)kGroups ? G : (unsigned)kGroups;
        uint32_t* gen = ctr + (kGroups + 1) * kLine;
        const uint32_t old = __hip_atomic_fetch_add(ctr + g * kLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == members - 1) {
            const uint32_t top = __hip_atomic_fetch_add(ctr + kGroups * kLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (top == ngroups - 1) __hip_atomic_store(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {   // 100 ms at 100 MHz
                __hip_atomic_store(timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return true;
}

__global__ __launch_bounds__(kB) void k_fused(const double* __restrict__ w, int64_t n, double* __restrict__ part,
                                              uint32_t* __restrict__ out, uint32_t* ctr, int* timeout) {
    __shared__ double red[kB / 64];
    const int64_t ntiles = (n + kTile - 1) / kTile;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) block_partial(tile_sum(w, n, t), red, part + t);
    xbar(ctr, timeout);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const double off = part[t > 0 ? t - 1 : 0];
#pragma unroll
        for (int k = 0; k < kTile / kB; ++k) {
            const int64_t i = t * kTile + k * kB + threadIdx.x;
            if (i < n) out[i] = (uint32_t)(w[i] + off);
        }
    }
}
__global__ __launch_bounds__(kB) void k_bar_only(uint32_t* ctr, int* timeout) { xbar(ctr, timeout); }

int main() {
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused, kB, 0));
    printf("CUs %d, occupancy API blocks/CU %d (grids used: 1, 2, 4 per CU)\n", ncu, occ);
    if (occ < 5) { printf("occupancy too low for the 4-per-CU grid\n"); return 3; }
    const int R = 200;
    const size_t ctr_words = (size_t)(kGroups + 2) * kLine;
    uint32_t* ctr;
    int* timeout;
    CK(hipMalloc(&ctr, sizeof(uint32_t) * ctr_words * R));
    CK(hipMalloc(&timeout, 64));
    CK(hipMemset(timeout, 0, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto enqueue, const char* what) -> int {
        hipGraph_t graph;
        hipGraphExec_t exec;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        CK(hipMemsetAsync(ctr, 0, sizeof(uint32_t) * ctr_words * R, s));
        for (int r = 0; r < R; ++r) enqueue(r);
        CK(hipStreamEndCapture(s, &graph));
        CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        CK(hipGraphLaunch(exec, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 3; ++k) CK(hipGraphLaunch(exec, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        int to = 0;
        CK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
        printf("%-58s %8.2f us per step%s\n", what, ms * 1e3 / (3 * R), to ? "  TIMEOUT" : "");
        CK(hipGraphExecDestroy(exec));
        CK(hipGraphDestroy(graph));
        return to ? 2 : 0;
    };
    char name[128];
    // barrier alone vs a boundary alone
    if (timed([&](int) { hipLaunchKernelGGL(k_empty, dim3(256), dim3(kB), 0, s); hipLaunchKernelGGL(k_empty, dim3(256), dim3(kB), 0, s); },
              "two empty launches (one boundary)")) return 2;
    for (int per : {1, 2, 4}) {
        const unsigned grid = (unsigned)(ncu * per);
        snprintf(name, sizeof name, "one launch, barrier only, grid %u", grid);
        if (timed([&](int r) { hipLaunchKernelGGL(k_bar_only, dim3(grid), dim3(kB), 0, s, ctr + ctr_words * r, timeout); },
                  name)) return 2;
    }
    for (int64_t n : {1000000ll, 8000000ll}) {
        const int64_t ntiles = (n + kTile - 1) / kTile;
        double *w, *part;
        uint32_t* out;
        CK(hipMalloc(&w, sizeof(double) * n));
        CK(hipMalloc(&part, sizeof(double) * ntiles));
        CK(hipMalloc(&out, sizeof(uint32_t) * n));
        CK(hipMemset(w, 0, sizeof(double) * n));
        snprintf(name, sizeof name, "n=%lld two launches (grid %lld each)", (long long)n, (long long)ntiles);
        if (timed([&](int) {
                hipLaunchKernelGGL(k_p1, dim3((unsigned)ntiles), dim3(kB), 0, s, w, n, part);
                hipLaunchKernelGGL(k_p2, dim3((unsigned)ntiles), dim3(kB), 0, s, w, n, part, out);
            }, name)) return 2;
        for (int per : {1, 2, 4}) {
            const unsigned grid = (unsigned)(ncu * per);
            snprintf(name, sizeof name, "n=%lld one launch + XCD-grouped barrier, grid %u", (long long)n, grid);
            if (timed([&](int r) {
                    hipLaunchKernelGGL(k_fused, dim3(grid), dim3(kB), 0, s, w, n, part, out, ctr + ctr_words * r, timeout);
                }, name)) return 2;
        }
        CK(hipFree(w)); CK(hipFree(part)); CK(hipFree(out));
    }
    CK(hipFree(ctr)); CK(hipFree(timeout));
    return 0;
}
