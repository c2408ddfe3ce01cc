// A libwsmc-free shape of the fused run's submission (the rocprofv3 crash of
// r03): one HIP graph of 3 x T streaming-kernel nodes captured from a stream, replayed R times,
// then synchronised. Run under `rocprofv3 --kernel-trace --stats` to see whether the tracer
// alone fails on R x 3T graph-launched dispatches.
//   tools/micro/graph_trace [T=100] [R=300] [N=1000000]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_a(const double* x, double* y, long n) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = x[i] * 1.0000001 + 1.0;
}
__global__ void k_b(const double* y, unsigned long long* q, long n) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) q[i] = (unsigned long long)(y[i] * 16.0);
}
__global__ void k_c(const unsigned long long* q, int* a, long n) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) a[i] = (int)(q[i] % (unsigned long long)n);
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 100;
    const int R = argc > 2 ? atoi(argv[2]) : 300;
    const long n = argc > 3 ? atol(argv[3]) : 1000000;
    double *x, *y;
    unsigned long long* q;
    int* a;
    CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&y, n * 8)); CK(hipMalloc(&q, n * 8)); CK(hipMalloc(&a, n * 4));
    CK(hipMemset(x, 0, n * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipGraph_t g;
    hipGraphExec_t ge;
    const dim3 grid((unsigned)((n + 255) / 256));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int t = 0; t < T; ++t) {
        hipLaunchKernelGGL(k_a, grid, dim3(256), 0, s, x, y, n);
        hipLaunchKernelGGL(k_b, grid, dim3(256), 0, s, y, q, n);
        hipLaunchKernelGGL(k_c, grid, dim3(256), 0, s, q, a, n);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    printf("graph_trace: %d replays of %d kernel nodes, %d dispatches: ok\n", R, 3 * T, 3 * T * R);
    return 0;
}
