// A libwsmc-free shape of the fused run's submission (the rocprofv3 crash of
// r03): one HIP graph of 3 x T streaming-kernel nodes captured from a stream, replayed R times,
// then synchronised. Run under `rocprofv3 --kernel-trace --stats` to see whether the tracer
// alone fails on R x 3T graph-launched dispatches.
//   tools/micro/graph_trace [T=100] [R=300] [N=1000000] [sync=0: 1 synchronises after every replay]
//                           [graph=1: 0 launches the same kernels on the stream, no graph]
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
    const int sync_each = argc > 4 ? atoi(argv[4]) : 0;
    const int use_graph = argc > 5 ? atoi(argv[5]) : 1;
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
    auto enqueue = [&]() {
        for (int t = 0; t < T; ++t) {
            hipLaunchKernelGGL(k_a, grid, dim3(256), 0, s, x, y, n);
            hipLaunchKernelGGL(k_b, grid, dim3(256), 0, s, y, q, n);
            hipLaunchKernelGGL(k_c, grid, dim3(256), 0, s, q, a, n);
        }
    };
    if (use_graph) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        enqueue();
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    for (int r = 0; r < R; ++r) {
        if (use_graph)
            CK(hipGraphLaunch(ge, s));
        else
            enqueue();
        if (sync_each) CK(hipStreamSynchronize(s));
    }
    CK(hipStreamSynchronize(s));
    printf("graph_trace: %d %s of %d kernels, %d dispatches%s: ok\n", R, use_graph ? "graph replays" : "stream runs",
           3 * T, 3 * T * R, sync_each ? ", synchronised after each" : "");
    return 0;
}
