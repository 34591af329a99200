// launch_gap — the GPU-side cost of a chain of small dependent kernels on one stream, launched one by one or
// replayed from a captured hipGraph (is C1's ~5 us per launch gap something a graph removes?).
//   ./launch_gap [kernels per chain (48)] [chains (400)] [blocks per kernel (1024)]
// Prints one JSON line per mode: microseconds per chain and per kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// A little work per thread and one dependent value, so the chain is real.
__global__ __launch_bounds__(256) void step(unsigned *buf, unsigned n, unsigned k) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = buf[i] * 1664525u + k + buf[(i + 1) % n];
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 48;
    const int R = argc > 2 ? atoi(argv[2]) : 400;
    const unsigned blocks = argc > 3 ? (unsigned)atoi(argv[3]) : 1024u;
    const unsigned n = blocks * 256u;
    unsigned *buf;
    CK(hipMalloc(&buf, n * sizeof(unsigned)));
    CK(hipMemset(buf, 0, n * sizeof(unsigned)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto chain = [&](void) {
        for (int k = 0; k < K; k++) step<<<blocks, 256, 0, st>>>(buf, n, (unsigned)k);
    };
    // 1) plain launches
    for (int w = 0; w < 20; w++) chain();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; r++) chain();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"mode\": \"stream\", \"kernels\": %d, \"blocks\": %u, \"us_per_chain\": %.2f, \"us_per_kernel\": %.3f}\n",
           K, blocks, 1e3 * ms / R, 1e3 * ms / R / K);
    // 2) one captured chain replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    chain();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 20; w++) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"mode\": \"graph\", \"kernels\": %d, \"blocks\": %u, \"us_per_chain\": %.2f, \"us_per_kernel\": %.3f}\n",
           K, blocks, 1e3 * ms / R, 1e3 * ms / R / K);
    // 3) a single kernel per chain: the kernel's own duration
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; r++) step<<<blocks, 256, 0, st>>>(buf, n, 1u);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"mode\": \"stream_single\", \"kernels\": 1, \"blocks\": %u, \"us_per_kernel\": %.3f}\n", blocks,
           1e3 * ms / R);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(buf));
    return 0;
}
