// Inter-kernel gap on one stream: a chain of dependent kernels launched one by
// one vs the same chain captured once into a hipGraph and replayed.  Each
// kernel: G workgroups of 256 threads, each thread reads one float of the
// previous kernel's output and writes one (a real dependency), plus SPIN
// iterations of arithmetic so the kernel is not empty.
//   hipcc --offload-arch=gfx950 -O3 -o graph_gap graph_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void step(const float* in, float* out, int n, int spin) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float v = in[i];
    for (int k = 0; k < spin; ++k) v = fmaf(v, 1.0000001f, 1e-7f);
    out[i] = v;
}

int main() {
    int dev = 0;
    CK(hipSetDevice(dev));
    const int chain = 4, reps = 500;
    for (int G : {1024, 4096, 32768}) {
        for (int spin : {0, 200}) {
            const int n = G * 256;
            float *a, *b;
            CK(hipMalloc(&a, n * sizeof(float)));
            CK(hipMalloc(&b, n * sizeof(float)));
            CK(hipMemset(a, 0, n * sizeof(float)));
            hipStream_t s;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            auto enqueue = [&](int k) {
                for (int j = 0; j < chain; ++j) {
                    const bool even = ((k * chain + j) & 1) == 0;
                    hipLaunchKernelGGL(step, dim3(G), dim3(256), 0, s, even ? a : b, even ? b : a, n, spin);
                }
            };
            // warm-up
            for (int k = 0; k < 20; ++k) enqueue(k);
            CK(hipStreamSynchronize(s));
            // stream launches
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) enqueue(k);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms_stream = 0;
            CK(hipEventElapsedTime(&ms_stream, e0, e1));
            // one kernel alone, many times with no dependency chain? (same stream: still ordered)
            // graph: capture `chain` kernels (two iterations so the ping-pong closes)
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            enqueue(0);
            enqueue(1);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int k = 0; k < 10; ++k) CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps / 2; ++k) CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms_graph = 0;
            CK(hipEventElapsedTime(&ms_graph, e0, e1));
            // a big graph: 50 iterations captured
            hipGraph_t g2;
            hipGraphExec_t ge2;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int k = 0; k < 50; ++k) enqueue(k);
            CK(hipStreamEndCapture(s, &g2));
            CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge2, s));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps / 50; ++k) CK(hipGraphLaunch(ge2, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms_graph50 = 0;
            CK(hipEventElapsedTime(&ms_graph50, e0, e1));
            const double nk = (double)reps * chain;
            printf("G=%6d spin=%4d  per kernel: stream %.2f us  graph(8) %.2f us  graph(200) %.2f us\n", G, spin,
                   ms_stream * 1e3 / nk, ms_graph * 1e3 / nk, ms_graph50 * 1e3 / nk);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
            CK(hipGraphExecDestroy(ge2));
            CK(hipGraphDestroy(g2));
            CK(hipStreamDestroy(s));
            CK(hipFree(a));
            CK(hipFree(b));
        }
    }
    return 0;
}
