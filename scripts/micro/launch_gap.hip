// Dependent-launch gap on one stream: K launches of a VALU-bound kernel of
// about the duration of a 4096^2 10-generation pass (2048 waves, ~16 us),
// issued (a) one by one on a stream, (b) as a captured hipGraph replayed.
// Gap per launch = (window - K x single) / K.  Answers whether the 4096^2
// wall-vs-kernel difference (5 us per launch) is a launch cost a graph
// removes.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/micro/launch_gap scripts/micro/launch_gap.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(256) void spin(uint32_t* out, int iters) {
    uint32_t a = threadIdx.x * 2654435761u + blockIdx.x, b = a ^ 0x9E3779B9u;
    for (int i = 0; i < iters; ++i) {
        a = __builtin_amdgcn_alignbit(a, b, 7) ^ b;
        b = (b + a) | (a >> 3);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b;  // vector store
}

int main(int argc, char** argv) {
    const int K = 100, blocks = 512;  // 512 x 4 waves = 2048 waves
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
    uint32_t* out;
    CK(hipMalloc(&out, blocks * 256 * sizeof(uint32_t)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 20; ++w) spin<<<blocks, 256, 0, st>>>(out, iters);
    CK(hipStreamSynchronize(st));

    // single launch duration (min of 20)
    float single = 1e30f;
    for (int r = 0; r < 20; ++r) {
        CK(hipEventRecord(e0, st));
        spin<<<blocks, 256, 0, st>>>(out, iters);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < single) single = ms;
    }
    // (a) stream
    float stream_ms = 1e30f, stream_wall = 1e30f;
    for (int r = 0; r < 5; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, st));
        for (int k = 0; k < K; ++k) spin<<<blocks, 256, 0, st>>>(out, iters);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        auto t1 = std::chrono::steady_clock::now();
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < stream_ms) stream_ms = ms;
        const float wall = std::chrono::duration<float, std::milli>(t1 - t0).count();
        if (wall < stream_wall) stream_wall = wall;
    }
    // (b) graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) spin<<<blocks, 256, 0, st>>>(out, iters);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    float graph_ms = 1e30f, graph_wall = 1e30f;
    for (int r = 0; r < 5; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        auto t1 = std::chrono::steady_clock::now();
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < graph_ms) graph_ms = ms;
        const float wall = std::chrono::duration<float, std::milli>(t1 - t0).count();
        if (wall < graph_wall) graph_wall = wall;
    }
    std::printf("iters=%d single_us=%.2f | stream: window_us/launch=%.2f gap_us=%.2f wall_us/launch=%.2f | "
                "graph: window_us/launch=%.2f gap_us=%.2f wall_us/launch=%.2f\n",
                iters, single * 1e3, stream_ms * 1e3 / K, (stream_ms - K * single) * 1e3 / K, stream_wall * 1e3 / K,
                graph_ms * 1e3 / K, (graph_ms - K * single) * 1e3 / K, graph_wall * 1e3 / K);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(out));
    return 0;
}
