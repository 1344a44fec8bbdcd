// Achievable HBM copy bandwidth on this device (the ceiling of a
// one-generation pass, which reads one plane and writes one): 512 MiB ->
// 512 MiB float4 copies, plain vs non-temporal loads / stores, grid-stride.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void copy_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint4 v;
        if constexpr (MODE & 1) {
            v.x = __builtin_nontemporal_load(&a[i].x); v.y = __builtin_nontemporal_load(&a[i].y);
            v.z = __builtin_nontemporal_load(&a[i].z); v.w = __builtin_nontemporal_load(&a[i].w);
        } else {
            v = a[i];
        }
        if constexpr (MODE & 2) {
            __builtin_nontemporal_store(v.x, &b[i].x); __builtin_nontemporal_store(v.y, &b[i].y);
            __builtin_nontemporal_store(v.z, &b[i].z); __builtin_nontemporal_store(v.w, &b[i].w);
        } else {
            b[i] = v;
        }
    }
}

template <int MODE>
int run(const char* name, const uint4* a, uint4* b, size_t n, int blocks) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(copy_k<MODE>, dim3(blocks), dim3(256), 0, 0, a, b, n);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 20; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(copy_k<MODE>, dim3(blocks), dim3(256), 0, 0, a, b, n);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    printf("%-28s blocks=%6d %.4f ms  %.0f GB/s (read + write)\n", name, blocks, best, 2.0 * n * 16 / (best * 1e-3) / 1e9);
    return 0;
}

int main() {
    const size_t bytes = 512ull << 20, n = bytes / 16;
    uint4 *a, *b;
    CHK(hipMalloc(&a, bytes)); CHK(hipMalloc(&b, bytes));
    CHK(hipMemset(a, 0x5a, bytes)); CHK(hipMemset(b, 0, bytes));
    hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
    for (int per_cu : {8, 32, 128}) {
        const int blocks = prop.multiProcessorCount * per_cu;
        run<0>("plain", a, b, n, blocks);
        run<2>("nt stores", a, b, n, blocks);
        run<1>("nt loads", a, b, n, blocks);
        run<3>("nt loads + nt stores", a, b, n, blocks);
    }
    return 0;
}
