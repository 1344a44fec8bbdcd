// Achievable HBM copy bandwidth on this device (the ceiling of a
// one-generation pass, which reads one plane and writes one): N -> N byte
// uint4 copies, plain vs non-temporal loads / stores: grid-stride loops with
// 1 or 4 uint4 per thread and iteration, and one-shot tiles of 1-8 uint4 per
// thread (U x 4 KiB per block), at the 65536^2 plane (512 MiB) and at a
// 2 GiB plane.  Prints one line per variant and, last, a JSON line with the
// best rate -- bench.py reads it from profiles/copy_peak.json as the
// measured stream-copy peak.
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/copy_bw.hip -o scripts/micro/copy_bw
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE, int U>
__global__ __launch_bounds__(256) void copy_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + u * stride;
            if (i >= n) break;
            if constexpr (MODE & 1) {
                v[u].x = __builtin_nontemporal_load(&a[i].x); v[u].y = __builtin_nontemporal_load(&a[i].y);
                v[u].z = __builtin_nontemporal_load(&a[i].z); v[u].w = __builtin_nontemporal_load(&a[i].w);
            } else {
                v[u] = a[i];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + u * stride;
            if (i >= n) break;
            if constexpr (MODE & 2) {
                __builtin_nontemporal_store(v[u].x, &b[i].x); __builtin_nontemporal_store(v[u].y, &b[i].y);
                __builtin_nontemporal_store(v[u].z, &b[i].z); __builtin_nontemporal_store(v[u].w, &b[i].w);
            } else {
                b[i] = v[u];
            }
        }
    }
}

// One-shot tiles: block b copies U x 256 consecutive uint4 (U x 4 KiB), each
// wave-instruction 1 KiB contiguous, all U loads issued before the stores --
// no grid-stride loop, so every wave has U loads in flight from its start.
template <int MODE, int U>
__global__ __launch_bounds__(256) void copy_tile_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            if constexpr (MODE & 1) {
                v[u].x = __builtin_nontemporal_load(&a[i].x); v[u].y = __builtin_nontemporal_load(&a[i].y);
                v[u].z = __builtin_nontemporal_load(&a[i].z); v[u].w = __builtin_nontemporal_load(&a[i].w);
            } else {
                v[u] = a[i];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            if constexpr (MODE & 2) {
                __builtin_nontemporal_store(v[u].x, &b[i].x); __builtin_nontemporal_store(v[u].y, &b[i].y);
                __builtin_nontemporal_store(v[u].z, &b[i].z); __builtin_nontemporal_store(v[u].w, &b[i].w);
            } else {
                b[i] = v[u];
            }
        }
    }
}

static double g_best = 0;
static char g_best_name[96];

template <int MODE, int U>
int run(const char* name, const uint4* a, uint4* b, size_t n, int blocks) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((copy_k<MODE, U>), dim3(blocks), dim3(256), 0, 0, a, b, n);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 20; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((copy_k<MODE, U>), dim3(blocks), dim3(256), 0, 0, a, b, n);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    const double gbs = 2.0 * n * 16 / (best * 1e-3) / 1e9;
    printf("%-22s x%d %5zu MiB blocks=%6d %.4f ms  %.0f GB/s (read + write)\n", name, U, n * 16 >> 20, blocks, best, gbs);
    if (gbs > g_best) {
        g_best = gbs;
        snprintf(g_best_name, sizeof g_best_name, "%s x%d, %zu MiB, %d blocks", name, U, n * 16 >> 20, blocks);
    }
    CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    return 0;
}

template <int MODE, int U>
int run_tile(const char* name, const uint4* a, uint4* b, size_t n) {
    const int blocks = (int)((n + 256 * U - 1) / (256 * U));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((copy_tile_k<MODE, U>), dim3(blocks), dim3(256), 0, 0, a, b, n);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 20; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((copy_tile_k<MODE, U>), dim3(blocks), dim3(256), 0, 0, a, b, n);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    const double gbs = 2.0 * n * 16 / (best * 1e-3) / 1e9;
    printf("tile %-17s x%d %5zu MiB blocks=%6d %.4f ms  %.0f GB/s (read + write)\n", name, U, n * 16 >> 20, blocks, best, gbs);
    if (gbs > g_best) {
        g_best = gbs;
        snprintf(g_best_name, sizeof g_best_name, "tile %s x%d, %zu MiB, %d blocks", name, U, n * 16 >> 20, blocks);
    }
    CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    return 0;
}

int main() {
    hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
    for (size_t mib : {512, 2048}) {
        const size_t bytes = mib << 20, n = bytes / 16;
        uint4 *a, *b;
        CHK(hipMalloc(&a, bytes)); CHK(hipMalloc(&b, bytes));
        CHK(hipMemset(a, 0x5a, bytes)); CHK(hipMemset(b, 0, bytes));
        for (int per_cu : {8, 32, 128}) {
            const int blocks = prop.multiProcessorCount * per_cu;
            if (run<0, 1>("plain", a, b, n, blocks) || run<2, 1>("nt stores", a, b, n, blocks) ||
                run<3, 1>("nt loads + nt stores", a, b, n, blocks) || run<0, 4>("plain", a, b, n, blocks) ||
                run<3, 4>("nt loads + nt stores", a, b, n, blocks))
                return 1;
        }
        if (run_tile<0, 1>("plain", a, b, n) || run_tile<0, 4>("plain", a, b, n) || run_tile<0, 8>("plain", a, b, n) ||
            run_tile<3, 1>("nt loads + nt stores", a, b, n) || run_tile<3, 4>("nt loads + nt stores", a, b, n) ||
            run_tile<3, 8>("nt loads + nt stores", a, b, n) || run_tile<2, 4>("nt stores", a, b, n))
            return 1;
        CHK(hipFree(a)); CHK(hipFree(b));
    }
    printf("{\"copy_peak_gbs\": %.1f, \"variant\": \"%s\", \"device\": \"%s\", \"cus\": %d}\n", g_best, g_best_name,
           prop.gcnArchName, prop.multiProcessorCount);
    return 0;
}
