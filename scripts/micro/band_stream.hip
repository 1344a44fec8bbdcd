// Memory-stream probe for the multi-generation step kernels (DESIGN.md §4
// "Memory operations"): the same wave -> (strip, band) decomposition and
// row streaming as multistep_hg_kernel, with the stencil replaced by a
// dependent chain of K v_bitop3 per word, so the bytes moved are the pass's
// (band + 2*halo rows read per wave, band rows written) and only the
// compute and the knobs differ.  Knobs: lane width VEC (8- or 16-byte
// lanes), prefetch distance PF, band height, halo rows, waves per CU
// (limited through dynamic LDS), chain length K.
//
//   hipcc -O3 --offload-arch=gfx950 band_stream.hip -o band_stream
//   ./band_stream [edge]       (default 262144: two 8 GiB planes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct P {
    const uint32_t* in;
    uint32_t* out;
    int wwords, rows, strips, band, halo, nbands;
};

template <int VEC>
struct W { uint32_t w[VEC]; };

template <int VEC>
__device__ __forceinline__ void ld(const uint32_t* p, W<VEC>& d) {
    if constexpr (VEC == 4) { const uint4 v = *reinterpret_cast<const uint4*>(p); d.w[0] = v.x; d.w[1] = v.y; d.w[2] = v.z; d.w[3] = v.w; }
    else { const uint2 v = *reinterpret_cast<const uint2*>(p); d.w[0] = v.x; d.w[1] = v.y; }
}
template <int VEC>
__device__ __forceinline__ void st(uint32_t* p, const W<VEC>& d) {
    if constexpr (VEC == 4) *reinterpret_cast<uint4*>(p) = make_uint4(d.w[0], d.w[1], d.w[2], d.w[3]);
    else *reinterpret_cast<uint2*>(p) = make_uint2(d.w[0], d.w[1]);
}

// MIS 0: 64-lane strips (512 / 1024 B aligned per wave-load); 1: the step
// kernels' 62-output-lane strips with halo lanes (loads straddle cache lines,
// adjacent strips share the straddled lines); 2: as 1 with an XCD-aware
// block order (consecutive blocks on one XCD, so the shared lines meet in
// that XCD's L2).
template <int VEC, int PF, int K, int MIS>
__global__ __launch_bounds__(256) void band_k(const P p) {
    constexpr int RING = 8;
    const int lane = threadIdx.x & 63;
    int blk = blockIdx.x;
    if constexpr (MIS == 2) {  // dispatch puts block b on XCD b % 8
        const int per = gridDim.x / 8;
        if (blk < per * 8) blk = (blk % 8) * per + blk / 8;
    }
    const int wave = blk * 4 + (threadIdx.x >> 6);
    const int strip = wave % p.strips, bandi = wave / p.strips;
    if (bandi >= p.nbands) return;
    const int r0 = bandi * p.band - p.halo;
    const int n = p.band + 2 * p.halo;
    int col = MIS ? strip * 62 * VEC + (lane - 1) * VEC : strip * 64 * VEC + lane * VEC;
    if (col < 0) col += p.wwords;
    if (col >= p.wwords) col -= p.wwords;
    auto rowp = [&](int q) {
        int r = r0 + min(q, n - 1);
        r = r < 0 ? r + p.rows : (r >= p.rows ? r - p.rows : r);
        return p.in + (size_t)r * p.wwords + col;
    };
    W<VEC> ring[RING];
#pragma unroll
    for (int t = 0; t < PF; ++t) ld<VEC>(rowp(t), ring[t]);
    W<VEC> acc;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc.w[j] = 0;
    for (int q0 = 0; q0 < n; q0 += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            const int q = q0 + u;
            ld<VEC>(rowp(q + PF), ring[(u + PF) % RING]);
            W<VEC> o;
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                uint32_t x = ring[u].w[j] ^ acc.w[j];
#pragma unroll
                for (int k = 0; k < K; ++k) x = __builtin_amdgcn_bitop3_b32(x, ring[u].w[j], acc.w[j] + k, 0x96);
                acc.w[j] = x;
                o.w[j] = x;
            }
            const int r = r0 + q;
            if (q >= p.halo && q < n - p.halo && r < p.rows && (MIS == 0 || (lane >= 1 && lane <= 62))) st<VEC>(p.out + (size_t)r * p.wwords + col, o);
        }
    }
}

template <int VEC, int PF, int K, int MIS = 0>
int run(const uint32_t* in, uint32_t* out, int edge, int band, int halo, int wpc) {
    P p;
    p.in = in; p.out = out; p.wwords = edge / 32; p.rows = edge; p.band = band; p.halo = halo;
    p.strips = MIS ? (p.wwords + 62 * VEC - 1) / (62 * VEC) : p.wwords / (64 * VEC);
    p.nbands = (edge + band - 1) / band;
    const int waves = p.strips * p.nbands;
    const int blocks = (waves + 3) / 4;
    const size_t lds = 160 * 1024 / (wpc / 4);  // dynamic LDS caps workgroups per CU
    CHK(hipFuncSetAttribute((const void*)band_k<VEC, PF, K, MIS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((band_k<VEC, PF, K, MIS>), dim3(blocks), dim3(256), lds - 1024, 0, p);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((band_k<VEC, PF, K, MIS>), dim3(blocks), dim3(256), lds - 1024, 0, p);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    const double plane = (double)edge * edge / 8;
    const double rd = plane * (double)(band + 2 * halo) / band, wr = plane;
    printf("MIS=%d VEC=%d PF=%d K=%2d band=%4d halo=%d waves/CU<=%2d  ms=%.3f  read+write %.2f TB/s (plane pair %.2f TB/s)\n",
           MIS, VEC, PF, K, band, halo, wpc, best, (rd + wr) / best / 1e9, 2 * plane / best / 1e9);
    CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    return 0;
}

int main(int argc, char** argv) {
    const int edge = argc > 1 ? atoi(argv[1]) : 262144;
    const size_t bytes = (size_t)edge * edge / 8;
    uint32_t *in, *out;
    CHK(hipMalloc(&in, bytes)); CHK(hipMalloc(&out, bytes));
    CHK(hipMemset(in, 0x5A, bytes)); CHK(hipMemset(out, 0, bytes));
    int rc = 0;
    // the multi-generation pass shape: 8-byte lanes, PF 2, band 216, G = 6 halos, 20 waves/CU
    rc |= run<2, 2, 0>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 0, 1>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 0, 2>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 40, 1>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 40, 2>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 0>(in, out, edge, 216, 0, 20);
    rc |= run<2, 2, 0>(in, out, edge, 16, 0, 20);
    rc |= run<2, 2, 0>(in, out, edge, 216, 6, 32);
    rc |= run<2, 4, 0>(in, out, edge, 216, 6, 20);
    rc |= run<2, 6, 0>(in, out, edge, 216, 6, 20);
    rc |= run<4, 2, 0>(in, out, edge, 216, 6, 20);
    rc |= run<4, 4, 0>(in, out, edge, 216, 6, 20);
    rc |= run<4, 2, 0>(in, out, edge, 16, 0, 32);
    // with a dependent compute chain per word and row (2K VALU per word and row; G = 6 at ~13 per word-generation ~ K = 40)
    rc |= run<2, 2, 8>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 24>(in, out, edge, 216, 6, 20);
    rc |= run<2, 2, 40>(in, out, edge, 216, 6, 20);
    rc |= run<2, 4, 40>(in, out, edge, 216, 6, 20);
    rc |= run<4, 2, 40>(in, out, edge, 216, 6, 20);
    CHK(hipFree(in)); CHK(hipFree(out));
    return rc;
}
