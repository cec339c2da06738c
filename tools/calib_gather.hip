// Calibration of FETCH_SIZE for k_topo_refit's access pattern (MI355X_MICROARCH.md
// §HBM: "other access widths are uncalibrated: calibrate on a known byte count in
// your own access pattern").  Three kernels over a 1M-triangle soup (36 B each):
//   k_stream16   16-B-per-lane streaming read of the 36 MB (the guide's known case)
//   k_stream36   one triangle per lane through 9 dword loads, lanes consecutive
//   k_gather36   one triangle per lane through a random permutation (the leaf gather
//                of k_topo_refit: tris[svals[k]])
// Each writes one dword per lane.  The host prints the distinct 64-B and 128-B
// lines each kernel touches, so FETCH_SIZE per dispatch (rocprofv3 --pmc) can be
// read against both request sizes.
// build: hipcc --offload-arch=gfx950 -O3 tools/calib_gather.hip -o tools/build/calib_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_stream16(const float4* __restrict__ src, uint32_t n4, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 v = src[i];
    out[i] = v.x + v.y + v.z + v.w;
}

__global__ __launch_bounds__(256) void k_stream36(const float* __restrict__ tris, uint32_t n, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* s = tris + (uint64_t)i * 9;
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < 9; ++c) a += s[c];
    out[i] = a;
}

__global__ __launch_bounds__(256) void k_gather36(const float* __restrict__ tris, const uint32_t* __restrict__ perm,
                                                  uint32_t n, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* s = tris + (uint64_t)perm[i] * 9;
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < 9; ++c) a += s[c];
    out[i] = a;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<float> h(n * 9ull);
    std::mt19937 rng(1);
    for (auto& x : h) x = (float)(rng() & 0xffff) * 1e-3f;
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    // distinct lines touched by the gather (= by every pattern: all triangles)
    auto lines = [&](uint64_t L) {
        uint64_t cnt = 0;
        for (uint32_t t = 0; t < n; ++t) {
            const uint64_t a = (uint64_t)t * 36, b = a + 35;
            cnt += b / L - a / L + 1;  // lines one triangle touches
        }
        return cnt;
    };
    const uint64_t d64 = (n * 36ull + 63) / 64, d128 = (n * 36ull + 127) / 128;
    printf("n=%u: 36 MB soup = %llu distinct 64-B / %llu distinct 128-B lines; per-triangle line touches: "
           "%llu x 64 B (%.1f MB), %llu x 128 B (%.1f MB)\n",
           n, (unsigned long long)d64, (unsigned long long)d128, (unsigned long long)lines(64), lines(64) * 64e-6,
           (unsigned long long)lines(128), lines(128) * 128e-6);
    float *d_tris, *d_out;
    uint32_t* d_perm;
    const uint32_t n4 = (uint32_t)(n * 9ull / 4);
    const uint64_t nout = n4 > n ? n4 : n;  // k_stream16 writes one dword per float4
    CK(hipMalloc(&d_tris, n * 36ull));
    CK(hipMalloc(&d_out, nout * 4ull));
    CK(hipMalloc(&d_perm, n * 4ull));
    CK(hipMemcpy(d_tris, h.data(), n * 36ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_perm, perm.data(), n * 4ull, hipMemcpyHostToDevice));
    if ((uint64_t)n4 * 16 > n * 36ull || nout < n4 || nout < n) { fprintf(stderr, "sizes\n"); return 1; }
    for (uint32_t i = 0; i < n; ++i)
        if (perm[i] >= n) { fprintf(stderr, "perm\n"); return 1; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps; ++r) {
        float ms[3];
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_stream16, dim3((n4 + 255) / 256), dim3(256), 0, 0, (const float4*)d_tris, n4, d_out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[0], e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_stream36, dim3((n + 255) / 256), dim3(256), 0, 0, d_tris, n, d_out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[1], e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_gather36, dim3((n + 255) / 256), dim3(256), 0, 0, d_tris, d_perm, n, d_out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[2], e0, e1));
        printf("rep %d: stream16 %.1f us, stream36 %.1f us, gather36 %.1f us\n", r, ms[0] * 1e3, ms[1] * 1e3,
               ms[2] * 1e3);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(d_tris));
    CK(hipFree(d_out));
    CK(hipFree(d_perm));
    return 0;
}
