// bench_stream.hip -- design experiment (not product code): read bandwidth
// of the K0 bounds pass over an AoS triangle soup, per load shape.
//   A  8 triangles per thread as 18 consecutive 16-B loads (lane stride
//      288 B: each wave-instruction touches 64 lines) -- the r02 k_bounds;
//   B  the same bytes loaded coalesced (lane l, instruction j: float4
//      j*64 + l of the wave's 18-KB span), staged through LDS, each lane then
//      reads triangles l, l+64, ... (dword stride 9: conflict-free);
//   R  a plain coalesced float4 sum over the same buffer (the ceiling).
// usage: bench_stream [n_tris]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

__device__ __forceinline__ float wmin(float v) {
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wmax(float v) {
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ void fold(const float* t, float* lo, float* hi) {
    for (int c = 0; c < 3; ++c) {
        const float mn = fminf(fminf(t[c], t[3 + c]), t[6 + c]);
        const float mx = fmaxf(fmaxf(t[c], t[3 + c]), t[6 + c]);
        const float cc = (mn + mx) * 0.5f;
        lo[c] = fminf(lo[c], cc);
        hi[c] = fmaxf(hi[c], cc);
    }
}

__device__ __forceinline__ void finish(float* lo, float* hi, float* out) {
    for (int c = 0; c < 3; ++c) { lo[c] = wmin(lo[c]); hi[c] = wmax(hi[c]); }
    const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) < 3) {
        const int c = threadIdx.x & 63;
        out[wave * 6 + c] = lo[c];
        out[wave * 6 + 3 + c] = hi[c];
    }
}

// A: 18 x 16-B loads per thread, lane stride 288 B (full groups only: n % 2048 == 0)
__global__ __launch_bounds__(256) void kA(const float* __restrict__ tris, unsigned n, float* out) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    const unsigned g = blockIdx.x * 256u + threadIdx.x;
    if (g * 8 < n) {
        const float4* p = reinterpret_cast<const float4*>(tris + (size_t)g * 72);
        float4 v[18];
#pragma unroll
        for (int j = 0; j < 18; ++j) v[j] = p[j];
        float t[72];
#pragma unroll
        for (int j = 0; j < 18; ++j) { t[4 * j] = v[j].x; t[4 * j + 1] = v[j].y; t[4 * j + 2] = v[j].z; t[4 * j + 3] = v[j].w; }
#pragma unroll
        for (int q = 0; q < 8; ++q) fold(t + 9 * q, lo, hi);
    }
    finish(lo, hi, out);
}

// B: coalesced loads of the wave's 512 triangles, LDS transpose
__global__ __launch_bounds__(256) void kB(const float* __restrict__ tris, unsigned n, float* out) {
    __shared__ float4 s[4][1152];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    const unsigned w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * 4u + w;
    if (wave * 512u < n) {
        const float4* p = reinterpret_cast<const float4*>(tris + (size_t)wave * 512 * 9);
        float4 v[18];
#pragma unroll
        for (int j = 0; j < 18; ++j) v[j] = p[j * 64 + l];
#pragma unroll
        for (int j = 0; j < 18; ++j) s[w][j * 64 + l] = v[j];
        __builtin_amdgcn_wave_barrier();
        const float* f = reinterpret_cast<const float*>(s[w]);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            float t[9];
#pragma unroll
            for (int c = 0; c < 9; ++c) t[c] = f[(q * 64 + l) * 9 + c];
            fold(t, lo, hi);
        }
    }
    finish(lo, hi, out);
}


// C: lane l of a wave takes triangles base + 64q + l, each as three 12-B
// (dwordx3) vertex loads: lane stride 36 B, every instruction spans 2304
// contiguous bytes (18 lines, a third of each), no LDS
struct F3 { float x, y, z; };
__global__ __launch_bounds__(256) void kC(const float* __restrict__ tris, unsigned n, float* out) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    const unsigned w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const unsigned base = (blockIdx.x * 4u + w) * 512u;
    const F3* p = reinterpret_cast<const F3*>(tris);
    F3 v[8][3];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const unsigned k = base + q * 64 + l;
#pragma unroll
        for (int j = 0; j < 3; ++j) v[q][j] = k < n ? p[(size_t)k * 3 + j] : F3{0, 0, 0};
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float t[9] = {v[q][0].x, v[q][0].y, v[q][0].z, v[q][1].x, v[q][1].y, v[q][1].z, v[q][2].x, v[q][2].y, v[q][2].z};
        if (base + q * 64 + l < n) fold(t, lo, hi);
    }
    finish(lo, hi, out);
}

// R: coalesced float4 read, summed
__global__ __launch_bounds__(256) void kR(const float4* __restrict__ p, size_t m, float* out) {
    float a = 0.0f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += (size_t)gridDim.x * 256)
        a += p[i].x + p[i].y + p[i].z + p[i].w;
    if (a == 12345.0f) out[7] = a;
}

int main(int argc, char** argv) {
    const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 10000384u;  // multiple of 2048
    const size_t bytes = (size_t)n * 36;
    std::vector<float> h((size_t)n * 9);
    unsigned long long s = 1;
    for (auto& x : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; x = (float)(s >> 40) * 0x1p-24f; }
    float *d, *o;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, (size_t)(n / 512 + 64) * 6 * 4));
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int R = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < R; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f us  %6.2f TB/s\n", name, 1e3 * ms / R, bytes / (1e-3 * ms / R) / 1e12);
    };
    const unsigned gA = (n / 8 + 255) / 256, gB = (n / 512 + 3) / 4;
    run("A strided 18x16B per thread", [&] { hipLaunchKernelGGL(kA, dim3(gA), dim3(256), 0, 0, d, n, o); });
    run("B coalesced + LDS transpose", [&] { hipLaunchKernelGGL(kB, dim3(gB), dim3(256), 0, 0, d, n, o); });
    run("C dwordx3 vertices, lane stride 36 B", [&] { hipLaunchKernelGGL(kC, dim3(gB), dim3(256), 0, 0, d, n, o); });
    run("R coalesced float4 read (grid 4096)", [&] { hipLaunchKernelGGL(kR, dim3(4096), dim3(256), 0, 0, (const float4*)d, bytes / 16, o); });
    run("R coalesced float4 read (grid n/1024)", [&] {
        hipLaunchKernelGGL(kR, dim3((unsigned)(bytes / 16 / 256 / 4)), dim3(256), 0, 0, (const float4*)d, bytes / 16, o);
    });
    CK(hipGetLastError());
    return 0;
}
