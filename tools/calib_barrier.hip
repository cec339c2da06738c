// Cost of a grid-wide barrier between co-resident blocks on MI355X (design
// experiment for fusing the build's first stages; never shipped).  245 blocks x
// 512 threads (the 1M build's sort tiles), each publishes a 24-B partial box:
//   k_plain  no barrier (reads whatever partials are there: timing baseline)
//   k_bar    partials written with agent-scope relaxed atomic stores (write-through,
//            no L2 writeback), a workgroup release (s_waitcnt), one agent-scope
//            atomicAdd per block, lane 0 spins on the counter, then every block
//            reads all partials with agent-scope atomic loads
//   k_bar3   three such barriers back to back
//   k_fence  the same barrier with __threadfence() (L2 writeback) instead
// Every spin gives up after ~20 ms (s_memrealtime) and flags it, so a
// non-resident grid cannot hang the GPU.
// build: hipcc --offload-arch=gfx950 -O3 tools/calib_barrier.hip -o tools/build/calib_barrier
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NT = 512;

__device__ __forceinline__ void publish(float* part, uint32_t b, const float (&v)[6]) {
    for (int c = 0; c < 6; ++c) __hip_atomic_store(part + b * 6 + c, v[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// returns false on timeout
template <bool FENCE>
__device__ __forceinline__ bool grid_barrier(uint32_t* ctr, uint32_t target, uint32_t* err) {
    __shared__ uint32_t s_ok;
    if (FENCE) __threadfence();
    else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t ok = 1;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) { ok = 0; atomicAdd(err, 1u); break; }
        }
        s_ok = ok;
    }
    __syncthreads();
    if (FENCE) __threadfence();
    return s_ok != 0;
}

template <int NBAR, int MODE>  // MODE 0 plain, 1 scoped atomics, 2 threadfence
__global__ __launch_bounds__(NT) void k_test(float* part, uint32_t* ctr, uint32_t epoch, uint32_t* err, float* out) {
    const uint32_t b = blockIdx.x, nb = gridDim.x;
    float v[6];
    for (int c = 0; c < 6; ++c) v[c] = (float)(b * 6 + c + epoch);
    float acc = 0.f;
    for (int k = 0; k < NBAR; ++k) {
        if (threadIdx.x == 0) {
            if (MODE == 0) for (int c = 0; c < 6; ++c) part[b * 6 + c] = v[c] + k;
            else publish(part, b, v);
        }
        if (MODE != 0) {
            const uint32_t target = (epoch * NBAR + k + 1) * nb;
            if (!grid_barrier<MODE == 2>(ctr, target, err)) return;
        } else {
            __syncthreads();
        }
        // every block reads all partials
        for (uint32_t j = threadIdx.x; j < nb * 6; j += NT)
            acc += MODE == 0 ? part[j] : __hip_atomic_load(part + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    out[b * NT + threadIdx.x] = acc;
}

template <int NBAR, int MODE>
static int run(const char* name, uint32_t nb, float* part, uint32_t* ctr, uint32_t* err, float* out) {
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    CK(hipMemset(ctr, 0, 4));
    const int reps = 50;
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < reps + 5; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((k_test<NBAR, MODE>), dim3(nb), dim3(NT), 0, 0, part, ctr, (uint32_t)r, err, out);
        CK(hipEventRecord(z, 0));
        CK(hipEventSynchronize(z));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, z));
        if (r >= 5) { sum += ms; best = ms < best ? ms : best; }
    }
    uint32_t e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("%-8s blocks %u: mean %.2f us, min %.2f us, timeouts %u\n", name, nb, sum / reps * 1e3f, best * 1e3f, e);
    return 0;
}

int main() {
    const uint32_t nb = 245;
    float *part, *out;
    uint32_t *ctr, *err;
    CK(hipMalloc(&part, 4096 * 6 * 4));
    CK(hipMalloc(&out, 4096 * NT * 4));
    CK(hipMalloc(&ctr, 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_test<1, 1>), NT, 0));
    printf("resident blocks per CU: %d\n", per_cu);
    for (int i = 0; i < 2; ++i) {
        if (run<1, 0>("plain", nb, part, ctr, err, out)) return 1;
        if (run<1, 1>("bar", nb, part, ctr, err, out)) return 1;
        if (run<3, 1>("bar3", nb, part, ctr, err, out)) return 1;
        if (run<1, 2>("fence", nb, part, ctr, err, out)) return 1;
        if (run<3, 2>("fence3", nb, part, ctr, err, out)) return 1;
    }
    return 0;
}
