// scatter_bench.hip — random 8-byte reads vs random 8-byte writes over a large
// table on MI355X (tools only): whether pushing a value to a random slot costs
// what pulling it from a random row does (the request-rate wall of the W = 64
// path).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/scatter_bench tools/scatter_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

template <int K>
__global__ __launch_bounds__(256) void gather8(const uint64_t* table, const uint32_t* idx, uint64_t n, uint64_t* out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * K;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * K; i0 < n; i0 += stride) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = i0 + k < n ? table[idx[i0 + k]] : 0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc |= v[k];
    }
    out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int K>
__global__ __launch_bounds__(256) void scatter8(uint64_t* table, const uint32_t* idx, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * K;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * K; i0 < n; i0 += stride) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (i0 + k < n) table[idx[i0 + k]] = i0 + k;
    }
}

int main() {
    const uint64_t n = 1ull << 27, rows = 1ull << 30;  // 8 GiB table of 8-byte slots
    uint64_t *table, *out;
    uint32_t* idx;
    CK(hipMalloc(&table, rows * 8));
    CK(hipMemset(table, 0, rows * 8));
    CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&out, 16384ull * 256 * 8));
    std::vector<uint32_t> h(n);
    uint64_t s = 88172645463325252ull;
    for (uint64_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = (uint32_t)(s % rows);
    }
    CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < 3; ++r) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 3;
    };
    for (int grid : {4096, 16384}) {
        const float g = timeit([&] { hipLaunchKernelGGL(gather8<8>, dim3(grid), dim3(256), 0, 0, table, idx, n, out); });
        const float w = timeit([&] { hipLaunchKernelGGL(scatter8<8>, dim3(grid), dim3(256), 0, 0, table, idx, n); });
        printf("grid %5d: random 8-byte reads %.1f G/s, random 8-byte writes %.1f G/s\n", grid, n / (g * 1e-3) / 1e9,
               n / (w * 1e-3) / 1e9);
        fflush(stdout);
    }
    return 0;
}
