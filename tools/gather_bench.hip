// gather_bench.hip — random whole-row gathers from a large table on MI355X
// (tools only; --calibrate also times random-row and coalesced stores, the
// write side of bench.py's line_frac): rows/s and GB/s for row sizes 32..512 B, uniformly random or
// power-law (row index = the top bits of a product of uniforms, hubs first),
// into registers (G lanes x 16 B per row, K rows in flight per lane) — the
// access shape of expand_stream's sender-row gathers at 8..64 lanes per node.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gather_bench tools/gather_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

// T tags the instantiation of a calibration regime (0: an 8 GiB table in HBM; 1: a
// 256 MiB table the 256 MB Infinity Cache can hold, the regime of C2's state
// arrays) so rocprofv3 tells their dispatches apart
template <int G, int K, int T = 0>
__global__ __launch_bounds__(256) void gather(const uint4* table, const uint32_t* idx, uint64_t n_rows_idx,
                                              uint4* out) {
    const int lg = threadIdx.x % G;
    const uint64_t groups = (uint64_t)gridDim.x * (256 / G);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint64_t r0 = ((uint64_t)blockIdx.x * (256 / G) + threadIdx.x / G) * K; r0 < n_rows_idx; r0 += groups * K) {
        uint32_t ix[K];
#pragma unroll
        for (int k = 0; k < K; ++k) ix[k] = r0 + k < n_rows_idx ? idx[r0 + k] : 0u;
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = table[(uint64_t)ix[k] * G + lg];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc.x |= v[k].x;
            acc.y |= v[k].y;
            acc.z |= v[k].z;
            acc.w |= v[k].w;
        }
    }
    out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// the write side of the calibration: K random rows per lane group stored (G
// lanes x 16 B each), and a coalesced sweep (reset_state's pattern)
template <int G, int K, int T = 0>
__global__ __launch_bounds__(256) void scatter(uint4* table, const uint32_t* idx, uint64_t n_rows_idx) {
    const int lg = threadIdx.x % G;
    const uint64_t groups = (uint64_t)gridDim.x * (256 / G);
    for (uint64_t r0 = ((uint64_t)blockIdx.x * (256 / G) + threadIdx.x / G) * K; r0 < n_rows_idx; r0 += groups * K) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (r0 + k < n_rows_idx) {
                const uint32_t ix = idx[r0 + k];
                table[(uint64_t)ix * G + lg] = make_uint4(ix, (uint32_t)lg, (uint32_t)k, 1u);
            }
    }
}

template <int T = 0>
__global__ __launch_bounds__(256) void seqwrite(uint4* table, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        table[i] = make_uint4((uint32_t)i, 0u, 0u, 1u);
}

template <int G, int K, int T = 0>
double run_scatter(uint4* table, const uint32_t* idx, uint64_t n, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((scatter<G, K, T>), dim3(blocks), dim3(256), 0, 0, table, idx, n);
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((scatter<G, K, T>), dim3(blocks), dim3(256), 0, 0, table, idx, n);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
}

template <int G, int K, int T = 0>
double run(const uint4* table, const uint32_t* idx, uint64_t n, uint4* out, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((gather<G, K, T>), dim3(blocks), dim3(256), 0, 0, table, idx, n, out);
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((gather<G, K, T>), dim3(blocks), dim3(256), 0, 0, table, idx, n, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
}

int main(int argc, char** argv) {
    const uint64_t n = 1ull << 27;
    uint4* table;
    uint32_t* idx;
    uint4* out;
    const uint64_t max_table = 8ull << 30;
    CK(hipMalloc(&table, max_table));
    CK(hipMemset(table, 1, max_table));
    CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&out, 8192ull * 256 * 16));
    std::vector<uint32_t> h(n);
    if (argc > 1 && std::string(argv[1]) == "--calibrate") {
        // the request ceiling for bench.py's line_frac: uniformly random rows of an
        // 8 GiB table (HBM), 64 / 128 / 512 B, K = 8; run under rocprofv3 --pmc
        // TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum for the requests a row costs
        // (tools/request_ceiling.py multiplies them with the rows/s printed here)
        const uint64_t tb = 8ull << 30;
        for (int rb : {64, 128, 512}) {
            const uint64_t rows = tb / rb;
            uint64_t s = 88172645463325252ull + rb;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)(rnd() % rows);
            CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
            const double ms = rb == 64 ? run<4, 8>(table, idx, n, out, 4096)
                              : rb == 128 ? run<8, 8>(table, idx, n, out, 4096) : run<32, 8>(table, idx, n, out, 4096);
            printf("calibrate rows %3d B G=%2d rows_per_dispatch %llu rows_per_s %.4e\n", rb, rb / 16,
                   (unsigned long long)n, n / (ms * 1e-3));
            fflush(stdout);
        }
        // writes: random rows of 16 / 64 / 128 B (scatter<G, 8>), then a coalesced
        // sweep of 2 GiB (seqwrite); the write-request ceiling is the highest rate
        for (int rb : {16, 64, 128}) {
            const uint64_t rows = tb / rb;
            uint64_t s = 0x9E3779B97F4A7C15ull + rb;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)(rnd() % rows);
            CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
            const double ms = rb == 16 ? run_scatter<1, 8>(table, idx, n, 4096)
                              : rb == 64 ? run_scatter<4, 8>(table, idx, n, 4096) : run_scatter<8, 8>(table, idx, n, 4096);
            printf("calibrate writes %3d B G=%2d rows_per_dispatch %llu rows_per_s %.4e\n", rb, rb / 16,
                   (unsigned long long)n, n / (ms * 1e-3));
            fflush(stdout);
        }
        {
            const uint64_t n16 = (2ull << 30) / 16;
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            hipLaunchKernelGGL(seqwrite<0>, dim3(8192), dim3(256), 0, 0, table, n16);
            CK(hipEventRecord(a, 0));
            for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(seqwrite<0>, dim3(8192), dim3(256), 0, 0, table, n16);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("calibrate seqwrite bytes_per_dispatch %llu bytes_per_s %.4e\n", (unsigned long long)(n16 * 16),
                   n16 * 16 / (ms / 3 * 1e-3));
            fflush(stdout);
        }
        // the same shapes on a 256 MiB table (regime T = 1: the Infinity Cache can hold it)
        const uint64_t tm = 256ull << 20;
        for (int rb : {64, 128}) {
            const uint64_t rows = tm / rb;
            uint64_t s = 0x2545F4914F6CDD1Dull + rb;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)(rnd() % rows);
            CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
            const double ms = rb == 64 ? run<4, 8, 1>(table, idx, n, out, 4096) : run<8, 8, 1>(table, idx, n, out, 4096);
            printf("calibrate rows_mall %3d B G=%2d rows_per_dispatch %llu rows_per_s %.4e\n", rb, rb / 16,
                   (unsigned long long)n, n / (ms * 1e-3));
            fflush(stdout);
        }
        for (int rb : {16, 64, 128}) {
            const uint64_t rows = tm / rb;
            uint64_t s = 0x5851F42D4C957F2Dull + rb;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)(rnd() % rows);
            CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
            const double ms = rb == 16 ? run_scatter<1, 8, 1>(table, idx, n, 4096)
                              : rb == 64 ? run_scatter<4, 8, 1>(table, idx, n, 4096)
                                         : run_scatter<8, 8, 1>(table, idx, n, 4096);
            printf("calibrate writes_mall %3d B G=%2d rows_per_dispatch %llu rows_per_s %.4e\n", rb, rb / 16,
                   (unsigned long long)n, n / (ms * 1e-3));
            fflush(stdout);
        }
        {
            const uint64_t n16 = tm / 16;
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            hipLaunchKernelGGL(seqwrite<1>, dim3(8192), dim3(256), 0, 0, table, n16);
            CK(hipEventRecord(a, 0));
            for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(seqwrite<1>, dim3(8192), dim3(256), 0, 0, table, n16);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("calibrate seqwrite_mall bytes_per_dispatch %llu bytes_per_s %.4e\n", (unsigned long long)(n16 * 16),
                   n16 * 16 / (ms / 10 * 1e-3));
            fflush(stdout);
        }
        return 0;
    }
    // where does the row-request ceiling sit? table in L2 (2 MB), in the
    // Infinity Cache (64 MB) or in HBM (8 GB); rows in flight per lane K
    for (uint64_t tb : {2ull << 20, 64ull << 20, 8ull << 30}) {
        for (int rb : {64, 128}) {
            const uint64_t rows = tb / rb;
            uint64_t s = 88172645463325252ull + rb;
            auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
            for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)(rnd() % rows);
            CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
            for (int K : {2, 8, 16}) {
                double ms = 0;
                if (rb == 64) ms = K == 2 ? run<4, 2>(table, idx, n, out, 4096) : K == 8 ? run<4, 8>(table, idx, n, out, 4096) : run<4, 16>(table, idx, n, out, 4096);
                else ms = K == 2 ? run<8, 2>(table, idx, n, out, 4096) : K == 8 ? run<8, 8>(table, idx, n, out, 4096) : run<8, 16>(table, idx, n, out, 4096);
                printf("table %6llu MB rows %3d B K=%2d: %.1f G rows/s  %.0f GB/s\n", (unsigned long long)(tb >> 20), rb, K,
                       n / (ms * 1e-3) / 1e9, n * (double)rb / (ms * 1e-3) / 1e9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
