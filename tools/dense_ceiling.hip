// dense_ceiling.hip — the memory traffic of one dense C2 round, without the
// round's logic (tools only): every node of the 2^20-node 4-ary tree reads
// its row pointers and in-list, its own 128-byte set row and the F rows of
// its senders, and writes its F row and its set row — the loads and stores
// expand_stream issues in a dense round, none of the claim chain, hashing,
// flags or counters. What this moves per round, and how fast, is the
// access-pattern ceiling the kernel's dense rounds are measured against
// (DESIGN.md §7c).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/dense_ceiling tools/dense_ceiling.hip
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

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// G = 8 lanes per node (16 bytes each), NT: non-temporal row stores, D senders
// in flight (the tree has at most 5).
template <bool NT>
__global__ __launch_bounds__(256) void dense_round(const int64_t* in_ptr, const uint32_t* in_col, const u64x2* F_prev,
                                                   u64x2* F_cur, u64x2* base, uint32_t n, uint32_t sel) {
    constexpr int G = 8, D = 5;
    const uint32_t lg = threadIdx.x % G;
    const uint32_t groups = gridDim.x * (256 / G);
    for (uint32_t v = blockIdx.x * (256 / G) + threadIdx.x / G; v < n; v += groups) {
        const int64_t p0 = in_ptr[v], p1 = in_ptr[v + 1];
        uint32_t c[D];
#pragma unroll
        for (int b = 0; b < D; ++b) c[b] = p0 + b < p1 ? in_col[p0 + b] : 0u;
        const u64x2 own = base[(uint64_t)v * G + lg];
        u64x2 x[D];
#pragma unroll
        for (int b = 0; b < D; ++b) x[b] = p0 + b < p1 ? F_prev[(uint64_t)c[b] * G + lg] : (u64x2){0, 0};
        u64x2 S = own;
#pragma unroll
        for (int b = 0; b < D; ++b) S |= x[b];
        const u64x2 F = S & ~own;
        // sel != 0 keeps the stores data-dependent without changing the traffic
        const u64x2 Fw = sel ? F : S;
        if (NT) {
            __builtin_nontemporal_store(Fw, F_cur + (uint64_t)v * G + lg);
            __builtin_nontemporal_store(S, base + (uint64_t)v * G + lg);
        } else {
            F_cur[(uint64_t)v * G + lg] = Fw;
            base[(uint64_t)v * G + lg] = S;
        }
    }
}

int main() {
    const uint32_t V = 1u << 20;
    // tree4 in-lists, senders ascending: parent (v-1)/4 and children 4v+1..4v+4
    std::vector<int64_t> rp(V + 1, 0);
    std::vector<uint32_t> col;
    for (uint32_t v = 0; v < V; ++v) {
        rp[v] = (int64_t)col.size();
        if (v) col.push_back((v - 1) / 4);
        for (uint32_t k = 1; k <= 4; ++k)
            if (4ull * v + k < V) col.push_back(4 * v + k);
    }
    rp[V] = (int64_t)col.size();
    const uint64_t E = col.size(), rowb = 128;
    int64_t* d_rp;
    uint32_t* d_col;
    u64x2 *F0, *F1, *B;
    CK(hipMalloc(&d_rp, (V + 1) * 8));
    CK(hipMalloc(&d_col, E * 4));
    CK(hipMalloc(&F0, V * rowb));
    CK(hipMalloc(&F1, V * rowb));
    CK(hipMalloc(&B, V * rowb));
    CK(hipMemcpy(d_rp, rp.data(), (V + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemset(F0, 0x11, V * rowb));
    CK(hipMemset(F1, 0x22, V * rowb));
    CK(hipMemset(B, 0x44, V * rowb));
    const double bytes = 8.0 * (V + 1) + 4.0 * E + rowb * (double)E + 3.0 * rowb * V;  // SURVEY §8d dense round
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int nt = 0; nt < 2; ++nt) {
        for (int grid : {cus * 8, cus * 16, cus * 32, cus * 64, (int)(V / 32)}) {
            auto launch = [&](int r) {
                const u64x2* Fp = (r & 1) ? F1 : F0;
                u64x2* Fc = (r & 1) ? F0 : F1;
                if (nt) hipLaunchKernelGGL(dense_round<true>, dim3(grid), dim3(256), 0, 0, d_rp, d_col, Fp, Fc, B, V, 1u);
                else hipLaunchKernelGGL(dense_round<false>, dim3(grid), dim3(256), 0, 0, d_rp, d_col, Fp, Fc, B, V, 1u);
            };
            for (int r = 0; r < 3; ++r) launch(r);
            CK(hipEventRecord(a, 0));
            const int reps = 20;
            for (int r = 0; r < reps; ++r) launch(r);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1e3 / reps;
            printf("%s stores, grid %6d: %.1f us per dense round, %.0f GB/s algorithmic (%.0f MB)\n",
                   nt ? "non-temporal" : "plain", grid, us, bytes / (us * 1e-6) / 1e9, bytes / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
