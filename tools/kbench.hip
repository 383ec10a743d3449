// kbench.hip — isolated timing of one dense propagation round of the lean
// expand kernel (tools only; not part of the product library).
//
// Builds a 4-ary tree CSR (V nodes), random node sets and frontier rows, marks
// every node active (ACT) and candidate, and times expand_round_lean on the
// same inputs repeatedly (inputs restored before every launch). Reports time
// and effective bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gossip-glomers-distributed-systems_amd/csrc tools/kbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "expand_kernels.hpp"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t V = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    constexpr int G = 8, WPL = 2;
    const uint32_t nwp = G * WPL, NG = gg::kBlock / G;
    // tree CSR (symmetric): parent then children
    std::vector<int64_t> ptr(V + 1, 0);
    std::vector<uint32_t> col;
    for (uint64_t i = 0; i < V; ++i) {
        if (i > 0) col.push_back((uint32_t)((i - 1) / 4) | gg::kRecipBit);
        for (uint64_t c = 4 * i + 1; c <= 4 * i + 4 && c < V; ++c) col.push_back((uint32_t)c | gg::kRecipBit);
        ptr[i + 1] = (int64_t)col.size();
    }
    const uint64_t E = col.size();
    const uint64_t rows = (V + 63) / 64 * 64;
    const uint64_t ntiles = (V + NG - 1) / NG;
    std::vector<uint64_t> hb(rows * nwp), hf(rows * nwp);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (auto& w : hb) w = rnd() & rnd();
    for (auto& w : hf) w = rnd() & rnd() & rnd();
    int64_t* d_ptr;
    uint32_t *d_col, *d_act;
    uint64_t *d_base, *d_base0, *d_Fp, *d_Fc, *d_fired;
    uint8_t *d_flgp, *d_flgc, *d_cand, *d_tc, *d_zm;
    unsigned long long* d_ctr;
    CK(hipMalloc(&d_ptr, (V + 1) * 8));
    CK(hipMalloc(&d_col, E * 4));
    CK(hipMalloc(&d_base, rows * nwp * 8));
    CK(hipMalloc(&d_base0, rows * nwp * 8));
    CK(hipMalloc(&d_Fp, rows * nwp * 8));
    CK(hipMalloc(&d_Fc, rows * nwp * 8));
    CK(hipMalloc(&d_fired, rows / 8 * 4));
    CK(hipMalloc(&d_flgp, rows));
    CK(hipMalloc(&d_flgc, rows));
    CK(hipMalloc(&d_cand, rows));
    CK(hipMalloc(&d_zm, rows));
    CK(hipMemset(d_zm, 0, rows));
    CK(hipMalloc(&d_tc, ntiles + 8));
    CK(hipMalloc(&d_act, 16));
    CK(hipMalloc(&d_ctr, gg::kSlots * gg::kCounters * 8));
    CK(hipMemcpy(d_ptr, ptr.data(), (V + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_base0, hb.data(), rows * nwp * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_Fp, hf.data(), rows * nwp * 8, hipMemcpyHostToDevice));
    const uint32_t act[4] = {(uint32_t)V, (uint32_t)V, (uint32_t)V, (uint32_t)V};  // every round dense
    CK(hipMemcpy(d_act, act, 16, hipMemcpyHostToDevice));
    CK(hipMemset(d_flgp, gg::FL_ACT, rows));
    CK(hipMemset(d_fired, 0, rows / 8 * 4));

    gg::RoundArgs a{};
    a.in_ptr = d_ptr;
    a.in_col = d_col;
    a.out_ptr = d_ptr;
    a.out_col = d_col;
    a.base = d_base;
    a.F_prev = d_Fp;
    a.F_cur = d_Fc;
    a.flg_prev = d_flgp;
    a.flg_cur = d_flgc;
    a.cand = d_cand;
    a.zmark = d_zm;
    a.tile_cand = d_tc;
    a.act = d_act;
    a.fired_m1 = a.fired_m2 = a.fired_m3 = d_fired;
    a.fired_cur = d_fired + rows / 64;
    a.counters = d_ctr;
    a.n_own = V;
    a.own0 = 0;
    a.lo = 0;
    a.nwp = nwp;
    a.nw = nwp;
    a.tile_nodes = NG;
    a.symmetric = 1;
    a.n_edges = E;
    a.rows = rows;
    a.round = 5;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t w = nwp * 8;
    const double bytes = 8.0 * (V + 1) + 4.0 * E + 2.0 * V + E + E * w + 3.0 * V * w;
    printf("V=%llu E=%llu rows %llu B, algorithmic bytes/round %.1f MB\n", (unsigned long long)V,
           (unsigned long long)E, (unsigned long long)w, bytes / 1e6);
    {
        a.stream_ok = 0;  // sparse path over every tile
        float best = 1e30f, sum = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemcpyAsync(d_base, d_base0, rows * nwp * 8, hipMemcpyDeviceToDevice, 0));
            CK(hipMemsetAsync(d_tc, 1, ntiles, 0));
            CK(hipMemsetAsync(d_cand, gg::CA_NODE, rows, 0));
            CK(hipMemsetAsync(d_ctr, 0, gg::kSlots * gg::kCounters * 8, 0));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL((gg::expand_round_lean<G, WPL>), dim3(2048), dim3(gg::kBlock), 0, 0, a);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            sum += ms;
        }
        printf("round  best %.4f ms  mean %.4f ms  -> %.0f GB/s algorithmic\n", best, sum / reps,
               bytes / (best * 1e-3) / 1e9);
    }
    // streaming kernel (the dense-round path of the library for WPL == 2)
    {
        a.stream_ok = 1;
        for (int blocks : {1024}) {
            float best = 1e30f, sum = 0;
            for (int r = 0; r < reps; ++r) {
                CK(hipMemcpyAsync(d_base, d_base0, rows * nwp * 8, hipMemcpyDeviceToDevice, 0));
                CK(hipMemsetAsync(d_cand, gg::CA_NODE, rows, 0));
                CK(hipMemsetAsync(d_ctr, 0, gg::kSlots * gg::kCounters * 8, 0));
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL((gg::expand_stream<G, WPL>), dim3(blocks), dim3(gg::kBlock), 0, 0, a);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
                sum += ms;
            }
            printf("stream blocks=%d  best %.4f ms  mean %.4f ms  -> %.0f GB/s algorithmic\n", blocks,
                   best, sum / reps, bytes / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
