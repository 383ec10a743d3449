// long_link_bins.hip — propagation blocking for C5's random long links, as a
// memory-pattern experiment (tools only; DESIGN.md §7b/§8 "next"). A dense
// W = 64 round gathers, per receiver, the 8-byte F words of two random senders
// (the long links): 1.3·10^8 random rows at 2^26 nodes, at the random-row
// request ceiling. Propagation blocking replaces the random reads by two
// streaming passes over a static layout built once per topology:
//   scatter: senders in ascending order write their F word into each long-link
//            receiver's bin slot (bins = receiver blocks of 8K nodes; inside a
//            bin, slots ascend by sender, so a block walking a contiguous sender
//            chunk appends to every bin in order);
//   merge:   one workgroup per bin ORs its slots into an LDS accumulator by the
//            receiver's offset in the block, then writes the block's words.
// The senders' OR is order-independent on a symmetric graph (every sender is
// also an out-neighbour, so every new bit is claimed by a reciprocal sender).
// Prints both variants' times and checks they produce the same words.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/long_link_bins tools/long_link_bins.hip
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

constexpr int kLB = 13;  // receivers per bin: 8K (64 KB of LDS words)
constexpr uint32_t kBin = 1u << kLB;

// pull: receiver v ORs F of its two long-link senders (K receivers per lane in flight)
template <int K>
__global__ __launch_bounds__(256) void pull_far(const uint64_t* F, const uint32_t* src, uint32_t n, uint64_t* out) {
    const uint32_t stride = gridDim.x * 256 * K;
    for (uint32_t v0 = blockIdx.x * 256 * K + threadIdx.x; v0 < n; v0 += stride) {
        uint32_t s[K][2];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t v = v0 + k * 256;
            s[k][0] = v < n ? src[2ull * v] : 0u;
            s[k][1] = v < n ? src[2ull * v + 1] : 0u;
        }
        uint64_t x[K][2];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t v = v0 + k * 256;
            x[k][0] = v < n ? F[s[k][0]] : 0ull;
            x[k][1] = v < n ? F[s[k][1]] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t v = v0 + k * 256;
            if (v < n) out[v] = x[k][0] | x[k][1];
        }
    }
}

// scatter: block b walks senders [b*chunk, (b+1)*chunk) in order
template <bool NT>
__global__ __launch_bounds__(256) void bin_scatter(const uint64_t* F, const uint32_t* out_ptr, const uint32_t* pos,
                                                   uint32_t n, uint32_t chunk, uint64_t* bins) {
    const uint32_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint32_t s = lo + threadIdx.x; s < hi; s += 256) {
        const uint64_t f = F[s];
        const uint32_t p0 = out_ptr[s], p1 = out_ptr[s + 1];
        for (uint32_t j = p0; j < p1; ++j) {
            if (NT) __builtin_nontemporal_store(f, bins + pos[j]);
            else bins[pos[j]] = f;
        }
    }
}

// merge: one workgroup per bin of 8K receivers (2 slots per receiver here)
__global__ __launch_bounds__(256) void bin_merge(const uint64_t* bins, const uint16_t* loc, const uint32_t* bin_ptr,
                                                 uint64_t* out) {
    __shared__ unsigned long long acc[kBin];
    for (uint32_t t = threadIdx.x; t < kBin; t += 256) acc[t] = 0;
    __syncthreads();
    const uint32_t p0 = bin_ptr[blockIdx.x], p1 = bin_ptr[blockIdx.x + 1];
    for (uint32_t j = p0 + threadIdx.x; j < p1; j += 256) atomicOr(&acc[loc[j]], (unsigned long long)bins[j]);
    __syncthreads();
    uint64_t* o = out + (uint64_t)blockIdx.x * kBin;
    for (uint32_t t = threadIdx.x; t < kBin; t += 256) o[t] = acc[t];
}

// window pull: items (long-link slots) ordered by (XCD, sender window, receiver);
// block i runs on XCD i % 8 (round-robin dispatch) and walks that XCD's items in
// chunk order, so the XCD's blocks read F from one or two L2-sized sender windows
// at a time (random reads that hit L2), and write each slot to its bin position
// ((bin, window, receiver) order: runs of ~64 consecutive slots)
__global__ __launch_bounds__(256) void window_pull(const uint64_t* F, const uint32_t* isrc, const uint32_t* ipos,
                                                   const uint64_t* xoff, uint64_t* bins) {
    const uint32_t x = blockIdx.x % 8, k = blockIdx.x / 8, nblk = gridDim.x / 8;
    const uint64_t lo = xoff[x], n = xoff[x + 1] - lo;
    constexpr uint32_t CH = 256 * 4;
    for (uint64_t c = (uint64_t)k * CH; c < n; c += (uint64_t)nblk * CH) {
        uint32_t s[4], p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t j = c + q * 256 + threadIdx.x;
            s[q] = j < n ? isrc[lo + j] : 0u;
            p[q] = j < n ? ipos[lo + j] : 0u;
        }
        uint64_t f[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) f[q] = F[s[q]];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c + q * 256 + threadIdx.x < n) bins[p[q]] = f[q];
    }
}

static inline uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

int main(int argc, char** argv) {
    const int LV = argc > 1 ? atoi(argv[1]) : 26;  // receivers = 2^LV (2^30: C5's size; ~60 GB host, 64 GB HBM)
    const uint32_t V = 1u << LV;
    const uint64_t E = 2ull * V;  // two long-link senders per receiver (edge e = 2v + j)
    const uint32_t nbins = V / kBin;
    std::vector<uint32_t> src(E);
    for (uint64_t e = 0; e < E; ++e) src[e] = (uint32_t)(mix(e + 12345) % V);
    // sender CSR over the edges, then slots by (bin, sender) with a stable pass in sender order
    std::vector<uint32_t> out_ptr(V + 1, 0), out_edge(E), pos(E), bin_ptr(nbins + 1), cur(nbins);
    std::vector<uint16_t> loc(E);
    for (uint64_t e = 0; e < E; ++e) out_ptr[src[e] + 1]++;
    for (uint32_t s = 0; s < V; ++s) out_ptr[s + 1] += out_ptr[s];
    {
        std::vector<uint32_t> fill(out_ptr.begin(), out_ptr.end() - 1);
        for (uint64_t e = 0; e < E; ++e) out_edge[fill[src[e]]++] = (uint32_t)e;
    }
    for (uint32_t b = 0; b <= nbins; ++b) bin_ptr[b] = b * 2 * kBin;
    for (uint32_t b = 0; b < nbins; ++b) cur[b] = bin_ptr[b];
    for (uint64_t j = 0; j < E; ++j) {
        const uint32_t v = out_edge[j] / 2;
        const uint32_t p = cur[v >> kLB]++;
        pos[j] = p;
        loc[p] = (uint16_t)(v & (kBin - 1));
    }
    std::vector<uint64_t> hF(V);
    for (uint32_t v = 0; v < V; ++v) hF[v] = mix(v * 7 + 1) & mix(v * 13 + 5);  // ~1/4 of bits set
    uint64_t *F, *bins, *o1, *o2;
    uint32_t *d_src, *d_optr, *d_pos, *d_bptr;
    uint16_t* d_loc;
    CK(hipMalloc(&F, V * 8ull));
    CK(hipMalloc(&bins, E * 8));
    CK(hipMalloc(&o1, V * 8ull));
    CK(hipMalloc(&o2, V * 8ull));
    CK(hipMalloc(&d_src, E * 4));
    CK(hipMalloc(&d_optr, (V + 1) * 4ull));
    CK(hipMalloc(&d_pos, E * 4));
    CK(hipMalloc(&d_bptr, (nbins + 1) * 4ull));
    CK(hipMalloc(&d_loc, E * 2));
    CK(hipMemcpy(F, hF.data(), V * 8ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_src, src.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_optr, out_ptr.data(), (V + 1) * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pos, pos.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_bptr, bin_ptr.data(), (nbins + 1) * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_loc, loc.data(), E * 2, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipEventRecord(a, 0));
        const int reps = 10;
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("V = 2^%d receivers, %llu long-link slots, %u bins of %u receivers\n", LV, (unsigned long long)E, nbins, kBin);
    for (int grid : {cus * 8, cus * 32}) {
        const float t = timeit([&] { hipLaunchKernelGGL(pull_far<4>, dim3(grid), dim3(256), 0, 0, F, d_src, V, o1); });
        printf("pull (random 8-byte gathers), grid %5d: %.3f ms, %.1f G rows/s\n", grid, t, E / (t * 1e-3) / 1e9);
        fflush(stdout);
    }
    for (int nt = 0; nt < 2; ++nt) {
        for (uint32_t chunk : {4096u, 16384u, 65536u, 262144u}) {
            const uint32_t grid = (V + chunk - 1) / chunk;
            const float ts = timeit([&] {
                if (nt) hipLaunchKernelGGL(bin_scatter<true>, dim3(grid), dim3(256), 0, 0, F, d_optr, d_pos, V, chunk, bins);
                else hipLaunchKernelGGL(bin_scatter<false>, dim3(grid), dim3(256), 0, 0, F, d_optr, d_pos, V, chunk, bins);
            });
            const double sb = V * 8.0 + (V + 1) * 4.0 + E * 4.0 + E * 8.0;
            printf("%s scatter, sender chunk %6u (grid %5u): %.3f ms (%.0f GB/s streamed)\n", nt ? "NT" : "plain", chunk,
                   grid, ts, sb / (ts * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    hipLaunchKernelGGL(bin_scatter<false>, dim3(V / 16384), dim3(256), 0, 0, F, d_optr, d_pos, V, 16384u, bins);
    const float tm2 = timeit([&] { hipLaunchKernelGGL(bin_merge, dim3(nbins), dim3(256), 0, 0, bins, d_loc, d_bptr, o2); });
    const double mb = E * 8.0 + E * 2.0 + V * 8.0;
    printf("merge: %.3f ms (%.0f GB/s streamed)\n", tm2, mb / (tm2 * 1e-3) / 1e9);
    hipLaunchKernelGGL(pull_far<4>, dim3(cus * 8), dim3(256), 0, 0, F, d_src, V, o1);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> h1(V), h2(V);
    CK(hipMemcpy(h1.data(), o1, V * 8ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), o2, V * 8ull, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint32_t v = 0; v < V; ++v) bad += h1[v] != h2[v];
    printf("check: %llu receivers differ\n", (unsigned long long)bad);
    fflush(stdout);
    if (bad) return 1;
    // ---- window pull: sender windows of 2^LW nodes, items by (XCD, window, receiver)
    for (int LW : {16, 17, 18}) {
        if (LV > 26) break;  // the window layout's host tables grow as V^2
        const uint32_t nw = V >> LW;
        std::vector<uint64_t> cntw(nw + 1, 0), cntbw((uint64_t)nbins * nw + 1, 0);
        auto wkey = [&](uint32_t w) { return (uint64_t)(w % 8) * (nw / 8) + w / 8; };
        for (uint64_t e = 0; e < E; ++e) {
            cntw[wkey(src[e] >> LW) + 1]++;
            cntbw[(uint64_t)((e / 2) >> kLB) * nw + (src[e] >> LW) + 1]++;
        }
        for (uint32_t w = 0; w < nw; ++w) cntw[w + 1] += cntw[w];
        for (uint64_t q = 0; q < (uint64_t)nbins * nw; ++q) cntbw[q + 1] += cntbw[q];
        std::vector<uint32_t> isrc(E), ipos(E);
        std::vector<uint16_t> wloc(E);
        std::vector<uint64_t> xoff(9);
        for (int x = 0; x <= 8; ++x) xoff[x] = cntw[(uint64_t)x * (nw / 8)];
        for (uint64_t e = 0; e < E; ++e) {  // natural order = receiver order: stable
            const uint32_t v = (uint32_t)(e / 2), w = src[e] >> LW;
            const uint64_t j = cntw[wkey(w)]++;
            const uint64_t p = cntbw[(uint64_t)(v >> kLB) * nw + w]++;
            isrc[j] = src[e];
            ipos[j] = (uint32_t)p;
            wloc[p] = (uint16_t)(v & (kBin - 1));
        }
        uint32_t *d_isrc, *d_ipos;
        uint64_t* d_xoff;
        CK(hipMalloc(&d_isrc, E * 4));
        CK(hipMalloc(&d_ipos, E * 4));
        CK(hipMalloc(&d_xoff, 9 * 8));
        CK(hipMemcpy(d_isrc, isrc.data(), E * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_ipos, ipos.data(), E * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_xoff, xoff.data(), 9 * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_loc, wloc.data(), E * 2, hipMemcpyHostToDevice));
        for (int grid : {cus * 4, cus * 8, cus * 16}) {
            const float tw = timeit([&] { hipLaunchKernelGGL(window_pull, dim3(grid), dim3(256), 0, 0, F, d_isrc, d_ipos, d_xoff, bins); });
            const float tg = timeit([&] { hipLaunchKernelGGL(bin_merge, dim3(nbins), dim3(256), 0, 0, bins, d_loc, d_bptr, o2); });
            printf("window pull 2^%d senders (%u windows), grid %5d: %.3f ms + merge %.3f ms = %.3f ms\n", LW, nw, grid, tw, tg,
                   tw + tg);
            fflush(stdout);
        }
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> h3(V);
        CK(hipMemcpy(h3.data(), o2, V * 8ull, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t v = 0; v < V; ++v) bad += h1[v] != h3[v];
        printf("window 2^%d check: %llu receivers differ\n", LW, (unsigned long long)bad);
        fflush(stdout);
        if (bad) return 1;
        CK(hipFree(d_isrc));
        CK(hipFree(d_ipos));
        CK(hipFree(d_xoff));
    }
    return bad ? 1 : 0;
}
