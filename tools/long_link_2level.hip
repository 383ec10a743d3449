// long_link_2level.hip — C5's long links as a memory pattern, two-level
// propagation blocking with LDS-staged runs (tools only).
// A dense W = 64 round gathers, per receiver, the 8-byte F words of its random
// long-link senders: at 2^30 receivers the pull runs at the random-row ceiling
// (≈39 G rows/s, 55 ms for 2^31 rows, long_link_bins.hip), and a one-level
// scatter into 2^17 bins is as random as the pull. Here every pass streams:
//   A  sender chunks in order: each block reads its senders' F words once, sorts
//      its (receiver, word) pairs by coarse bin (receiver >> (LV-8): 256 bins) in
//      LDS and appends each bin's run at a cursor (one atomic per block and bin);
//   B  per coarse bin, chunks of its entries: the same LDS sort by fine bin
//      (8K receivers), runs appended at fine-bin cursors (16-bit offsets kept);
//   C  per fine bin: OR into an LDS accumulator by offset, write the 8K words.
// The OR is order-free on a symmetric graph (every sender is reciprocal), so the
// runs' order inside a bin does not matter. Prints each pass's time, the total
// against the pull, and checks the words are equal.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/long_link_2level tools/long_link_2level.hip
//   tools/long_link_2level [LV]        (receivers = 2^LV, default 26)
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

constexpr int kFB = 13;                // receivers per fine bin: 8K (64 KB of LDS words)
constexpr uint32_t kNC = 256;          // coarse bins
constexpr uint32_t kCA = 2048;         // senders per block of pass A
constexpr uint32_t kCapA = 6144;       // LDS entries of pass A (2 long links per sender, with slack)
constexpr uint32_t kCB = 4096;         // entries per block of pass B
constexpr uint32_t kNFmax = 1024;      // fine bins per coarse bin at most (LV <= 31)

static inline uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

__global__ __launch_bounds__(256) void pull_far(const uint64_t* F, const uint32_t* src, uint32_t n, uint64_t* out) {
    constexpr int K = 4;
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

// pass A: block b = senders [b*kCA, (b+1)*kCA); out_ptr/out_rcv: sender CSR of the long links
__global__ __launch_bounds__(256) void pass_a(const uint64_t* F, const uint32_t* out_ptr, const uint32_t* out_rcv,
                                              uint32_t V, int cshift, unsigned long long* curA, uint32_t* A_rcv,
                                              uint64_t* A_f) {
    __shared__ uint32_t hist[kNC], start[kNC], fill[kNC];
    __shared__ unsigned long long gpos[kNC];
    __shared__ uint32_t l_rcv[kCapA];
    __shared__ unsigned long long l_f[kCapA];
    const uint32_t s0 = blockIdx.x * kCA, s1 = min(V, s0 + kCA);
    const uint32_t e0 = out_ptr[s0], n = out_ptr[s1] - e0;
    for (uint32_t t = threadIdx.x; t < kNC; t += 256) hist[t] = fill[t] = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < n; k += 256) atomicAdd(&hist[out_rcv[e0 + k] >> cshift], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 256 counts (4 per lane) + the bins' global runs
        uint32_t c[4], s = 0;
        for (int q = 0; q < 4; ++q) { c[q] = hist[threadIdx.x * 4 + q]; s += c[q]; }
        uint32_t incl = s;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if ((int)threadIdx.x >= o) incl += y;
        }
        uint32_t base = incl - s;
        for (int q = 0; q < 4; ++q) {
            const uint32_t j = threadIdx.x * 4 + q;
            start[j] = base;
            gpos[j] = c[q] ? atomicAdd(&curA[j], (unsigned long long)c[q]) : 0ull;
            base += c[q];
        }
    }
    __syncthreads();
    // senders in order: thread per sender reads its F word once
    for (uint32_t s = s0 + threadIdx.x; s < s1; s += 256) {
        const uint64_t f = F[s];
        for (uint32_t e = out_ptr[s]; e < out_ptr[s + 1]; ++e) {
            const uint32_t r = out_rcv[e], j = r >> cshift;
            const uint32_t k = start[j] + atomicAdd(&fill[j], 1u);
            l_rcv[k] = r;
            l_f[k] = f;
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < n; k += 256) {
        const uint32_t r = l_rcv[k], j = r >> cshift;
        const unsigned long long p = gpos[j] + (k - start[j]);
        A_rcv[p] = r;
        A_f[p] = l_f[k];
    }
}

struct ChunkB {
    unsigned long long e0;
    uint32_t n, bin;
};

// pass B: chunk of coarse bin `bin`: sort by fine bin, append runs at the fine cursors
__global__ __launch_bounds__(256) void pass_b(const ChunkB* chunks, const uint32_t* A_rcv, const uint64_t* A_f,
                                              uint32_t nf, unsigned long long* curB, uint16_t* B_lo, uint64_t* B_f) {
    __shared__ uint32_t hist[kNFmax], start[kNFmax], fill[kNFmax];
    __shared__ unsigned long long gpos[kNFmax];
    __shared__ uint32_t l_rcv[kCB];
    const ChunkB c = chunks[blockIdx.x];
    for (uint32_t t = threadIdx.x; t < nf; t += 256) hist[t] = fill[t] = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < c.n; k += 256) {
        const uint32_t r = A_rcv[c.e0 + k];
        l_rcv[k] = r;
        atomicAdd(&hist[(r >> kFB) & (nf - 1)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // (nf <= 1024 counts: one thread)
        uint32_t base = 0;
        for (uint32_t j = 0; j < nf; ++j) {
            start[j] = base;
            base += hist[j];
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nf; j += 256)
        gpos[j] = hist[j] ? atomicAdd(&curB[(unsigned long long)c.bin * nf + j], (unsigned long long)hist[j]) : 0ull;
    __syncthreads();
    __shared__ uint32_t l_ord[kCB];  // sorted position of entry k
    for (uint32_t k = threadIdx.x; k < c.n; k += 256) {
        const uint32_t j = (l_rcv[k] >> kFB) & (nf - 1);
        l_ord[start[j] + atomicAdd(&fill[j], 1u)] = k;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < c.n; k += 256) {
        const uint32_t src = l_ord[k];
        const uint32_t r = l_rcv[src], j = (r >> kFB) & (nf - 1);
        const unsigned long long p = gpos[j] + (k - start[j]);
        B_lo[p] = (uint16_t)(r & ((1u << kFB) - 1));
        B_f[p] = A_f[c.e0 + src];
    }
}

// pass C: fine bin b -> the OR of its entries per receiver
__global__ __launch_bounds__(256) void pass_c(const unsigned long long* bin_ptr, const uint16_t* B_lo,
                                              const uint64_t* B_f, uint64_t* out) {
    __shared__ unsigned long long acc[1u << kFB];
    for (uint32_t t = threadIdx.x; t < (1u << kFB); t += 256) acc[t] = 0;
    __syncthreads();
    const unsigned long long p0 = bin_ptr[blockIdx.x], p1 = bin_ptr[blockIdx.x + 1];
    for (unsigned long long j = p0 + threadIdx.x; j < p1; j += 256) atomicOr(&acc[B_lo[j]], (unsigned long long)B_f[j]);
    __syncthreads();
    uint64_t* o = out + ((unsigned long long)blockIdx.x << kFB);
    for (uint32_t t = threadIdx.x; t < (1u << kFB); t += 256) o[t] = acc[t];
}

int main(int argc, char** argv) {
    const int LV = argc > 1 ? atoi(argv[1]) : 26;
    const uint32_t V = 1u << LV;
    const uint64_t E = 2ull * V;
    const int cshift = LV - 8;                      // coarse bin = receiver >> cshift
    const uint32_t nf = 1u << (cshift - kFB);       // fine bins per coarse bin
    const uint32_t nbins = V >> kFB;                // fine bins in all
    if (nf > kNFmax || LV < 22) {
        fprintf(stderr, "LV out of range\n");
        return 1;
    }
    std::vector<uint32_t> src(E);
    for (uint64_t e = 0; e < E; ++e) src[e] = (uint32_t)(mix(e + 12345) % V);
    // sender CSR of the links (edge e: sender src[e] -> receiver e/2)
    std::vector<uint32_t> out_ptr(V + 1, 0), out_rcv(E);
    for (uint64_t e = 0; e < E; ++e) out_ptr[src[e] + 1]++;
    for (uint32_t s = 0; s < V; ++s) out_ptr[s + 1] += out_ptr[s];
    {
        std::vector<uint32_t> fill(out_ptr.begin(), out_ptr.end() - 1);
        for (uint64_t e = 0; e < E; ++e) out_rcv[fill[src[e]]++] = (uint32_t)(e / 2);
    }
    uint32_t maxA = 0;
    for (uint32_t b = 0; b < V / kCA; ++b) maxA = std::max(maxA, out_ptr[(b + 1) * kCA] - out_ptr[b * kCA]);
    if (maxA > kCapA) {
        fprintf(stderr, "a sender chunk has %u links > %u\n", maxA, kCapA);
        return 1;
    }
    // bin totals -> cursors' bases; pass-B chunks
    std::vector<unsigned long long> cnt_c(kNC + 1, 0), cnt_f((uint64_t)nbins + 1, 0);
    for (uint64_t e = 0; e < E; ++e) {
        const uint32_t v = (uint32_t)(e / 2);
        cnt_c[(v >> cshift) + 1]++;
        cnt_f[(v >> kFB) + 1]++;
    }
    for (uint32_t j = 0; j < kNC; ++j) cnt_c[j + 1] += cnt_c[j];
    for (uint32_t j = 0; j < nbins; ++j) cnt_f[j + 1] += cnt_f[j];
    std::vector<ChunkB> chunks;
    for (uint32_t j = 0; j < kNC; ++j)
        for (unsigned long long p = cnt_c[j]; p < cnt_c[j + 1]; p += kCB)
            chunks.push_back({p, (uint32_t)std::min<unsigned long long>(kCB, cnt_c[j + 1] - p), j});
    std::vector<uint64_t> hF(V);
    for (uint32_t v = 0; v < V; ++v) hF[v] = mix(v * 7 + 1) & mix(v * 13 + 5);
    uint64_t *F, *A_f, *B_f, *o1, *o2;
    uint32_t *d_src, *d_optr, *d_orcv, *A_rcv;
    uint16_t* B_lo;
    unsigned long long *curA, *curB, *baseA, *baseB, *binptr;
    ChunkB* d_chunks;
    CK(hipMalloc(&F, V * 8ull));
    CK(hipMalloc(&o1, V * 8ull));
    CK(hipMalloc(&o2, V * 8ull));
    CK(hipMalloc(&d_src, E * 4));
    CK(hipMalloc(&d_optr, (V + 1) * 4ull));
    CK(hipMalloc(&d_orcv, E * 4));
    CK(hipMalloc(&A_rcv, E * 4));
    CK(hipMalloc(&A_f, E * 8));
    CK(hipMalloc(&B_lo, E * 2));
    CK(hipMalloc(&B_f, E * 8));
    CK(hipMalloc(&curA, kNC * 8));
    CK(hipMalloc(&baseA, kNC * 8));
    CK(hipMalloc(&curB, (uint64_t)nbins * 8));
    CK(hipMalloc(&baseB, (uint64_t)nbins * 8));
    CK(hipMalloc(&binptr, ((uint64_t)nbins + 1) * 8));
    CK(hipMalloc(&d_chunks, chunks.size() * sizeof(ChunkB)));
    CK(hipMemcpy(F, hF.data(), V * 8ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_src, src.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_optr, out_ptr.data(), (V + 1) * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_orcv, out_rcv.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(baseA, cnt_c.data(), kNC * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(baseB, cnt_f.data(), (uint64_t)nbins * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(binptr, cnt_f.data(), ((uint64_t)nbins + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_chunks, chunks.data(), chunks.size() * sizeof(ChunkB), hipMemcpyHostToDevice));
    hipEvent_t ev[5];
    for (auto& x : ev) CK(hipEventCreate(&x));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 5;
    float tp = 0, ta = 0, tb = 0, tc = 0;
    for (int r = 0; r <= reps; ++r) {
        CK(hipEventRecord(ev[0], 0));
        hipLaunchKernelGGL(pull_far, dim3(cus * 8), dim3(256), 0, 0, F, d_src, V, o1);
        CK(hipEventRecord(ev[1], 0));
        CK(hipMemcpyAsync(curA, baseA, kNC * 8, hipMemcpyDeviceToDevice, 0));
        CK(hipMemcpyAsync(curB, baseB, (uint64_t)nbins * 8, hipMemcpyDeviceToDevice, 0));
        CK(hipEventRecord(ev[2], 0));
        hipLaunchKernelGGL(pass_a, dim3(V / kCA), dim3(256), 0, 0, F, d_optr, d_orcv, V, cshift, curA, A_rcv, A_f);
        CK(hipEventRecord(ev[3], 0));
        hipLaunchKernelGGL(pass_b, dim3((unsigned)chunks.size()), dim3(256), 0, 0, d_chunks, A_rcv, A_f, nf, curB, B_lo,
                           B_f);
        CK(hipEventRecord(ev[4], 0));
        hipLaunchKernelGGL(pass_c, dim3(nbins), dim3(256), 0, 0, binptr, B_lo, B_f, o2);
        CK(hipDeviceSynchronize());
        hipEvent_t e5;
        CK(hipEventCreate(&e5));
        CK(hipEventRecord(e5, 0));
        CK(hipEventSynchronize(e5));
        float a, b, c, d;
        CK(hipEventElapsedTime(&a, ev[0], ev[1]));
        CK(hipEventElapsedTime(&b, ev[2], ev[3]));
        CK(hipEventElapsedTime(&c, ev[3], ev[4]));
        CK(hipEventElapsedTime(&d, ev[4], e5));
        CK(hipEventDestroy(e5));
        if (r) {  // the first repetition warms up
            tp += a / reps;
            ta += b / reps;
            tb += c / reps;
            tc += d / reps;
        }
    }
    printf("V = 2^%d receivers, %llu long-link slots; 256 coarse bins, %u fine bins of 8K receivers\n", LV,
           (unsigned long long)E, nbins);
    printf("pull (random 8-byte gathers): %.3f ms, %.1f G rows/s\n", tp, E / (tp * 1e-3) / 1e9);
    printf("two-level blocking: A %.3f ms + B %.3f ms + C %.3f ms = %.3f ms (%.2fx the pull)\n", ta, tb, tc,
           ta + tb + tc, tp / (ta + tb + tc));
    std::vector<uint64_t> h1(V), h2(V);
    CK(hipMemcpy(h1.data(), o1, V * 8ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), o2, V * 8ull, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint32_t v = 0; v < V; ++v) bad += h1[v] != h2[v];
    printf("check: %llu receivers differ\n", (unsigned long long)bad);
    return bad ? 1 : 0;
}
