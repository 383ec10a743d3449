// generate.hip — on-device builders of the synthetic topologies (gossip_gen.h).
//
// The graphs are the host builders' (host/topology.cpp), restated for the
// device so that a 10^9-node CSR never exists in host memory:
//   * ggh_tree              -> tree_csr: closed form, one thread per row;
//   * ggh_grid_links        -> grid_pairs: right/down neighbour + the seeded
//                              long link of every node (same splitmix stream);
//   * ggh_random_regular    -> perm_pairs: (v, pi_j(v)) per seeded permutation;
//   * ggh_rmat              -> rmat_pairs: the same per-sample stream, the same
//                              rejection of ids >= V, the same relabelling.
// Permutations are the host's sequential Fisher-Yates (host/topology.cpp:100),
// drawn on the host (V x 4 bytes each) and uploaded. Every undirected pair
// becomes two packed keys (row << cb | col), self loops none. The keys are
// emitted grouped into row-range parts of <= 2^31 keys (a bucket histogram of
// the same deterministic pair stream plans the parts), and each part is radix
// sorted on its own (rocPRIM, double buffer); the parts are in row order, so the
// array is then sorted by (row, col) and duplicates are adjacent: a row's
// distinct columns come from one linear pass (row_bounds -> row_count ->
// exclusive scan -> row_write) — the symmetrize + dedup rule of build_sym_csr
// (host/topology.cpp:55-98).
//
// HBM at the 2^30-node grid (C5): keys 6.44e9 x 8 B = 51.5 GB + one part's
// sort buffer 17.2 GB (both freed before the engine allocates its state),
// bounds + counts + row_ptr 3 x 8.6 GB, columns 25.8 GB.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "generate.h"
#include "gossip_spec.h"

namespace gg_gen {
namespace {

constexpr unsigned kBlk = 256;

struct DevRng {  // the host builders' splitmix64 stream (host/topology.cpp:28-35)
    uint64_t s;
    __device__ explicit DevRng(uint64_t seed) : s(seed) {}
    __device__ uint64_t next() { return gg_mix64(s += 0x9E3779B97F4A7C15ull); }
    __device__ uint64_t below(uint64_t n) { return __umul64hi(next(), n); }
};

// Pair generators, one undirected pair per slot (false: no pair — a missing
// grid neighbour or a self loop, both dropped by build_sym_csr).
struct GenParams {
    uint32_t kind;
    uint64_t V, side, seed;
    uint32_t scale;           // R-MAT: log2 of the sampling square
    uint64_t ta, tb, tc;      // R-MAT: quadrant thresholds (x < ta: a, < tb: b, < tc: c, else d)
    const uint32_t* perm;     // R-MAT: relabelling; regular: the k/2 permutations, [j*V + v]
    uint64_t rlo, rhi;        // rows kept: [rlo, rhi) (a vertex-sharded rank's own rows)
};

__device__ __forceinline__ bool pair_at(const GenParams& g, uint64_t slot, uint64_t& a, uint64_t& b) {
    if (g.kind == GG_GEN_GRID_LINKS) {
        // slot 3v+0: right neighbour, 3v+1: down neighbour, 3v+2: the long link
        // (ggh_grid_links, host/topology.cpp:215-232)
        const uint64_t v = slot / 3, t = slot % 3, x = v % g.side, y = v / g.side;
        a = v;
        if (t == 0) {
            if (x + 1 >= g.side) return false;
            b = v + 1;
        } else if (t == 1) {
            if (y + 1 >= g.side) return false;
            b = v + g.side;
        } else {
            DevRng r(gg_mix64(g.seed ^ 0x4c494e4bull) ^ gg_mix64(v));
            b = r.below(g.V);
        }
    } else if (g.kind == GG_GEN_RANDOM_REGULAR) {
        // block j of V pairs: (v, pi_j(v)) (ggh_random_regular, host/topology.cpp:150-163)
        a = slot % g.V;
        b = g.perm[slot];
    } else {
        // sample `slot` of the R-MAT stream, relabelled (ggh_rmat, host/topology.cpp:168-211)
        DevRng r(gg_mix64(g.seed ^ 0x524d4154ull) ^ gg_mix64(slot));
        uint64_t u, v;
        do {
            u = v = 0;
            for (uint32_t s = 0; s < g.scale; ++s) {
                const uint64_t x = r.next();
                uint64_t bu = 0, bv = 0;
                if (x < g.ta) {
                } else if (x < g.tb) {
                    bv = 1;
                } else if (x < g.tc) {
                    bu = 1;
                } else {
                    bu = bv = 1;
                }
                u = (u << 1) | bu;
                v = (v << 1) | bv;
            }
        } while (u >= g.V || v >= g.V);
        a = g.perm[u];
        b = g.perm[v];
    }
    return a != b;
}

// row i starts after the i-1 parent links of rows 1..i-1 and the min(V-1, i*k)
// child links of rows 0..i-1 (ggh_tree, host/topology.cpp:121)
__host__ __device__ inline int64_t tree_row_start(uint64_t V, uint32_t k, uint64_t i) {
    return i >= V ? (int64_t)(2 * (V - 1)) : (int64_t)(i ? i - 1 : 0) + (int64_t)std::min<uint64_t>(V - 1, i * k);
}

// rows [rlo, rhi) of the tree (row_ptr relative to row rlo's first entry)
__global__ void tree_csr(uint64_t V, uint32_t k, uint64_t rlo, uint64_t rhi, int64_t* rp, uint32_t* col,
                         uint32_t col_or) {
    const int64_t s0 = tree_row_start(V, k, rlo);
    for (uint64_t i = rlo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= rhi;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t start = tree_row_start(V, k, i) - s0;
        rp[i - rlo] = start;
        if (i == rhi) continue;
        int64_t p = start;
        if (i > 0) col[p++] = (uint32_t)((i - 1) / k) | col_or;
        for (uint64_t c = i * k + 1; c <= i * k + k && c < V; ++c) col[p++] = (uint32_t)c | col_or;
    }
}

constexpr int kBuckets = 1024;  // row buckets of the part plan
constexpr size_t kMaxParts = 64;
constexpr uint64_t kPartKeys = 1ull << 31;  // keys per sort

// Keys per row bucket (both directions of every pair); LDS histogram per
// block, one global atomic per non-empty bucket per block.
__global__ __launch_bounds__(kBlk) void bucket_hist(GenParams g, uint64_t pairs, uint32_t bshift,
                                                    unsigned long long* hist) {
    __shared__ unsigned int h[kBuckets];
    for (int i = threadIdx.x; i < kBuckets; i += kBlk) h[i] = 0;
    __syncthreads();
    for (uint64_t s = (uint64_t)blockIdx.x * kBlk + threadIdx.x; s < pairs; s += (uint64_t)gridDim.x * kBlk) {
        uint64_t a, b;
        if (!pair_at(g, s, a, b)) continue;
        if (a >= g.rlo && a < g.rhi) atomicAdd(&h[(a - g.rlo) >> bshift], 1u);
        if (b >= g.rlo && b < g.rhi) atomicAdd(&h[(b - g.rlo) >> bshift], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kBuckets; i += kBlk)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// Both keys (row << cb | col) of every pair into the slice of their row's
// part; cursor[p] starts at the part's offset. One atomic per part per wave.
__global__ __launch_bounds__(kBlk) void emit_keys(GenParams g, uint64_t pairs, uint32_t cb, uint32_t n_parts,
                                                  const uint64_t* part_row0, unsigned long long* cursor,
                                                  uint64_t* keys) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlk; base < pairs; base += (uint64_t)gridDim.x * kBlk) {
        const uint64_t s = base + threadIdx.x;
        uint64_t a = 0, b = 0;
        const bool ok = s < pairs && pair_at(g, s, a, b);
        for (int d = 0; d < 2; ++d) {
            const uint64_t row = (d ? b : a) - g.rlo, colv = d ? a : b;  // row local to [rlo, rhi)
            int p = -1;
            if (ok && (d ? b : a) >= g.rlo && (d ? b : a) < g.rhi) {
                p = 0;
                while (p + 1 < (int)n_parts && row >= part_row0[p + 1]) ++p;
            }
            for (uint32_t q = 0; q < n_parts; ++q) {
                const unsigned long long m = __ballot(p == (int)q);
                if (!m) continue;
                const int leader = __ffsll((long long)m) - 1;
                unsigned long long at = 0;
                if (lane == leader) at = atomicAdd(&cursor[q], (unsigned long long)__popcll(m));
                at = __shfl(at, leader, 64);
                if (p == (int)q) keys[at + __popcll(m & lt)] = (row << cb) | colv;
            }
        }
    }
}

// first[r] = index of the first sorted key of row r (rows without keys take the
// next row's index); first[V] = M
__global__ void row_bounds(const uint64_t* keys, uint64_t M, uint64_t V, uint32_t cb, int64_t* first) {
    auto row = [&](uint64_t i) -> uint64_t { return i >= M ? V : keys[i] >> cb; };
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= M; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = row(k);
        const uint64_t lo = k ? row(k - 1) + 1 : 0;
        for (uint64_t q = lo; q <= r && q <= V; ++q) first[q] = (int64_t)k;
    }
}

__global__ void row_count(const uint64_t* keys, const int64_t* first, uint64_t V, int64_t* cnt) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= V; v += (uint64_t)gridDim.x * blockDim.x) {
        int64_t c = 0;
        uint64_t last = ~0ull;  // never a key: rows are < 2^cb - 1
        if (v < V)
            for (int64_t i = first[v]; i < first[v + 1]; ++i) {
                const uint64_t key = keys[i];
                c += key != last;
                last = key;
            }
        cnt[v] = c;
    }
}

__global__ void row_write(const uint64_t* keys, const int64_t* first, const int64_t* rp, uint64_t V, uint32_t cb,
                          uint32_t col_or, uint32_t* col) {
    const uint64_t cmask = (1ull << cb) - 1;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (uint64_t)gridDim.x * blockDim.x) {
        int64_t p = rp[v];
        uint64_t last = ~0ull;
        for (int64_t i = first[v]; i < first[v + 1]; ++i) {
            const uint64_t key = keys[i];
            if (key != last) col[p++] = (uint32_t)(key & cmask) | col_or;
            last = key;
        }
    }
}

__global__ void degree_max(const int64_t* rp, uint64_t V, unsigned long long* out) {
    unsigned long long m = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (uint64_t)gridDim.x * blockDim.x)
        m = std::max<unsigned long long>(m, (unsigned long long)(rp[v + 1] - rp[v]));
    __shared__ unsigned long long s[kBlk];
    s[threadIdx.x] = m;
    __syncthreads();
    for (unsigned w = kBlk / 2; w; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = std::max(s[threadIdx.x], s[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(out, s[0]);
}

// Grids are capped and every kernel strides: a dispatch's grid size in
// work-items is a 32-bit field, so 2^32 or more threads (6.4e9 keys at C5)
// cannot be launched one per item.
// grid-stride kernels: at least one block (an empty input still launches validly)
unsigned grid_of(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + kBlk - 1) / kBlk, 1u << 16)); }

// host/topology.cpp:100-106 (the permutation is part of the graph's definition)
std::vector<uint32_t> permutation(uint64_t V, uint64_t seed) {
    std::vector<uint32_t> p(V);
    for (uint64_t i = 0; i < V; ++i) p[i] = (uint32_t)i;
    uint64_t s = seed;
    for (uint64_t i = V; i > 1; --i) {
        const uint64_t x = gg_mix64(s += 0x9E3779B97F4A7C15ull);
        std::swap(p[i - 1], p[(uint64_t)(((unsigned __int128)x * i) >> 64)]);
    }
    return p;
}

struct Scoped {  // device allocations released on every exit path
    std::vector<void*> ptrs;
    ~Scoped() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    hipError_t alloc(T** p, size_t bytes) {
        hipError_t e = hipMalloc((void**)p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) ptrs.push_back((void*)*p);
        return e;
    }
    void release(void* p) {  // free now
        auto it = std::find(ptrs.begin(), ptrs.end(), p);
        if (it != ptrs.end()) {
            (void)hipFree(p);
            ptrs.erase(it);
        }
    }
    void keep(void* p) {  // ownership to the caller
        auto it = std::find(ptrs.begin(), ptrs.end(), p);
        if (it != ptrs.end()) ptrs.erase(it);
    }
};

}  // namespace

#define GCHK(x)                                                              \
    do {                                                                     \
        hipError_t err_ = (x);                                               \
        if (err_ != hipSuccess) {                                            \
            *err = std::string(#x) + ": " + hipGetErrorString(err_);         \
            return -5;                                                       \
        }                                                                    \
    } while (0)

uint64_t spec_nodes(const gg_gen_spec& s) { return s.kind == GG_GEN_GRID_LINKS ? s.n * s.n : s.n; }

int build_csr(const gg_gen_spec& s, hipStream_t st, uint32_t col_or, Csr* out, std::string* err) {
    return build_csr_rows(s, st, col_or, 0, spec_nodes(s), out, err);
}

int build_csr_rows(const gg_gen_spec& s, hipStream_t st, uint32_t col_or, uint64_t rlo, uint64_t rhi, Csr* out,
                   std::string* err) {
    const uint64_t V = spec_nodes(s);
    if (V == 0 || V > 0x7fffffffull) {
        *err = "generator: node count must be in [1, 2^31)";
        return -22;
    }
    if (rlo > rhi || rhi > V) {
        *err = "generator: row range outside [0, V]";
        return -22;
    }
    const uint64_t n = rhi - rlo;  // rows built
    Scoped mem;
    int64_t* rp = nullptr;
    uint32_t* col = nullptr;
    GCHK(mem.alloc(&rp, (n + 1) * 8));
    if (s.kind == GG_GEN_TREE) {
        if (s.k == 0) {
            *err = "generator: tree arity must be >= 1";
            return -22;
        }
        const uint64_t nnz = (uint64_t)(tree_row_start(V, s.k, rhi) - tree_row_start(V, s.k, rlo));
        GCHK(mem.alloc(&col, nnz * 4));
        hipLaunchKernelGGL(tree_csr, dim3(grid_of(n + 1)), dim3(kBlk), 0, st, V, s.k, rlo, rhi, rp, col, col_or);
        GCHK(hipGetLastError());
        GCHK(hipStreamSynchronize(st));
        mem.keep(rp);
        mem.keep(col);
        *out = {rp, col, n, nnz};
        return 0;
    }
    // undirected pairs -> packed keys (row << cb | col), both directions
    uint32_t cb = 1;
    while ((1ull << cb) <= V) ++cb;
    GenParams g{};
    g.kind = s.kind;
    g.V = V;
    g.side = s.n;
    g.seed = s.seed;
    g.rlo = rlo;
    g.rhi = rhi;
    uint64_t pairs = 0;
    std::vector<uint32_t> perm;
    uint32_t* d_perm = nullptr;
    switch (s.kind) {
    case GG_GEN_GRID_LINKS:
        if (s.n < 2) { *err = "generator: grid side must be >= 2"; return -22; }
        pairs = 3 * V;
        break;
    case GG_GEN_RANDOM_REGULAR:
        if (s.k < 2 || s.k % 2) { *err = "generator: regular degree must be even and >= 2"; return -22; }
        pairs = V * (s.k / 2);
        GCHK(mem.alloc(&d_perm, pairs * 4));
        for (uint32_t j = 0; j < s.k / 2; ++j) {
            perm = permutation(V, gg_mix64(s.seed ^ (0x52454755ull + j)));
            GCHK(hipMemcpy(d_perm + (uint64_t)j * V, perm.data(), V * 4, hipMemcpyHostToDevice));
        }
        break;
    case GG_GEN_RMAT:
        if (V < 2 || s.k == 0) { *err = "generator: R-MAT needs >= 2 nodes and edge factor >= 1"; return -22; }
        pairs = V * s.k;
        while ((1ull << g.scale) < V) ++g.scale;
        g.ta = (uint64_t)(s.a * 18446744073709551616.0);
        g.tb = (uint64_t)((s.a + s.b) * 18446744073709551616.0);
        g.tc = (uint64_t)((s.a + s.b + s.c) * 18446744073709551616.0);
        perm = permutation(V, gg_mix64(s.seed ^ 0x5045524dull));
        GCHK(mem.alloc(&d_perm, V * 4));
        GCHK(hipMemcpy(d_perm, perm.data(), V * 4, hipMemcpyHostToDevice));
        break;
    default:
        *err = "generator: unknown kind";
        return -22;
    }
    std::vector<uint32_t>().swap(perm);
    g.perm = d_perm;
    // part plan: row ranges of at most kPartKeys keys each, sorted one at a time
    // (rocPRIM's radix sort keeps 32-bit digit counts: one sort stays < 2^32 keys)
    uint64_t part_keys = kPartKeys;
    if (const char* e = getenv("GG_GEN_PART_KEYS")) part_keys = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    uint32_t bshift = 0;
    while (n > 1 && (n - 1) >> bshift >= (uint64_t)kBuckets) ++bshift;
    unsigned long long* d_hist = nullptr;
    GCHK(mem.alloc(&d_hist, (kBuckets + kMaxParts) * 8));
    GCHK(hipMemsetAsync(d_hist, 0, kBuckets * 8, st));
    const unsigned gblocks = std::min(grid_of(pairs), 4096u);
    hipLaunchKernelGGL(bucket_hist, dim3(gblocks), dim3(kBlk), 0, st, g, pairs, bshift, d_hist);
    GCHK(hipGetLastError());
    std::vector<unsigned long long> hist(kBuckets);
    GCHK(hipMemcpyAsync(hist.data(), d_hist, kBuckets * 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    std::vector<uint64_t> row0{0}, off{0};  // part p: rows [row0[p], row0[p+1]), keys [off[p], off[p+1])
    uint64_t in_part = 0, M = 0;
    for (int q = 0; q < kBuckets; ++q) {
        if (in_part && in_part + hist[q] > part_keys && row0.size() < kMaxParts) {
            row0.push_back((uint64_t)q << bshift);
            off.push_back(M);
            in_part = 0;
        }
        in_part += hist[q];
        M += hist[q];
    }
    row0.push_back(n);
    off.push_back(M);
    const uint32_t n_parts = (uint32_t)row0.size() - 1;
    uint64_t max_part = 0;
    for (uint32_t q = 0; q < n_parts; ++q) max_part = std::max(max_part, off[q + 1] - off[q]);
    if (max_part >= (1ull << 32)) {
        *err = "generator: a row bucket holds >= 2^32 adjacency entries";
        return -22;
    }
    uint64_t* keys = nullptr;
    uint64_t* alt = nullptr;
    uint64_t* d_row0 = nullptr;
    GCHK(mem.alloc(&keys, M * 8));
    GCHK(mem.alloc(&d_row0, row0.size() * 8));
    GCHK(hipMemcpy(d_row0, row0.data(), row0.size() * 8, hipMemcpyHostToDevice));
    unsigned long long* d_cur = d_hist + kBuckets;
    GCHK(hipMemcpy(d_cur, off.data(), n_parts * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(emit_keys, dim3(gblocks), dim3(kBlk), 0, st, g, pairs, cb, n_parts, d_row0, d_cur, keys);
    GCHK(hipGetLastError());
    GCHK(hipStreamSynchronize(st));
    if (d_perm) mem.release(d_perm);
    // sort each part's slice by (row, col): the parts are row ranges in order,
    // so the whole array ends up sorted
    GCHK(mem.alloc(&alt, max_part * 8));
    size_t tmp_bytes = 0;
    void* tmp = nullptr;
    {
        rocprim::double_buffer<uint64_t> db(keys, alt);
        GCHK(rocprim::radix_sort_keys(nullptr, tmp_bytes, db, (size_t)max_part, 0, 2 * cb, st));
        GCHK(mem.alloc(&tmp, tmp_bytes));
    }
    for (uint32_t q = 0; q < n_parts; ++q) {
        const uint64_t n = off[q + 1] - off[q];
        if (n < 2) continue;
        rocprim::double_buffer<uint64_t> db(keys + off[q], alt);
        size_t tb = tmp_bytes;
        GCHK(rocprim::radix_sort_keys(tmp, tb, db, (size_t)n, 0, 2 * cb, st));
        if (db.current() != keys + off[q])
            GCHK(hipMemcpyAsync(keys + off[q], db.current(), n * 8, hipMemcpyDeviceToDevice, st));
    }
    GCHK(hipStreamSynchronize(st));
    mem.release(tmp);
    mem.release(alt);
    // CSR of the distinct (row, col) keys
    int64_t* first = nullptr;
    int64_t* cnt = nullptr;
    GCHK(mem.alloc(&first, (n + 1) * 8));
    GCHK(mem.alloc(&cnt, (n + 1) * 8));
    hipLaunchKernelGGL(row_bounds, dim3(grid_of(M + 1)), dim3(kBlk), 0, st, keys, M, n, cb, first);
    GCHK(hipGetLastError());
    hipLaunchKernelGGL(row_count, dim3(grid_of(n + 1)), dim3(kBlk), 0, st, keys, first, n, cnt);
    GCHK(hipGetLastError());
    tmp_bytes = 0;
    GCHK(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt, rp, (int64_t)0, n + 1, rocprim::plus<int64_t>(), st));
    GCHK(mem.alloc(&tmp, tmp_bytes));
    GCHK(rocprim::exclusive_scan(tmp, tmp_bytes, cnt, rp, (int64_t)0, n + 1, rocprim::plus<int64_t>(), st));
    int64_t nnz = 0;
    GCHK(hipMemcpyAsync(&nnz, rp + n, 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    mem.release(tmp);
    mem.release(cnt);
    GCHK(mem.alloc(&col, (uint64_t)nnz * 4));
    hipLaunchKernelGGL(row_write, dim3(grid_of(n)), dim3(kBlk), 0, st, keys, first, rp, n, cb, col_or, col);
    GCHK(hipGetLastError());
    GCHK(hipStreamSynchronize(st));
    mem.keep(rp);
    mem.keep(col);
    *out = {rp, col, n, (uint64_t)nnz};
    return 0;
}

namespace {

__global__ void deg_keys(const int64_t* rp, uint64_t V, uint64_t* keys) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (uint64_t)gridDim.x * blockDim.x)
        keys[v] = ((uint64_t)(0xffffffffu - (uint32_t)(rp[v + 1] - rp[v])) << 32) | v;  // descending degree, then id
}

__global__ void order_from_keys(const uint64_t* keys, const int64_t* rp, uint64_t V, uint64_t rows, uint32_t* gid,
                                uint32_t* loc, int64_t* ndeg) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i >= V) {
            gid[i] = ~0u;  // padding rows
            continue;
        }
        const uint32_t v = (uint32_t)(keys[i] & 0xffffffffu);
        gid[i] = v;
        loc[v] = (uint32_t)i;
        ndeg[i] = rp[v + 1] - rp[v];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ndeg[V] = 0;
}

// Column j of the reordered CSR: its row i (binary search in nrp), that row's
// node v = gid[i], entry j - nrp[i] of v's old list, mapped to its local row.
// Edge-parallel, so a 10^6-entry hub row costs no more than its share.
__global__ void copy_reordered(const int64_t* rp, const uint32_t* col, const int64_t* nrp, const uint32_t* gid,
                               const uint32_t* loc, uint64_t V, uint64_t nnz, uint32_t col_or, uint32_t* ncol) {
    const uint32_t cmask = 0x7fffffffu;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz; j += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = V - 1;
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if ((uint64_t)nrp[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t v = gid[lo];
        ncol[j] = loc[col[rp[v] + (int64_t)(j - (uint64_t)nrp[lo])] & cmask] | col_or;
    }
}

}  // namespace

int degree_reorder(Csr* g, uint64_t rows, hipStream_t st, uint32_t col_or, uint32_t** gid_out,
                   std::vector<uint32_t>* gid_host, std::vector<uint32_t>* loc_host, std::string* err) {
    const uint64_t V = g->V;
    Scoped mem;
    uint64_t* keys = nullptr;
    uint64_t* alt = nullptr;
    uint32_t* gid = nullptr;
    uint32_t* loc = nullptr;
    int64_t* ndeg = nullptr;
    int64_t* nrp = nullptr;
    uint32_t* ncol = nullptr;
    GCHK(mem.alloc(&keys, V * 8));
    GCHK(mem.alloc(&alt, V * 8));
    hipLaunchKernelGGL(deg_keys, dim3(grid_of(V)), dim3(kBlk), 0, st, g->row_ptr, V, keys);
    GCHK(hipGetLastError());
    size_t tmp_bytes = 0;
    void* tmp = nullptr;
    {
        rocprim::double_buffer<uint64_t> db(keys, alt);
        GCHK(rocprim::radix_sort_keys(nullptr, tmp_bytes, db, (size_t)V, 0, 64, st));
        GCHK(mem.alloc(&tmp, tmp_bytes));
        GCHK(rocprim::radix_sort_keys(tmp, tmp_bytes, db, (size_t)V, 0, 64, st));
        if (db.current() != keys) std::swap(keys, alt);
    }
    mem.release(tmp);
    GCHK(mem.alloc(&gid, rows * 4));
    GCHK(mem.alloc(&loc, V * 4));
    GCHK(mem.alloc(&ndeg, (V + 1) * 8));
    hipLaunchKernelGGL(order_from_keys, dim3(grid_of(rows)), dim3(kBlk), 0, st, keys, g->row_ptr, V, rows, gid, loc,
                       ndeg);
    GCHK(hipGetLastError());
    mem.release(keys);
    mem.release(alt);
    GCHK(mem.alloc(&nrp, (V + 1) * 8));
    tmp_bytes = 0;
    GCHK(rocprim::exclusive_scan(nullptr, tmp_bytes, ndeg, nrp, (int64_t)0, V + 1, rocprim::plus<int64_t>(), st));
    GCHK(mem.alloc(&tmp, tmp_bytes));
    GCHK(rocprim::exclusive_scan(tmp, tmp_bytes, ndeg, nrp, (int64_t)0, V + 1, rocprim::plus<int64_t>(), st));
    mem.release(tmp);
    mem.release(ndeg);
    GCHK(mem.alloc(&ncol, g->nnz * 4));
    if (g->nnz) {
        hipLaunchKernelGGL(copy_reordered, dim3(grid_of(g->nnz)), dim3(kBlk), 0, st, g->row_ptr, g->col, nrp, gid,
                           loc, V, g->nnz, col_or, ncol);
        GCHK(hipGetLastError());
    }
    gid_host->resize(rows);
    loc_host->resize(V);
    GCHK(hipMemcpyAsync(gid_host->data(), gid, rows * 4, hipMemcpyDeviceToHost, st));
    GCHK(hipMemcpyAsync(loc_host->data(), loc, V * 4, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    (void)hipFree(g->row_ptr);
    (void)hipFree(g->col);
    g->row_ptr = nrp;
    g->col = ncol;
    mem.keep(nrp);
    mem.keep(ncol);
    mem.keep(gid);
    *gid_out = gid;
    return 0;
}

int max_degree(const int64_t* d_rp, uint64_t V, hipStream_t st, uint64_t* out, std::string* err) {
    unsigned long long* d = nullptr;
    GCHK(hipMalloc(&d, 8));
    hipError_t e1 = hipMemsetAsync(d, 0, 8, st);
    if (e1 == hipSuccess) {
        const unsigned blocks = (unsigned)std::min<uint64_t>(4096, std::max<uint64_t>(1, grid_of(V)));
        hipLaunchKernelGGL(degree_max, dim3(blocks), dim3(kBlk), 0, st, d_rp, V, d);
        e1 = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e1 == hipSuccess) e1 = hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, st);
    if (e1 == hipSuccess) e1 = hipStreamSynchronize(st);
    (void)hipFree(d);
    GCHK(e1);
    *out = h;
    return 0;
}


// ---------------------------------------------------------------------------
// Vertex-sharded ranks: one rank's own rows [lo, hi) of a symmetric generated
// graph (build_csr_rows) -> its ghosts, send lists and ghost -> owned lists,
// all on the device (nothing of the whole graph anywhere). Symmetric: owned u
// is a ghost on part q iff u has a neighbour in q, so u's send list to q is
// read off u's own row, in the same ascending-id order as q's ghosts from here.
namespace {

__device__ __forceinline__ uint32_t part_of(const uint64_t* plo, uint32_t P, uint64_t v) {
    uint32_t lo = 0, hi = P;  // largest p with plo[p] <= v
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (plo[mid] <= v) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t lower_bound32(const uint32_t* a, uint64_t n, uint32_t x) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// edge k's row (one thread per row)
__global__ void edge_rows(const int64_t* rp, uint64_t n, uint32_t* erow) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) erow[k] = (uint32_t)i;
}

// remote columns (~0u for own rows' columns: they sort last)
__global__ void remote_cols(const uint32_t* col, uint64_t m, uint64_t lo, uint64_t hi, uint32_t* out) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = col[k];
        out[k] = (c >= lo && c < hi) ? ~0u : (uint32_t)c;
    }
}

// send keys (part << 32 | owned row), ghost keys (ghost << 32 | owned row);
// ~0 for an edge inside the part; per-part send counts come after the unique
__global__ void cut_keys(const uint32_t* col, const uint32_t* erow, uint64_t m, uint64_t lo, uint64_t hi,
                         const uint64_t* plo, uint32_t P, const uint32_t* ghosts, uint64_t n_ghost, uint64_t* skey,
                         uint64_t* gkey, unsigned long long* gcnt) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = col[k];
        if (c >= lo && c < hi) {
            skey[k] = gkey[k] = ~0ull;
            continue;
        }
        const uint64_t gi = lower_bound32(ghosts, n_ghost, (uint32_t)c);
        skey[k] = ((uint64_t)part_of(plo, P, c) << 32) | erow[k];
        gkey[k] = (gi << 32) | erow[k];
        atomicAdd(&gcnt[gi], 1ull);
    }
}

__global__ void send_counts(const uint64_t* skey, uint64_t n, unsigned long long* cnt) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
        atomicAdd(&cnt[skey[k] >> 32], 1ull);
    }
}

__global__ void low_words(const uint64_t* key, uint64_t n, uint32_t* out) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
        out[k] = (uint32_t)key[k];
}

// ghost -> owned edge j: the owned row, and its entry in the send list to the
// ghost's part (the list is ascending, so a binary search)
__global__ void ghost_lists(const uint64_t* gkey, uint64_t m, const uint64_t* recv_off, const uint64_t* send_off,
                            uint32_t P, const uint32_t* send_idx, uint32_t* gout_col, uint32_t* gout_sidx) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = gkey[j] >> 32;
        const uint32_t u = (uint32_t)gkey[j];
        const uint32_t p = part_of(recv_off, P, g);
        gout_col[j] = u;
        gout_sidx[j] = (uint32_t)(send_off[p] + lower_bound32(send_idx + send_off[p], send_off[p + 1] - send_off[p], u));
    }
}

// columns -> local rows: own rows first, ghosts from ghost0 (| col_or)
__global__ void remap_cols(uint32_t* col, uint64_t m, uint64_t lo, uint64_t hi, const uint32_t* ghosts,
                           uint64_t n_ghost, uint64_t ghost0, uint32_t col_or) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = col[k];
        const uint64_t r = (c >= lo && c < hi) ? c - lo : ghost0 + lower_bound32(ghosts, n_ghost, (uint32_t)c);
        col[k] = (uint32_t)r | col_or;
    }
}

// Every index the round kernels will follow, checked before any of them runs:
// columns are own rows or ghost rows, receivers own rows, send entries in range.
__global__ void check_shard(const int64_t* rp, uint64_t n, const uint32_t* col, uint64_t m, uint64_t ghost0,
                            uint64_t n_ghost, const uint32_t* send_idx, uint64_t n_send, const int64_t* gout_ptr,
                            const uint32_t* gout_col, const uint32_t* gout_sidx, uint64_t n_cut,
                            unsigned long long* bad) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long b = 0;
    for (uint64_t k = t; k < m; k += st) {
        const uint64_t c = col[k] & 0x7fffffffu;
        b += !(c < n || (c >= ghost0 && c < ghost0 + n_ghost));
    }
    for (uint64_t i = t; i < n; i += st) b += rp[i + 1] < rp[i];
    for (uint64_t k = t; k < n_send; k += st) b += send_idx[k] >= n;
    for (uint64_t j = t; j < n_cut; j += st) b += gout_col[j] >= n || gout_sidx[j] >= n_send;
    for (uint64_t g = t; g < n_ghost; g += st) b += gout_ptr[g + 1] < gout_ptr[g];
    if (b) atomicAdd(bad, b);
}

// local row -> node id (owned: lo + row; ghosts from ghost0; ~0u padding)
__global__ void fill_gid(uint64_t rows, uint64_t lo, uint64_t n_own, uint64_t ghost0, const uint32_t* ghosts,
                         uint64_t n_ghost, uint32_t* gid) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (uint64_t)gridDim.x * blockDim.x)
        gid[r] = r < n_own ? (uint32_t)(lo + r)
                 : (r >= ghost0 && r < ghost0 + n_ghost) ? ghosts[r - ghost0] : ~0u;
}

// ---- shard_reorder ----------------------------------------------------------
// keys of n items: (0xffffffff - count) << 32 | item, count = ptr[i+1] - ptr[i]
__global__ void count_keys(const int64_t* ptr, uint64_t n, uint64_t* keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keys[i] = ((uint64_t)(0xffffffffu - (uint32_t)(ptr[i + 1] - ptr[i])) << 32) | i;
}

// sorted keys -> order[new] = old, inverse perm[old] = new, new counts (for the scan)
__global__ void perm_from_keys(const uint64_t* keys, const int64_t* ptr, uint64_t n, uint32_t* order, uint32_t* perm,
                               int64_t* ncnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t old = (uint32_t)(keys[i] & 0xffffffffu);
        order[i] = old;
        perm[old] = (uint32_t)i;
        ncnt[i] = ptr[old + 1] - ptr[old];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ncnt[n] = 0;
}

// a local row under the new numbering (owned: perm, ghosts: gperm; | the recip bit kept)
__device__ __forceinline__ uint32_t renum(uint32_t c, uint64_t n_own, uint64_t ghost0, const uint32_t* perm,
                                          const uint32_t* gperm) {
    const uint32_t r = c & 0x7fffffffu, hi = c & 0x80000000u;
    if (r < n_own) return perm[r] | hi;
    if (r >= ghost0) return (uint32_t)(ghost0 + gperm[r - ghost0]) | hi;
    return c;
}

// entry j of the reordered list arrays: its new row (binary search in nptr),
// that row's old row, the same entry of the old list, renumbered
__global__ void copy_lists(const int64_t* ptr, const uint32_t* vals, const int64_t* nptr, const uint32_t* order,
                           uint64_t n, uint64_t nnz, int renumber, uint64_t n_own, uint64_t ghost0,
                           const uint32_t* perm, const uint32_t* gperm, const uint32_t* vals2, uint32_t* nvals,
                           uint32_t* nvals2) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz; j += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = n - 1;
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if ((uint64_t)nptr[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const uint64_t src = (uint64_t)ptr[order[lo]] + (j - (uint64_t)nptr[lo]);
        const uint32_t v = vals[src];
        nvals[j] = renumber ? renum(v, n_own, ghost0, perm, gperm) : v;
        if (nvals2) nvals2[j] = vals2[src];
    }
}

__global__ void renum_array(uint32_t* a, uint64_t n, uint64_t n_own, uint64_t ghost0, const uint32_t* perm,
                            const uint32_t* gperm) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = renum(a[i], n_own, ghost0, perm, gperm);
}

__global__ void permute_gid(const uint32_t* gid, uint64_t rows, uint64_t n_own, uint64_t ghost0, uint64_t n_ghost,
                            const uint32_t* order, const uint32_t* gorder, uint32_t* ngid) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (uint64_t)gridDim.x * blockDim.x) {
        if (r < n_own) ngid[r] = gid[order[r]];
        else if (r >= ghost0 && r < ghost0 + n_ghost) ngid[r] = gid[ghost0 + gorder[r - ghost0]];
        else ngid[r] = gid[r];
    }
}

}  // namespace

namespace {
// order/perm of n items by descending count (ptr differences), and the new ptr
int order_by_count(const int64_t* ptr, uint64_t n, hipStream_t st, Scoped& mem, uint32_t** order, uint32_t** perm,
                   int64_t** nptr, std::string* err) {
    uint64_t* keys = nullptr;
    uint64_t* alt = nullptr;
    int64_t* ncnt = nullptr;
    GCHK(mem.alloc(&keys, std::max<uint64_t>(1, n) * 8));
    GCHK(mem.alloc(&alt, std::max<uint64_t>(1, n) * 8));
    GCHK(mem.alloc(order, std::max<uint64_t>(1, n) * 4));
    GCHK(mem.alloc(perm, std::max<uint64_t>(1, n) * 4));
    GCHK(mem.alloc(&ncnt, (n + 1) * 8));
    GCHK(mem.alloc(nptr, (n + 1) * 8));
    hipLaunchKernelGGL(count_keys, dim3(grid_of(n)), dim3(kBlk), 0, st, ptr, n, keys);
    GCHK(hipGetLastError());
    size_t tb = 0;
    void* tmp = nullptr;
    if (n) {
        rocprim::double_buffer<uint64_t> db(keys, alt);
        GCHK(rocprim::radix_sort_keys(nullptr, tb, db, (size_t)n, 0, 64, st));
        GCHK(mem.alloc(&tmp, tb));
        GCHK(rocprim::radix_sort_keys(tmp, tb, db, (size_t)n, 0, 64, st));
        if (db.current() != keys) std::swap(keys, alt);
        mem.release(tmp);
    }
    hipLaunchKernelGGL(perm_from_keys, dim3(grid_of(n)), dim3(kBlk), 0, st, keys, ptr, n, *order, *perm, ncnt);
    GCHK(hipGetLastError());
    tb = 0;
    GCHK(rocprim::exclusive_scan(nullptr, tb, ncnt, *nptr, (int64_t)0, n + 1, rocprim::plus<int64_t>(), st));
    GCHK(mem.alloc(&tmp, tb));
    GCHK(rocprim::exclusive_scan(tmp, tb, ncnt, *nptr, (int64_t)0, n + 1, rocprim::plus<int64_t>(), st));
    mem.release(tmp);
    mem.release(keys);
    mem.release(alt);
    mem.release(ncnt);
    return 0;
}
}  // namespace

int shard_reorder(Csr* g, Shard* sh, uint64_t ghost0, uint32_t col_or, hipStream_t st, uint32_t** grow_out,
                  std::vector<uint32_t>* own_row, std::string* err) {
    (void)col_or;
    const uint64_t n = g->V, m = g->nnz, ng = sh->n_ghost, nc = sh->n_cut;
    const uint64_t rows = std::max<uint64_t>(64, (ghost0 + ng + 63) / 64 * 64);
    Scoped mem;
    uint32_t *order = nullptr, *perm = nullptr, *gorder = nullptr, *gperm = nullptr;
    int64_t *nrp = nullptr, *ngp = nullptr;
    if (int r = order_by_count(g->row_ptr, n, st, mem, &order, &perm, &nrp, err)) return r;
    if (int r = order_by_count(sh->gout_ptr, ng, st, mem, &gorder, &gperm, &ngp, err)) return r;
    uint32_t *ncol = nullptr, *ngcol = nullptr, *ngsidx = nullptr, *ngid = nullptr;
    GCHK(mem.alloc(&ncol, std::max<uint64_t>(1, m) * 4));
    GCHK(mem.alloc(&ngcol, std::max<uint64_t>(1, nc) * 4));
    GCHK(mem.alloc(&ngsidx, std::max<uint64_t>(1, nc) * 4));
    GCHK(mem.alloc(&ngid, rows * 4));
    if (m) {
        hipLaunchKernelGGL(copy_lists, dim3(grid_of(m)), dim3(kBlk), 0, st, g->row_ptr, g->col, nrp, order, n, m, 1,
                           n, ghost0, perm, gperm, (const uint32_t*)nullptr, ncol, (uint32_t*)nullptr);
        GCHK(hipGetLastError());
    }
    if (nc) {  // ghost -> owned lists by new ghost row: receivers renumbered, send entries kept
        hipLaunchKernelGGL(copy_lists, dim3(grid_of(nc)), dim3(kBlk), 0, st, sh->gout_ptr, sh->gout_col, ngp, gorder,
                           ng, nc, 1, n, ghost0, perm, gperm, sh->gout_sidx, ngcol, ngsidx);
        GCHK(hipGetLastError());
    }
    if (sh->n_send) {  // send entries keep their positions (the receiver's ghost order); rows renumbered
        hipLaunchKernelGGL(renum_array, dim3(grid_of(sh->n_send)), dim3(kBlk), 0, st, sh->send_idx, sh->n_send, n,
                           ghost0, perm, gperm);
        GCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(permute_gid, dim3(grid_of(rows)), dim3(kBlk), 0, st, sh->gid, rows, n, ghost0, ng, order,
                       gorder, ngid);
    GCHK(hipGetLastError());
    own_row->resize(n);
    if (n) GCHK(hipMemcpyAsync(own_row->data(), perm, n * 4, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    (void)hipFree(g->row_ptr);
    (void)hipFree(g->col);
    (void)hipFree(sh->gout_ptr);
    (void)hipFree(sh->gout_col);
    (void)hipFree(sh->gout_sidx);
    (void)hipFree(sh->gid);
    g->row_ptr = nrp;
    g->col = ncol;
    sh->gout_ptr = ngp;
    sh->gout_col = ngcol;
    sh->gout_sidx = ngsidx;
    sh->gid = ngid;
    mem.keep(nrp);
    mem.keep(ncol);
    mem.keep(ngp);
    mem.keep(ngcol);
    mem.keep(ngsidx);
    mem.keep(ngid);
    mem.keep(gperm);
    *grow_out = gperm;
    return 0;
}

namespace {

template <class K>
int sort_unique(K* keys, uint64_t n, int bits, hipStream_t st, uint64_t* n_unique, std::string* err) {
    Scoped mem;
    K* alt = nullptr;
    GCHK(mem.alloc(&alt, n * sizeof(K)));
    size_t tb = 0;
    void* tmp = nullptr;
    {
        rocprim::double_buffer<K> db(keys, alt);
        GCHK(rocprim::radix_sort_keys(nullptr, tb, db, (size_t)n, 0, bits, st));
        GCHK(mem.alloc(&tmp, tb));
        GCHK(rocprim::radix_sort_keys(tmp, tb, db, (size_t)n, 0, bits, st));
        if (db.current() != keys) GCHK(hipMemcpyAsync(keys, db.current(), n * sizeof(K), hipMemcpyDeviceToDevice, st));
    }
    mem.release(tmp);
    if (!n_unique) {
        GCHK(hipStreamSynchronize(st));
        return 0;
    }
    size_t* d_cnt = nullptr;
    GCHK(mem.alloc(&d_cnt, sizeof(size_t)));
    tb = 0;
    GCHK(rocprim::unique(nullptr, tb, keys, alt, d_cnt, (size_t)n, rocprim::equal_to<K>(), st));
    GCHK(mem.alloc(&tmp, tb));
    GCHK(rocprim::unique(tmp, tb, keys, alt, d_cnt, (size_t)n, rocprim::equal_to<K>(), st));
    size_t h = 0;
    GCHK(hipMemcpyAsync(&h, d_cnt, sizeof(size_t), hipMemcpyDeviceToHost, st));
    GCHK(hipMemcpyAsync(keys, alt, n * sizeof(K), hipMemcpyDeviceToDevice, st));
    GCHK(hipStreamSynchronize(st));
    *n_unique = h;
    return 0;
}

}  // namespace

int shard_csr(Csr* g, uint64_t lo, uint64_t hi, const std::vector<uint64_t>& plo, uint64_t ghost0, uint32_t col_or,
              hipStream_t st, Shard* out, std::string* err) {
    const uint64_t m = g->nnz, n = hi - lo;
    const uint32_t P = (uint32_t)plo.size() - 1;
    Scoped mem;
    uint32_t* rc = nullptr;  // remote columns -> ghosts
    uint32_t* erow = nullptr;
    uint64_t* d_plo = nullptr;
    GCHK(mem.alloc(&rc, m * 4));
    GCHK(mem.alloc(&erow, m * 4));
    GCHK(mem.alloc(&d_plo, plo.size() * 8));
    GCHK(hipMemcpyAsync(d_plo, plo.data(), plo.size() * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(edge_rows, dim3(grid_of(n)), dim3(kBlk), 0, st, g->row_ptr, n, erow);
    hipLaunchKernelGGL(remote_cols, dim3(grid_of(m)), dim3(kBlk), 0, st, g->col, m, lo, hi, rc);
    GCHK(hipGetLastError());
    uint64_t nu = 0;
    if (int r = sort_unique(rc, m, 32, st, &nu, err)) return r;
    std::vector<uint32_t> last(1, 0);
    if (nu) GCHK(hipMemcpyAsync(last.data(), rc + nu - 1, 4, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    const uint64_t n_ghost = (nu && last[0] == ~0u) ? nu - 1 : nu;
    out->n_ghost = n_ghost;
    out->ghosts_host.resize(n_ghost);
    if (n_ghost) GCHK(hipMemcpyAsync(out->ghosts_host.data(), rc, n_ghost * 4, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    out->recv_off.assign(P + 1, 0);
    for (uint32_t q = 0; q <= P; ++q)
        out->recv_off[q] = (uint64_t)(std::lower_bound(out->ghosts_host.begin(), out->ghosts_host.end(),
                                                       (uint32_t)std::min<uint64_t>(plo[q], 0xffffffffull)) -
                                      out->ghosts_host.begin());
    out->recv_off[P] = n_ghost;
    // cut edges: send keys and ghost keys
    uint64_t* skey = nullptr;
    uint64_t* gkey = nullptr;
    unsigned long long* gcnt = nullptr;
    GCHK(mem.alloc(&skey, m * 8));
    GCHK(mem.alloc(&gkey, m * 8));
    GCHK(mem.alloc(&gcnt, (n_ghost + 1) * 8));
    GCHK(hipMemsetAsync(gcnt, 0, (n_ghost + 1) * 8, st));
    hipLaunchKernelGGL(cut_keys, dim3(grid_of(m)), dim3(kBlk), 0, st, g->col, erow, m, lo, hi, d_plo, P, rc, n_ghost,
                       skey, gkey, gcnt);
    GCHK(hipGetLastError());
    mem.release(erow);
    // send lists: unique (part, row), ascending
    uint64_t ns = 0;
    if (int r = sort_unique(skey, m, 64, st, &ns, err)) return r;
    std::vector<uint64_t> lastk(1, 0);
    if (ns) GCHK(hipMemcpyAsync(lastk.data(), skey + ns - 1, 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    if (ns && lastk[0] == ~0ull) --ns;
    unsigned long long* scnt = nullptr;
    GCHK(mem.alloc(&scnt, (P + 1) * 8));
    GCHK(hipMemsetAsync(scnt, 0, (P + 1) * 8, st));
    hipLaunchKernelGGL(send_counts, dim3(grid_of(ns)), dim3(kBlk), 0, st, skey, ns, scnt);
    GCHK(hipGetLastError());
    std::vector<unsigned long long> sc(P + 1);
    GCHK(hipMemcpyAsync(sc.data(), scnt, (P + 1) * 8, hipMemcpyDeviceToHost, st));  // the stream is non-blocking:
    GCHK(hipStreamSynchronize(st));                                                 // copies go on it, then wait
    out->send_off.assign(P + 1, 0);
    for (uint32_t q = 0; q < P; ++q) out->send_off[q + 1] = out->send_off[q] + sc[q];
    GCHK(mem.alloc(&out->send_idx, ns * 4));
    hipLaunchKernelGGL(low_words, dim3(grid_of(ns)), dim3(kBlk), 0, st, skey, ns, out->send_idx);
    GCHK(hipGetLastError());
    out->n_send = ns;
    mem.release(skey);
    // ghost -> owned lists: ghost keys sorted (every cut edge once)
    if (int r = sort_unique<uint64_t>(gkey, m, 64, st, nullptr, err)) return r;
    uint64_t n_cut = 0;
    {
        // the cut edges are the keys before the ~0 tail: their count = sum of gcnt
        GCHK(mem.alloc(&out->gout_ptr, (n_ghost + 1) * 8));
        size_t tb = 0;
        void* tmp = nullptr;
        GCHK(rocprim::exclusive_scan(nullptr, tb, (int64_t*)gcnt, out->gout_ptr, (int64_t)0, n_ghost + 1,
                                     rocprim::plus<int64_t>(), st));
        GCHK(mem.alloc(&tmp, tb));
        GCHK(rocprim::exclusive_scan(tmp, tb, (int64_t*)gcnt, out->gout_ptr, (int64_t)0, n_ghost + 1,
                                     rocprim::plus<int64_t>(), st));
        int64_t h = 0;
        GCHK(hipMemcpyAsync(&h, out->gout_ptr + n_ghost, 8, hipMemcpyDeviceToHost, st));
        GCHK(hipStreamSynchronize(st));
        mem.release(tmp);
        n_cut = (uint64_t)h;
    }
    uint64_t* d_roff = nullptr;
    uint64_t* d_soff = nullptr;
    GCHK(mem.alloc(&d_roff, (P + 1) * 8));
    GCHK(mem.alloc(&d_soff, (P + 1) * 8));
    GCHK(hipMemcpyAsync(d_roff, out->recv_off.data(), (P + 1) * 8, hipMemcpyHostToDevice, st));
    GCHK(hipMemcpyAsync(d_soff, out->send_off.data(), (P + 1) * 8, hipMemcpyHostToDevice, st));
    GCHK(mem.alloc(&out->gout_col, n_cut * 4));
    GCHK(mem.alloc(&out->gout_sidx, n_cut * 4));
    hipLaunchKernelGGL(ghost_lists, dim3(grid_of(n_cut)), dim3(kBlk), 0, st, gkey, n_cut, d_roff, d_soff, P,
                       out->send_idx, out->gout_col, out->gout_sidx);
    GCHK(hipGetLastError());
    out->n_cut = n_cut;
    // columns -> local rows, and the row -> node map
    hipLaunchKernelGGL(remap_cols, dim3(grid_of(m)), dim3(kBlk), 0, st, g->col, m, lo, hi, rc, n_ghost, ghost0, col_or);
    GCHK(hipGetLastError());
    const uint64_t rows = std::max<uint64_t>(64, (ghost0 + n_ghost + 63) / 64 * 64);
    GCHK(mem.alloc(&out->gid, rows * 4));
    hipLaunchKernelGGL(fill_gid, dim3(grid_of(rows)), dim3(kBlk), 0, st, rows, lo, n, ghost0, rc, n_ghost, out->gid);
    GCHK(hipGetLastError());
    unsigned long long* d_bad = nullptr;
    GCHK(mem.alloc(&d_bad, 8));
    GCHK(hipMemsetAsync(d_bad, 0, 8, st));
    hipLaunchKernelGGL(check_shard, dim3(std::min(grid_of(m), 4096u)), dim3(kBlk), 0, st, g->row_ptr, n, g->col, m,
                       ghost0, n_ghost, out->send_idx, ns, out->gout_ptr, out->gout_col, out->gout_sidx, n_cut, d_bad);
    GCHK(hipGetLastError());
    unsigned long long bad = 0;
    GCHK(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    if (bad || out->send_off[P] != ns) {
        *err = "shard_csr: " + std::to_string(bad) + " inconsistent indices";
        return -5;
    }
    mem.keep(out->send_idx);
    mem.keep(out->gout_ptr);
    mem.keep(out->gout_col);
    mem.keep(out->gout_sidx);
    mem.keep(out->gid);
    return 0;
}

}  // namespace gg_gen
