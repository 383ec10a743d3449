// expand_kernels.hpp — the per-round gossip kernels for gfx950 (CDNA4).
//
// One launch of `expand_round` executes one lockstep round for every owned
// node: it is the device form of HandleBroadcast (`broadcast/broadcast.go:59-79`)
// + rebroadcastAllExcept (`:50-57`) + the SyncBroadcast callback (`:82-117`) +
// the sync timer (`broadcast/main.go:42-51`), in the determinized order of
// DESIGN.md §2 (client broadcasts, node broadcasts by ascending sender, read_ok
// callbacks by ascending peer, reads, timer).
//
// Work mapping: a node's set is nwp 64-bit words; a *node group*
// of G lanes owns one node, lane l holding words [l*WPL, l*WPL+WPL) (16-byte
// loads for WPL = 2), so one wave64 streams 64/G rows per instruction. Every
// bitwise step (claim = src & ~S, S |= claim, callback new/push) is lane-local;
// the sequential semantics (first deliverer claims, callbacks in peer order)
// are a loop over the CSR list inside the group, so no cross-lane reduction is
// needed on the hot path. Message counts are linear in per-lane popcounts and
// are summed per lane, reduced once per block, and added into one of 64 counter
// slots (64 x 16 u64) to keep atomic contention low.
//
// Memory-bound, no MFMA: per round it streams row_ptr, col, seen_prev, the
// gathered neighbour frontier rows, and writes seen_cur and F_cur.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gossip_spec.h"

namespace gg {

constexpr int kBlock = 256;
constexpr int kSlots = 64;     // counter slots
constexpr int kCounters = 16;  // per slot
constexpr uint32_t kColMask = 0x7fffffffu;
constexpr uint32_t kRecipBit = 0x80000000u;

enum Counter : int {
    C_NEW = 0, C_FWD_SENT, C_FWD_DELIV, C_PUSH, C_PUSH_DELIV, C_READS, C_READ_OKS,
    C_DROPPED, C_FIRED, C_HASH, C_NEXT_ACKS, C_NEXT_ACKDROP, C_NUM
};

struct RoundArgs {
    const int64_t* in_ptr;     // [n_own+1]
    const uint32_t* in_col;    // replica row of the sender | kRecipBit if sender in out(v)
    const int64_t* out_ptr;    // [n_own+1]
    const uint32_t* out_col;   // replica rows
    const uint64_t* seen_prev; // [rows][nwp]
    uint64_t* seen_cur;
    const uint64_t* F_prev;
    uint64_t* F_cur;
    const uint64_t* fired_m1;  // fired bitmaps of rounds r-1, r-2, r-3 (replica rows)
    const uint64_t* fired_m2;
    const uint64_t* fired_m3;
    uint64_t* fired_cur;       // round r (cleared before launch)
    int32_t* sync_next;        // [n_own]
    uint32_t* sync_k;
    const uint8_t* grp[5];     // partition groups of rounds r-3..r+1 (nullptr: no window)
    const uint32_t* inj;       // (local node, lane) pairs sorted by node
    uint32_t n_inj;
    unsigned long long* counters;  // [kSlots][kCounters]
    uint64_t n_own, own0, lo;
    uint32_t nwp, nw;
    int64_t round;
    uint64_t seed;
    uint32_t sync_base, sync_jitter;
    int32_t enable_sync;
};

template <int WPL>
struct Row {
    uint64_t w[WPL];
};

template <int WPL>
__device__ __forceinline__ Row<WPL> load_row(const uint64_t* p) {
    Row<WPL> r;
    if constexpr (WPL == 2) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p);
        r.w[0] = v.x;
        r.w[1] = v.y;
    } else {
#pragma unroll
        for (int k = 0; k < WPL; ++k) r.w[k] = p[k];
    }
    return r;
}

template <int WPL>
__device__ __forceinline__ void store_row(uint64_t* p, const Row<WPL>& r) {
    if constexpr (WPL == 2) {
        *reinterpret_cast<ulonglong2*>(p) = make_ulonglong2(r.w[0], r.w[1]);
    } else {
#pragma unroll
        for (int k = 0; k < WPL; ++k) p[k] = r.w[k];
    }
}

__device__ __forceinline__ bool bit_at(const uint64_t* bm, uint64_t row) {
    return (bm[row >> 6] >> (row & 63)) & 1ull;
}

// message from replica row a to replica row b in round (r-3+k) dropped?
template <bool MASKW>
__device__ __forceinline__ bool masked(const RoundArgs& a, int k, uint64_t ra, uint64_t rb) {
    if constexpr (!MASKW) {
        return false;
    } else {
        const uint8_t* g = a.grp[k];
        return g != nullptr && g[ra] != g[rb];
    }
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// One round. G lanes per node, WPL words per lane; SYNCW: sync events possible
// in r-3..r-1; MASKW: some partition window covers r-3..r+1.
template <int G, int WPL, bool SYNCW, bool MASKW>
__global__ __launch_bounds__(kBlock) void expand_round(RoundArgs a) {
    constexpr int kGroups = kBlock / G;
    constexpr int kUnroll = 4;
    const int lg = threadIdx.x % G;
    const uint64_t stride = (uint64_t)gridDim.x * kGroups;
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;

    for (uint64_t i = (uint64_t)blockIdx.x * kGroups + threadIdx.x / G; i < a.n_own; i += stride) {
        const uint64_t rep = a.own0 + i;
        const uint64_t off = (uint64_t)lg * WPL;
        const Row<WPL> sp = load_row<WPL>(a.seen_prev + rep * a.nwp + off);
        Row<WPL> S = sp;

        // (1) client broadcasts of this round (HandleBroadcast from a client)
        if (a.n_inj) {
            uint32_t lo = 0, hi = a.n_inj;
            while (lo < hi) {
                uint32_t mid = (lo + hi) >> 1;
                if (a.inj[2 * mid] < (uint32_t)i) lo = mid + 1;
                else hi = mid;
            }
            for (uint32_t k = lo; k < a.n_inj && a.inj[2 * k] == (uint32_t)i; ++k) {
                const uint32_t lane = a.inj[2 * k + 1];
                const uint32_t word = lane >> 6;
                if (word / WPL == (uint32_t)lg) S.w[word % WPL] |= 1ull << (lane & 63);
            }
        }

        // (2) node broadcasts, ascending sender: first deliverer claims
        unsigned long long cl_recip = 0, cl_deliv = 0, cl_ackdrop = 0, n_readok = 0, d_readok = 0;
        const int64_t e0 = a.in_ptr[i], e1 = a.in_ptr[i + 1];
        for (int64_t e = e0; e < e1; e += kUnroll) {
            uint32_t c[kUnroll];
            bool live[kUnroll];
            Row<WPL> src[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) {
                const bool valid = e + k < e1;
                c[k] = valid ? a.in_col[e + k] : 0u;
                const uint64_t u = c[k] & kColMask;
                bool drop = masked<MASKW>(a, 2, u, rep);  // sent in r-1
                bool push = false;
                if constexpr (SYNCW) {
                    if (valid && bit_at(a.fired_m1, u) && !drop) {  // u's read arrives now
                        n_readok++;
                        if (masked<MASKW>(a, 3, rep, u)) d_readok++;
                    }
                    push = bit_at(a.fired_m3, u) && !masked<MASKW>(a, 0, u, rep) &&
                           !masked<MASKW>(a, 1, rep, u);
                }
                live[k] = valid && !drop;
                const uint64_t* base = push ? a.seen_prev : a.F_prev;
                if (live[k]) {
                    src[k] = load_row<WPL>(base + u * a.nwp + off);
                } else {
#pragma unroll
                    for (int w = 0; w < WPL; ++w) src[k].w[w] = 0;
                }
            }
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) {
                unsigned long long pc = 0;
#pragma unroll
                for (int w = 0; w < WPL; ++w) {
                    const uint64_t claim = src[k].w[w] & ~S.w[w];
                    S.w[w] |= claim;
                    pc += __popcll(claim);
                }
                if (live[k] && (c[k] & kRecipBit)) {
                    cl_recip += pc;
                    const uint64_t u = c[k] & kColMask;
                    if (!masked<MASKW>(a, 3, rep, u)) {
                        cl_deliv += pc;
                        if (masked<MASKW>(a, 4, u, rep)) cl_ackdrop += pc;
                    }
                }
            }
        }

        // (3) sync callback: v fired in r-2, read_oks of peers in ascending order
        unsigned long long cb_new = 0, cb_new_deliv = 0, cb_new_ackdrop = 0;
        unsigned long long push_sent = 0, push_deliv = 0, push_ackdrop = 0;
        const int64_t o0 = a.out_ptr[i], o1 = a.out_ptr[i + 1];
        if constexpr (SYNCW) {
            if (bit_at(a.fired_m2, rep)) {
                for (int64_t e = o0; e < o1; ++e) {
                    const uint64_t w = a.out_col[e] & kColMask;
                    if (masked<MASKW>(a, 1, rep, w) || masked<MASKW>(a, 2, w, rep)) continue;
                    const Row<WPL> R = load_row<WPL>(a.seen_prev + w * a.nwp + off);
                    unsigned long long pn = 0, pp = 0;
#pragma unroll
                    for (int k = 0; k < WPL; ++k) {
                        pn += __popcll(R.w[k] & ~S.w[k]);
                        pp += __popcll(S.w[k] & ~R.w[k]);
                        S.w[k] |= R.w[k];
                    }
                    cb_new += pn;
                    push_sent += pp;
                    if (!masked<MASKW>(a, 3, rep, w)) {
                        cb_new_deliv += pn;
                        push_deliv += pp;
                        if (masked<MASKW>(a, 4, w, rep)) {
                            cb_new_ackdrop += pn;
                            push_ackdrop += pp;
                        }
                    }
                }
            }
        }

        // new state
        Row<WPL> F;
        unsigned long long T = 0;
        const uint64_t g = a.lo + i;
#pragma unroll
        for (int k = 0; k < WPL; ++k) {
            F.w[k] = S.w[k] & ~sp.w[k];
            T += __popcll(F.w[k]);
            if (S.w[k]) acc[C_HASH] += gg_word_hash(g * a.nw + off + k, S.w[k]);
        }
        store_row<WPL>(a.seen_cur + rep * a.nwp + off, S);
        store_row<WPL>(a.F_cur + rep * a.nwp + off, F);

        // messages v sends in round r (rebroadcastAllExcept :50-57, pushes :106)
        const unsigned long long deg = (unsigned long long)(o1 - o0);
        unsigned long long U = deg, AD = 0, mdrop = 0;
        if constexpr (MASKW) {
            if (a.grp[3] != nullptr || a.grp[4] != nullptr) {
                U = 0;
                for (int64_t e = o0; e < o1; ++e) {
                    const uint64_t w = a.out_col[e] & kColMask;
                    if (!masked<MASKW>(a, 3, rep, w)) {
                        U++;
                        if (masked<MASKW>(a, 4, w, rep)) AD++;
                    } else {
                        mdrop++;
                    }
                }
            }
        }
        const unsigned long long fs = deg * T - cl_recip - cb_new;
        const unsigned long long fd = U * T - cl_deliv - cb_new_deliv;
        acc[C_NEW] += T;
        acc[C_FWD_SENT] += fs;
        acc[C_FWD_DELIV] += fd;
        acc[C_PUSH] += push_sent;
        acc[C_PUSH_DELIV] += push_deliv;
        acc[C_DROPPED] += (fs - fd) + (push_sent - push_deliv);
        acc[C_NEXT_ACKS] += fd + push_deliv;
        acc[C_NEXT_ACKDROP] += AD * T - cl_ackdrop - cb_new_ackdrop + push_ackdrop;

        if (lg == 0) {  // node-uniform events, counted once per node
            acc[C_READ_OKS] += n_readok;
            acc[C_DROPPED] += d_readok;
            // (5) sync timer (main.go:42-51)
            if (a.enable_sync && (int64_t)a.sync_next[i] == a.round) {
                atomicOr((unsigned long long*)&a.fired_cur[rep >> 6], 1ull << (rep & 63));
                acc[C_FIRED] += 1;
                acc[C_READS] += deg;
                acc[C_DROPPED] += mdrop;
                const uint32_t k = a.sync_k[i] + 1;
                a.sync_k[i] = k;
                a.sync_next[i] = (int32_t)(a.round + gg_sync_interval(a.seed, g, k, a.sync_base,
                                                                      a.sync_jitter));
            }
        }
    }

    // block reduction -> one atomic per counter per block into slot blockIdx % 64
    __shared__ unsigned long long red[kBlock / 64][C_NUM];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) {
        const unsigned long long s = wave_sum(acc[k]);
        if (lane == 0) red[wave][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < C_NUM) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
        if (s) atomicAdd(&a.counters[(blockIdx.x % kSlots) * kCounters + threadIdx.x], s);
    }
}

// First-seen round of every new bit (GG_TRACK_DELIVERY only; observation).
__global__ void track_delivery(const uint64_t* F_cur, int32_t* dr, uint64_t n_own, uint64_t own0,
                               uint32_t nwp, uint32_t nw, uint32_t W, int32_t round) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_own * nw) return;
    const uint64_t i = t / nw, j = t % nw;
    uint64_t x = F_cur[(own0 + i) * nwp + j];
    while (x) {
        const int b = __builtin_ctzll(x);
        x &= x - 1;
        dr[i * W + j * 64 + b] = round;
    }
}

__global__ void sync_init(int32_t* sync_next, uint32_t* sync_k, uint64_t n_own, uint64_t lo,
                          uint64_t seed, uint32_t base, uint32_t jitter) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_own) return;
    sync_k[i] = 0;
    sync_next[i] = (int32_t)gg_sync_interval(seed, lo + i, 0, base, jitter);
}

// Seeded bisection groups in replica-row order (padding rows: group 0, unused).
__global__ void fill_seeded_groups(uint8_t* grp, uint64_t rows, uint64_t slice,
                                   const uint64_t* rank_lo, uint32_t world, uint64_t seed,
                                   uint64_t epoch_seed) {
    const uint64_t rr = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rr >= rows) return;
    const uint64_t p = rr / slice;
    const uint64_t g = rank_lo[p] + (rr - p * slice);
    grp[rr] = (p < world && g < rank_lo[p + 1]) ? (uint8_t)gg_part_group(seed, epoch_seed, g) : 0;
}

}  // namespace gg
