// expand_kernels.hpp — the per-round gossip kernels for gfx950 (CDNA4).
//
// One lockstep round is two launches:
//   round_prep   — one thread per node: the sync timer (`broadcast/main.go:42-51`,
//                  `SyncBroadcast` reads, `broadcast.go:119-121`), the read_oks
//                  that answer last round's reads (`HandleRead`, `:124-132`), and
//                  *candidate marking*: a node can change this round only if a
//                  sender of its in-list was active (or pushed) last round, it has
//                  a deferred fold (LAG), a sync callback, or a client broadcast;
//                  active senders mark their out-lists (single-engine mode).
//   expand_round — the device form of HandleBroadcast (`:59-79`) +
//                  rebroadcastAllExcept (`:50-57`) + the SyncBroadcast callback
//                  (`:82-117`) for every candidate node, in the determinized order
//                  of DESIGN.md §2 (client broadcasts, node broadcasts by ascending
//                  sender, read_ok callbacks by ascending peer).
//
// State: `base` holds every node's set *in place*; F[r&1] holds
// the bits a node learned in round r (what it forwards in r+1), valid only
// where flags[r&1] has ACT. A node whose set is read by a sync peer in round r
// (a read_ok payload or a push) keeps base = its round r-1 set and marks LAG;
// then its true set is base | F. So every reader computes
//     set(u) = base[u] | (LAG(u) ? F_prev[u] : 0)
// and idle nodes move no row.
//
// Work mapping of expand_round: the live tiles (NG = 256/G consecutive nodes
// with at least one candidate) are compacted into a worklist (compact_tiles)
// and dealt round-robin to blocks. For a live tile the CSR slice (row_ptr, col)
// is staged in LDS with coalesced loads in one round trip (the worklist entry
// carries the tile's edge range), plus per-sender flags unless the round is
// dense and lean (then flags and rows are gathered together); a *node group* of G lanes owns one node, lane l holding
// words [l*WPL, l*WPL+WPL) of its set (16-byte accesses for WPL = 2). Pass 1
// compacts the node's contributing senders in LDS; pass 2 gathers their rows 4
// at a time and runs the claim chain (first deliverer, ascending sender) in
// registers. Counters are linear in per-lane popcounts: summed per lane,
// reduced once per block, added to one of 64 counter slots.
//
// Memory-bound, no MFMA: HBM traffic per round is the active senders' rows,
// the changed nodes' base/F rows, and the CSR of candidate tiles.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gossip_spec.h"

namespace gg {

// Occupancy target of the lean round kernel (no sync events, no partition
// masks: the propagation phase): 4 blocks/CU, the LDS budget of its DMA landing slots.
#ifndef GG_LEAN_WAVES_PER_EU
#define GG_LEAN_WAVES_PER_EU 4
#endif

// Sender rows a lane keeps in flight (LDS slots) in expand_stream, and its occupancy.
#ifndef GG_STREAM_ROWS
#define GG_STREAM_ROWS 6
#endif
#ifndef GG_STREAM_WAVES_PER_EU
#define GG_STREAM_WAVES_PER_EU 6
#endif
constexpr int kStreamRows = GG_STREAM_ROWS;

// Sender (flag, row) pairs a lane keeps in flight in dense lean rounds.
#ifndef GG_SPEC_BATCH
#define GG_SPEC_BATCH 4
#endif

constexpr int kBlock = 256;
constexpr int kSlots = 64;       // counter slots
constexpr int kCounters = 16;    // per slot
constexpr int kEdgeStage = 2048; // in-edges staged in LDS per tile
constexpr uint32_t kColMask = 0x7fffffffu;
constexpr uint32_t kRecipBit = 0x80000000u;

// node flags (flags[r&1][row])
constexpr uint8_t FL_ACT = 1;  // F row of this round is valid and non-zero
constexpr uint8_t FL_LAG = 2;  // base lacks this round's F (set = base | F)
// staged per-sender flags
constexpr uint8_t SE_ACT = 1, SE_LAG = 2, SE_FM2 = 8, SE_FM3 = 16;
// candidate bytes
constexpr uint8_t CA_NODE = 1, CA_INJ = 2;

enum Counter : int {
    C_NEW = 0, C_FWD_SENT, C_FWD_DELIV, C_PUSH, C_PUSH_DELIV, C_READS, C_READ_OKS,
    C_DROPPED, C_FIRED, C_HASH, C_NEXT_ACKS, C_NEXT_ACKDROP, C_ACTIVE, C_GATHERS, C_NUM
};
// per-slot device clock stamps (s_memrealtime, 100 MHz): ~first block start
// (stored complemented, so a max of zero-initialised slots gives the min) and
// last block end of the round's kernels
constexpr int C_TSTART_INV = 14, C_TEND = 15;

__device__ __forceinline__ unsigned long long clock100() { return __builtin_amdgcn_s_memrealtime(); }

struct TileWork {
    uint32_t tile;   // tile index (nodes tile*NG ..)
    uint32_t ne;     // in-edges of the tile
    int64_t eb;      // in_ptr of the tile's first node
};

struct RoundArgs {
    const int64_t* in_ptr;      // [n_own+1]
    const uint32_t* in_col;     // replica row of the sender | kRecipBit if sender in out(v)
    const int64_t* out_ptr;     // [n_own+1]
    const uint32_t* out_col;    // replica rows (| kRecipBit when shared with in_col)
    uint64_t* base;             // [rows][nwp] node sets, in place
    const uint64_t* F_prev;     // [rows][nwp] new bits of round r-1 (valid where ACT)
    uint64_t* F_cur;
    const uint8_t* flg_prev;    // [rows] FL_* of round r-1
    uint8_t* flg_cur;
    uint8_t* cand;              // [rows] candidate bytes of this round (cleared by expand)
    uint8_t* zmark;             // [rows] F row of this parity is stale (node active 2 rounds ago)
    uint8_t* tile_cand;         // [n_tiles rounded to 8] tile has a candidate
    struct TileWork* work;      // live tiles of the round (compact_tiles)
    uint32_t* n_work;           // number of live tiles
    const uint64_t* fired_m1;   // sync-fired bitmaps of rounds r-1, r-2, r-3
    const uint64_t* fired_m2;
    const uint64_t* fired_m3;
    uint64_t* fired_cur;        // round r (written whole by round_prep)
    int32_t* sync_next;         // [n_own]
    uint32_t* sync_k;
    const uint8_t* grp[5];      // partition groups of rounds r-3..r+1 (nullptr: no window)
    const uint32_t* inj;        // (local node, lane) pairs sorted by node
    uint32_t n_inj;
    unsigned long long* counters;  // [kSlots][kCounters]
    uint64_t n_own, own0, lo;
    uint32_t nwp, nw;
    uint32_t tile_nodes;        // NG of the expand kernel
    int32_t symmetric;          // out-lists == in-lists
    uint64_t n_edges;           // in_col entries of this engine
    uint64_t rows;              // replica rows
    int32_t mark_all;           // sharded engines: every owned node is a candidate
    uint32_t ablate;            // DIAGNOSTIC timing builds only (GG_ABLATE): 1 no row stores,
                                // 2 no sender-row gathers, 4 no own-row loads, 8 no hash; results invalid
    int64_t round;
    uint64_t seed;
    uint32_t sync_base, sync_jitter;
    int32_t enable_sync;
};

template <int WPL>
struct Row {
    uint64_t w[WPL];
};

// S.w[w] |= bit b, with w a runtime value: selects, not a runtime-indexed
// register array (which would live in scratch).
template <int WPL>
__device__ __forceinline__ void set_lane_bit(Row<WPL>& S, uint32_t w, uint32_t b) {
#pragma unroll
    for (int q = 0; q < WPL; ++q)
        if ((uint32_t)q == w) S.w[q] |= 1ull << b;
}

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

// message from replica row ra to replica row rb in round (r-3+k) dropped?
template <bool MASKW>
__device__ __forceinline__ bool masked(const RoundArgs& a, int k, uint64_t ra, uint64_t rb) {
    if constexpr (!MASKW) {
        return false;
    } else {
        const uint8_t* g = a.grp[k];
        return g != nullptr && g[ra] != g[rb];
    }
}

template <bool SYNCW>
__device__ __forceinline__ uint8_t sender_flags(const RoundArgs& a, uint64_t u) {
    uint8_t f = a.flg_prev[u] & (FL_ACT | FL_LAG);
    if constexpr (SYNCW) {
        f |= (bit_at(a.fired_m2, u) ? SE_FM2 : 0) | (bit_at(a.fired_m3, u) ? SE_FM3 : 0);
    }
    return f;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt), not for its global stores/loads (vmcnt counts stores on CDNA, so
// __syncthreads() would stall every tile on the previous tile's row stores).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Push edge: u's sync callback of round r-1 pushed to v (u fired in r-3, its
// read reached v in r-3 and v's read_ok reached u in r-2), so v receives u's
// whole round r-1 set.
template <bool SYNCW, bool MASKW>
__device__ __forceinline__ bool is_push(const RoundArgs& a, uint8_t ef, uint64_t u, uint64_t v) {
    if constexpr (!SYNCW) {
        return false;
    } else {
        return (ef & SE_FM3) && !masked<MASKW>(a, 0, u, v) && !masked<MASKW>(a, 1, v, u);
    }
}

// Block reduction of C_NUM per-thread counters -> one atomic per counter per
// block into slot blockIdx % 64.
// Wait until every vector-memory op of this wave (loads, stores, LDS-DMA) is
// done: s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15). Issued through the builtin
// so the compiler's waitcnt pass sees it and does not add drains of its own
// for loads this wait already covers.
__device__ __forceinline__ void vm_drain() {
    __builtin_amdgcn_s_waitcnt(0x0F70);
    asm volatile("" ::: "memory");
}

// 16-byte LDS-DMA (global_load_lds_dwordx4): LDS destination = M0 (wave-uniform
// base) + lane * 16. Issued from inline asm because the compiler's waitcnt
// pass cannot tell one wave's DMA slots apart and puts a full vmcnt(0) drain
// in front of every builtin DMA, serialising them; callers wait themselves
// (s_waitcnt vmcnt(0)) before reading the slots. Extra vector-memory ops the
// compiler does not see only make its own vmcnt(N) waits stricter.
__device__ __forceinline__ void dma16(const void* src, const void* lds_wave_base) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds_wave_base);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0)
                 : "memory");
}

__device__ __forceinline__ void flush_counters(const RoundArgs& a, unsigned long long (&acc)[C_NUM],
                                               unsigned long long (*s_red)[C_NUM], unsigned long long t_start) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) {
        const unsigned long long s = wave_sum(acc[k]);
        if (lane == 0) s_red[wave][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < C_NUM) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += s_red[w][threadIdx.x];
        if (s) atomicAdd(&a.counters[(blockIdx.x % kSlots) * kCounters + threadIdx.x], s);
    }
    if (threadIdx.x == 0) {
        unsigned long long* slot = a.counters + (blockIdx.x % kSlots) * kCounters;
        atomicMax(slot + C_TSTART_INV, ~t_start);
        atomicMax(slot + C_TEND, clock100());
    }
}

// ---------------------------------------------------------------------------
// round_prep: one thread per owned node (64 consecutive nodes per wave, so a
// wave owns whole words of the fired bitmap).
template <bool SYNCW, bool MASKW>
__global__ __launch_bounds__(kBlock) void round_prep(RoundArgs a) {
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    unsigned long long c_reads = 0, c_read_oks = 0, c_dropped = 0, c_fired = 0;
    const uint64_t nwords = (a.n_own + 63) / 64;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.n_work = 0;  // compact_tiles runs after this kernel
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < nwords * 64; t += stride) {
        const uint64_t i = t;
        const bool valid = i < a.n_own;
        const uint64_t rep = a.own0 + i;
        bool fire = false;
        if (valid) {
            const uint8_t f = a.flg_prev[rep];
            // flg_cur still holds round r-2's flags: an F row written then is
            // stale in this round's F buffer; expand zeroes it unless the node
            // writes a new one, so F rows stay zero for inactive nodes.
            if (a.flg_cur[rep] & FL_ACT) {
                a.zmark[rep] = 1;
                a.tile_cand[i / a.tile_nodes] = 1;
            }
            a.flg_cur[rep] = 0;  // expand_round sets the flags of changed nodes
            const int64_t o0 = a.out_ptr[i], o1 = a.out_ptr[i + 1];
            bool fm1 = false, fm2 = false, fm3 = false;
            if constexpr (SYNCW) {
                fm1 = bit_at(a.fired_m1, rep);
                fm2 = bit_at(a.fired_m2, rep);
                fm3 = bit_at(a.fired_m3, rep);
            }
            // candidates of this round
            if (a.mark_all || (f & FL_LAG) || fm2) {
                a.cand[rep] = CA_NODE;
                a.tile_cand[i / a.tile_nodes] = 1;
            }
            if (!a.mark_all && ((f & FL_ACT) || fm3)) {  // senders mark their receivers
                for (int64_t e = o0; e < o1; ++e) {
                    const uint64_t w = a.out_col[e] & kColMask;  // single engine: w == local row
                    a.cand[w] = CA_NODE;
                    a.tile_cand[(w - a.own0) / a.tile_nodes] = 1;
                }
            }
            if constexpr (SYNCW) {
                // reads v sent in r-1 arrive now; each answered by a read_ok (:131)
                if (fm1) {
                    for (int64_t e = o0; e < o1; ++e) {
                        const uint64_t w = a.out_col[e] & kColMask;
                        if (masked<MASKW>(a, 2, rep, w)) continue;
                        c_read_oks++;
                        if (masked<MASKW>(a, 3, w, rep)) c_dropped++;
                    }
                }
                // (5) the sync timer (main.go:42-51): read RPC to every neighbour (:119-121)
                if ((int64_t)a.sync_next[i] == a.round) {
                    fire = true;
                    c_fired++;
                    c_reads += (unsigned long long)(o1 - o0);
                    if constexpr (MASKW) {
                        for (int64_t e = o0; e < o1; ++e)
                            c_dropped += masked<MASKW>(a, 3, rep, a.out_col[e] & kColMask) ? 1 : 0;
                    }
                    const uint32_t kk = a.sync_k[i] + 1;
                    a.sync_k[i] = kk;
                    a.sync_next[i] = (int32_t)(a.round + gg_sync_interval(a.seed, a.lo + i, kk,
                                                                          a.sync_base, a.sync_jitter));
                }
            }
        }
        const unsigned long long word = __ballot(fire);
        if ((threadIdx.x & 63) == 0) a.fired_cur[(a.own0 + (i & ~63ull)) >> 6] = word;
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_READS] = c_reads;
    acc[C_READ_OKS] = c_read_oks;
    acc[C_DROPPED] = c_dropped;
    acc[C_FIRED] = c_fired;
    flush_counters(a, acc, s_red, t_start);
}

// Client broadcasts of this round mark their nodes (after round_prep).
__global__ void mark_injections(RoundArgs a) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_inj) return;
    const uint64_t i = a.inj[2 * k];
    a.cand[a.own0 + i] = CA_NODE | CA_INJ;
    a.tile_cand[i / a.tile_nodes] = 1;
}

// Live tiles -> worklist (order irrelevant: tiles are independent and counters
// are sums). 8 tile flags per thread; clears the flags for the next round.
__global__ __launch_bounds__(kBlock) void compact_tiles(RoundArgs a) {
    __shared__ uint32_t s_cnt[kBlock / 64];
    __shared__ uint32_t s_base;
    const uint64_t ntiles = (a.n_own + a.tile_nodes - 1) / a.tile_nodes;
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;  // 8-tile group
    unsigned long long tb = 0;
    if (q * 8 < ntiles) {
        tb = *reinterpret_cast<const unsigned long long*>(a.tile_cand + q * 8);
        if (tb) *reinterpret_cast<unsigned long long*>(a.tile_cand + q * 8) = 0ull;
    }
    uint32_t c = 0;
    for (int t = 0; t < 8; ++t) c += ((tb >> (8 * t)) & 0xff) ? 1u : 0u;
    // block exclusive scan of c
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_cnt[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const uint32_t x = s_cnt[w];
            s_cnt[w] = tot;
            tot += x;
        }
        s_base = tot ? atomicAdd(a.n_work, tot) : 0u;
    }
    __syncthreads();
    uint32_t pos = s_base + s_cnt[wave] + incl - c;
    for (int t = 0; t < 8; ++t) {
        if (!((tb >> (8 * t)) & 0xff)) continue;
        const uint64_t tile = q * 8 + t;
        const uint64_t n0 = tile * a.tile_nodes;
        const uint64_t n1 = n0 + a.tile_nodes < a.n_own ? n0 + a.tile_nodes : a.n_own;
        TileWork w;
        w.tile = (uint32_t)tile;
        w.eb = a.in_ptr[n0];
        w.ne = (uint32_t)(a.in_ptr[n1] - w.eb);
        a.work[pos++] = w;
    }
}

// ---------------------------------------------------------------------------
// expand_round. G lanes per node, WPL words per lane; SYNCW: sync events
// possible in r-3..r (timers fire from r >= sync_base); MASKW: some partition
// window covers r-3..r+1.
template <int G, int WPL, bool SYNCW, bool MASKW>
__device__ __forceinline__ void expand_body(const RoundArgs& a) {
    constexpr int NG = kBlock / G;  // nodes per tile
    constexpr int kBatch = 4;       // flags-first: contributing rows in flight per lane
    constexpr int kSpec = GG_SPEC_BATCH;  // dense lean rounds: (flag, row) pairs in flight per lane
    constexpr int kPre = 64;        // worklist entries preloaded per chunk
    constexpr bool LEAN = !SYNCW && !MASKW;
    constexpr int kDmaRows = 6;     // dense lean rounds: sender rows in flight per lane (via LDS)
    constexpr uint8_t L_PUSH = 1, L_LAG = 2;  // compacted-list flags
    // per-wave LDS landing slots of the dense lean path (kDmaRows x 1 KiB per wave)
    __shared__ __attribute__((aligned(16))) uint8_t s_rows[(LEAN && WPL == 2) ? 4 * kDmaRows * 1024 : 16];
    __shared__ int64_t s_ptr[NG + 1];
    __shared__ uint32_t s_col[kEdgeStage];
    __shared__ uint8_t s_ef[kEdgeStage];
    __shared__ TileWork s_work[kPre];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];

    const int j = threadIdx.x / G;
    const int lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    const unsigned long long t_start = clock100();
    // always-live counters
    unsigned long long c_new = 0, c_fwd = 0, c_hash = 0, c_active = 0, c_gathers = 0;
    // MASKW-only
    unsigned long long c_fwd_deliv = 0, c_push_deliv = 0, c_dropped = 0, c_next_ackdrop = 0;
    // SYNCW-only
    unsigned long long c_push = 0;

    const uint64_t n_work = *a.n_work;
    const uint64_t ntiles = (a.n_own + NG - 1) / NG;
    // most tiles live: load sender flags together with their rows (speculative
    // gathers; a row of an inactive sender is ignored) instead of flags first
    const bool dense = LEAN && n_work * 2 > ntiles;
    if constexpr (LEAN && WPL == 2) {
        if (dense) {  // expand_stream runs this round
            unsigned long long acc[C_NUM];
#pragma unroll
            for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
            flush_counters(a, acc, s_red, t_start);
            return;
        }
    }

    for (uint64_t base = blockIdx.x; base < n_work; base += (uint64_t)kPre * gridDim.x) {
        if (threadIdx.x < kPre) {
            const uint64_t idx = base + (uint64_t)threadIdx.x * gridDim.x;
            if (idx < n_work) s_work[threadIdx.x] = a.work[idx];
        }
        lds_barrier();
        for (int q = 0; q < kPre; ++q) {
            if (base + (uint64_t)q * gridDim.x >= n_work) break;  // block-uniform
            const TileWork tw = s_work[q];
            const uint64_t t0 = (uint64_t)tw.tile * NG;
            const int64_t eb = tw.eb;
            const int ns = tw.ne < (uint32_t)kEdgeStage ? (int)tw.ne : kEdgeStage;
            const uint64_t i = t0 + j;
            const uint64_t rep = a.own0 + i;
            // per-node bytes, issued with the staging loads (same round trip)
            const uint8_t ca = i < a.n_own ? a.cand[rep] : 0;
            const uint8_t zm = i < a.n_own ? a.zmark[rep] : 0;
            const uint8_t own = i < a.n_own ? a.flg_prev[rep] : 0;
            // ---- stage the tile's row_ptr and col slices (one round trip)
            for (int t = threadIdx.x; t <= NG; t += kBlock) {  // NG + 1 entries (NG may be kBlock)
                const uint64_t idx = t0 + t < a.n_own ? t0 + t : a.n_own;
                s_ptr[t] = a.in_ptr[idx];
            }
            for (int k = threadIdx.x; k < ns; k += kBlock) {
                const uint32_t c = a.in_col[eb + k];
                s_col[k] = c;
                if (!dense) s_ef[k] = sender_flags<SYNCW>(a, c & kColMask);
            }
            lds_barrier();

            if (zm && !ca) {  // only the stale F row to clear
                if (!(a.ablate & 1)) {
                    Row<WPL> z;
#pragma unroll
                    for (int w = 0; w < WPL; ++w) z.w[w] = 0;
                    store_row<WPL>(a.F_cur + rep * a.nwp + off, z);
                }
                if (lg == 0) a.zmark[rep] = 0;
            }
            if (ca) {
                if (lg == 0) a.cand[rep] = 0;
                const int64_t k0 = s_ptr[j] - eb, k1 = s_ptr[j + 1] - eb;
                const bool staged = k1 <= ns;  // else: hub slow path straight from global
                const bool lag = own & FL_LAG;
                const bool has_inj = (ca & CA_INJ) != 0;
                bool callback = false, keep = false;
                if constexpr (SYNCW) {
                    callback = bit_at(a.fired_m2, rep);
                    keep = bit_at(a.fired_m3, rep);  // v pushed in r-1: its set is read now
                }
                Row<WPL> sp, S;
                unsigned long long cl_recip = 0, cl_deliv = 0, cl_ackdrop = 0;
                unsigned long long cb_new = 0, cb_new_deliv = 0, cb_new_ackdrop = 0;
                unsigned long long push_sent = 0, push_deliv = 0, push_ackdrop = 0;
                auto load_own = [&]() {
                    if (a.ablate & 4) {
#pragma unroll
                        for (int w = 0; w < WPL; ++w) sp.w[w] = 0;
                    } else {
                        sp = load_row<WPL>(a.base + rep * a.nwp + off);
                    }
                    if (lag) {
                        const Row<WPL> f = load_row<WPL>(a.F_prev + rep * a.nwp + off);
#pragma unroll
                        for (int w = 0; w < WPL; ++w) sp.w[w] |= f.w[w];
                    }
                    S = sp;
                    // (1) client broadcasts of this round
                    if (has_inj) {
                        uint32_t lo = 0, hi = a.n_inj;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (a.inj[2 * mid] < (uint32_t)i) lo = mid + 1;
                            else hi = mid;
                        }
                        for (uint32_t k = lo; k < a.n_inj && a.inj[2 * k] == (uint32_t)i; ++k) {
                            const uint32_t lane = a.inj[2 * k + 1];
                            const uint32_t word = lane >> 6;
                            if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
                        }
                    }
                };
                // (2) first deliverer claims, ascending sender
                auto claim = [&](const Row<WPL>& src, uint32_t c) {
                    unsigned long long pc = 0;
#pragma unroll
                    for (int w = 0; w < WPL; ++w) {
                        const uint64_t cw = src.w[w] & ~S.w[w];
                        S.w[w] |= cw;
                        pc += __popcll(cw);
                    }
                    if (c & kRecipBit) {
                        cl_recip += pc;
                        if constexpr (MASKW) {
                            const uint64_t u = c & kColMask;
                            if (!masked<MASKW>(a, 3, rep, u)) {
                                cl_deliv += pc;
                                if (masked<MASKW>(a, 4, u, rep)) cl_ackdrop += pc;
                            }
                        }
                    }
                };
                auto sender_row = [&](uint32_t c, bool push, bool slag) {
                    const uint64_t u = c & kColMask;
                    if (SYNCW && push) {  // push edge: u's whole set of round r-1
                        Row<WPL> r = load_row<WPL>(a.base + u * a.nwp + off);
                        if (slag) {
                            const Row<WPL> f = load_row<WPL>(a.F_prev + u * a.nwp + off);
#pragma unroll
                            for (int w = 0; w < WPL; ++w) r.w[w] |= f.w[w];
                        }
                        return r;
                    }
                    return load_row<WPL>(a.F_prev + u * a.nwp + off);
                };
                bool work = true;
                if (dense) {
                    // ---- lean dense path: own row + (flag, row) of every sender.
                    load_own();
                    if constexpr (WPL == 2) {
                        // Each lane DMAs its own 16-byte chunk of kDmaRows sender rows
                        // into its wave's LDS slots (global_load_lds_dwordx4: LDS
                        // address = wave-uniform base + lane*16), waits vmcnt, and
                        // reads back exactly what it loaded: in-flight rows cost
                        // LDS, not VGPRs, and no other wave touches the slots.
                        uint8_t* const my = &s_rows[(threadIdx.x >> 6) * kDmaRows * 1024];
                        const uint32_t lane16 = (threadIdx.x & 63) * 16;
                        for (int64_t k = k0; k < k1; k += kDmaRows) {
                            uint32_t cb[kDmaRows];
#pragma unroll
                            for (int b = 0; b < kDmaRows; ++b) {
                                const bool v = k + b < k1;
                                cb[b] = v ? (k + b < ns ? s_col[k + b] : a.in_col[eb + k + b]) : 0u;
                                const uint64_t u = cb[b] & kColMask;
                                if (v && !(a.ablate & 2))
                                    dma16((const void*)(a.F_prev + u * a.nwp + off), my + b * 1024);
                            }
                            vm_drain();
                            // F rows of inactive senders are zero: claim every row
#pragma unroll
                            for (int b = 0; b < kDmaRows; ++b) {
                                if (k + b < k1) {
                                    const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(my + b * 1024 + lane16);
                                    Row<WPL> src;
                                    src.w[0] = x.x;
                                    src.w[1 % WPL] = x.y;
                                    claim(src, cb[b]);
                                    c_gathers += (lg == 0) ? 1ull : 0ull;
                                }
                            }
                        }
                    } else {
                        for (int64_t k = k0; k < k1; k += kSpec) {
                            uint32_t cb[kSpec];
                            uint8_t fb[kSpec];
                            Row<WPL> src[kSpec];
#pragma unroll
                            for (int b = 0; b < kSpec; ++b) {
                                const bool v = k + b < k1;
                                cb[b] = v ? (k + b < ns ? s_col[k + b] : a.in_col[eb + k + b]) : 0u;
                                const uint64_t u = cb[b] & kColMask;
                                fb[b] = v ? a.flg_prev[u] : (uint8_t)0;
                                if (v) {
                                    src[b] = load_row<WPL>(a.F_prev + u * a.nwp + off);
                                } else {
#pragma unroll
                                    for (int w = 0; w < WPL; ++w) src[b].w[w] = 0;
                                }
                            }
#pragma unroll
                            for (int b = 0; b < kSpec; ++b) {
                                if (fb[b] & FL_ACT) {
                                    claim(src[b], cb[b]);
                                    c_gathers += (lg == 0) ? 1ull : 0ull;
                                }
                            }
                        }
                    }
                } else {
                    // ---- pass 1: who reaches v this round (no row traffic); compact the
                    // contributing senders of a staged node in place in LDS.
                    int m = 0;
                    bool need = false;
                    for (int64_t k = k0; k < k1; ++k) {
                        uint32_t c;
                        uint8_t ef;
                        if (staged) {
                            c = s_col[k];
                            ef = s_ef[k];
                        } else {
                            c = a.in_col[eb + k];
                            ef = sender_flags<SYNCW>(a, c & kColMask);
                        }
                        const uint64_t u = c & kColMask;
                        const bool drop = masked<MASKW>(a, 2, u, rep);  // sent in r-1
                        if constexpr (SYNCW) keep |= (ef & SE_FM2) != 0;  // u's callback reads v now
                        const bool p = !drop && is_push<SYNCW, MASKW>(a, ef, u, rep);
                        if (!drop && ((ef & SE_ACT) || p)) {
                            need = true;
                            if (staged) {  // every lane of the group writes the same entry
                                s_col[k0 + m] = c;
                                s_ef[k0 + m] = (p ? L_PUSH : 0) | ((ef & SE_LAG) ? L_LAG : 0);
                                ++m;
                            }
                        }
                    }
                    work = need || lag || callback || has_inj;
                    if (work) {
                        // ---- pass 2: gather the contributing senders' rows
                        load_own();
                        if (staged) {
                            c_gathers += (lg == 0) ? (unsigned long long)m : 0ull;
                            for (int b0 = 0; b0 < m; b0 += kBatch) {
                                uint32_t cb[kBatch];
                                Row<WPL> src[kBatch];
#pragma unroll
                                for (int b = 0; b < kBatch; ++b) {
                                    const bool v = b0 + b < m;
                                    cb[b] = v ? s_col[k0 + b0 + b] : 0u;
                                    const uint8_t lf = v ? s_ef[k0 + b0 + b] : 0;
                                    if (v) {
                                        src[b] = sender_row(cb[b], lf & L_PUSH, lf & L_LAG);
                                    } else {
#pragma unroll
                                        for (int w = 0; w < WPL; ++w) src[b].w[w] = 0;
                                    }
                                }
#pragma unroll
                                for (int b = 0; b < kBatch; ++b) claim(src[b], cb[b]);
                            }
                        } else {
                            for (int64_t k = k0; k < k1; ++k) {  // hub slow path
                                const uint32_t c = a.in_col[eb + k];
                                const uint64_t u = c & kColMask;
                                const uint8_t ef = sender_flags<SYNCW>(a, u);
                                if (masked<MASKW>(a, 2, u, rep)) continue;
                                const bool p = is_push<SYNCW, MASKW>(a, ef, u, rep);
                                if (!(ef & SE_ACT) && !p) continue;
                                c_gathers += (lg == 0) ? 1ull : 0ull;
                                claim(sender_row(c, p, (ef & SE_LAG) != 0), c);
                            }
                        }
                        // (3) sync callback: v fired in r-2, read_oks of peers in ascending order
                        if constexpr (SYNCW) {
                            if (callback) {
                                const int64_t o0 = a.out_ptr[i], o1 = a.out_ptr[i + 1];
                                for (int64_t e = o0; e < o1; ++e) {
                                    const uint64_t w = a.out_col[e] & kColMask;
                                    if (masked<MASKW>(a, 1, rep, w) || masked<MASKW>(a, 2, w, rep)) continue;
                                    const Row<WPL> R =
                                        sender_row((uint32_t)w, true, (a.flg_prev[w] & FL_LAG) != 0);
                                    unsigned long long pn = 0, pp = 0;
#pragma unroll
                                    for (int q2 = 0; q2 < WPL; ++q2) {
                                        pn += __popcll(R.w[q2] & ~S.w[q2]);
                                        pp += __popcll(S.w[q2] & ~R.w[q2]);
                                        S.w[q2] |= R.w[q2];
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
                    }
                }
                if (work) {
                    const unsigned long long deg = (unsigned long long)(a.out_ptr[i + 1] - a.out_ptr[i]);
                    // ---- new state
                    Row<WPL> F;
                    unsigned long long T = 0;
                    const uint64_t g = a.lo + i;
#pragma unroll
                    for (int w = 0; w < WPL; ++w) {
                        F.w[w] = S.w[w] & ~sp.w[w];
                        T += __popcll(F.w[w]);
                        if (F.w[w] && !(a.ablate & 8)) {  // seen_hash delta of a changed word
                            const uint64_t idx = g * a.nw + off + w;
                            c_hash += gg_word_hash(idx, S.w[w]) - (sp.w[w] ? gg_word_hash(idx, sp.w[w]) : 0ull);
                        }
                    }
                    const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
                    if ((any || zm) && !(a.ablate & 1)) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
                    if (zm && lg == 0) a.zmark[rep] = 0;
                    if (a.ablate & 1) {
                    } else if (keep) {
                        if (lag) store_row<WPL>(a.base + rep * a.nwp + off, sp);
                    } else if (any || lag) {
                        store_row<WPL>(a.base + rep * a.nwp + off, S);
                    }
                    if (lg == 0 && any) a.flg_cur[rep] = (uint8_t)(FL_ACT | (keep ? FL_LAG : 0));

                    // messages v sends in round r (rebroadcastAllExcept :50-57, pushes :106)
                    const unsigned long long fs = deg * T - cl_recip - cb_new;
                    c_new += T;
                    c_fwd += fs;
                    c_active += (lg == 0) ? 1ull : 0ull;
                    if constexpr (SYNCW) c_push += push_sent;
                    if constexpr (MASKW) {
                        unsigned long long U = deg, AD = 0;
                        if (a.grp[3] != nullptr || a.grp[4] != nullptr) {
                            U = 0;
                            for (int64_t e = a.out_ptr[i]; e < a.out_ptr[i + 1]; ++e) {
                                const uint64_t w = a.out_col[e] & kColMask;
                                if (!masked<MASKW>(a, 3, rep, w)) {
                                    U++;
                                    if (masked<MASKW>(a, 4, w, rep)) AD++;
                                }
                            }
                        }
                        const unsigned long long fd = U * T - cl_deliv - cb_new_deliv;
                        c_fwd_deliv += fd;
                        c_push_deliv += push_deliv;
                        c_dropped += (fs - fd) + (push_sent - push_deliv);
                        c_next_ackdrop += AD * T - cl_ackdrop - cb_new_ackdrop + push_ackdrop;
                    }
                }
            }
            lds_barrier();  // LDS reuse by the next tile
        }
        lds_barrier();  // s_work reuse
    }

    // without partition masks nothing is dropped: delivered = sent
    if constexpr (!MASKW) {
        c_fwd_deliv = c_fwd;
        c_push_deliv = c_push;
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_fwd;
    acc[C_FWD_DELIV] = c_fwd_deliv;
    acc[C_PUSH] = c_push;
    acc[C_PUSH_DELIV] = c_push_deliv;
    acc[C_DROPPED] = c_dropped;
    acc[C_HASH] = c_hash;
    acc[C_NEXT_ACKS] = c_fwd_deliv + c_push_deliv;
    acc[C_NEXT_ACKDROP] = c_next_ackdrop;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers;
    flush_counters(a, acc, s_red, t_start);
}

template <int G, int WPL, bool SYNCW, bool MASKW>
__global__ __launch_bounds__(kBlock) void expand_round(RoundArgs a) {
    expand_body<G, WPL, SYNCW, MASKW>(a);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_LEAN_WAVES_PER_EU)))
void expand_round_lean(RoundArgs a) {
    expand_body<G, WPL, false, false>(a);
}


// ---------------------------------------------------------------------------
// expand_stream: the dense propagation round (no sync events, no masks, most
// tiles live). No tiles, no barriers: node group q (G lanes) walks nodes
// q, q + n_groups, ... with a software pipeline — while node i's own row and
// sender rows land in its wave's LDS slots by DMA, node i+1's column list and
// node i+2's row pointers and bytes are already in flight — so each node
// costs about one memory round trip. F rows of inactive senders are zero, so
// every sender row is claimed without looking at sender flags.
template <int G, int WPL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_STREAM_WAVES_PER_EU)))
void expand_stream(RoundArgs a) {
    static_assert(WPL == 2, "DMA slots hold 16 bytes per lane");
    constexpr int NGB = kBlock / G;  // node groups per block
    constexpr int D = kStreamRows;   // sender rows per DMA batch
    __shared__ __attribute__((aligned(16))) uint8_t s_slots[(kBlock / 64) * (D + 1) * 1024];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    unsigned long long c_new = 0, c_fwd = 0, c_hash = 0, c_active = 0, c_gathers = 0;

    const uint64_t n_work = *a.n_work;
    const uint64_t ntiles = (a.n_own + a.tile_nodes - 1) / a.tile_nodes;
    if (n_work * 2 > ntiles) {
        const int lg = threadIdx.x % G;
        const uint64_t off = (uint64_t)lg * WPL;
        const int gshift = (threadIdx.x & 63) / G * G;
        const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
        uint8_t* const my = &s_slots[(threadIdx.x >> 6) * (D + 1) * 1024];
        const uint32_t lane16 = (threadIdx.x & 63) * 16;
        const uint64_t stride = (uint64_t)gridDim.x * NGB;

        struct Meta {
            int64_t p0, p1;
            uint8_t ca, zm;
        };
        auto fetch_meta = [&](uint64_t n, Meta& m) {
            if (n < a.n_own && (a.ablate & 64)) {  // diagnostic: synthetic metadata
                m.p0 = 2 * n;
                m.p1 = 2 * n + 2;
                m.ca = CA_NODE;
                m.zm = 0;
            } else if (n < a.n_own) {
                m.p0 = a.in_ptr[n];
                m.p1 = a.in_ptr[n + 1];
                m.ca = a.cand[a.own0 + n];
                m.zm = a.zmark[a.own0 + n];
            } else {
                m.p0 = m.p1 = 0;
                m.ca = m.zm = 0;
            }
        };
        auto fetch_cols = [&](const Meta& m, uint32_t (&c)[D]) {
#pragma unroll
            for (int b = 0; b < D; ++b)
                c[b] = (m.ca && m.p0 + b < m.p1) ? ((a.ablate & 32) ? (uint32_t)((m.p0 + b) / 2) : a.in_col[m.p0 + b])
                                                 : 0u;
        };

        uint64_t i = (uint64_t)blockIdx.x * NGB + threadIdx.x / G;
        Meta m0, m1;
        uint32_t c0[D], c1[D];
        fetch_meta(i, m0);
        fetch_cols(m0, c0);
        fetch_meta(i + stride, m1);
        vm_drain();  // nothing pending at the loop head: no compiler drains inside
        for (; i < a.n_own; i += stride) {
            const uint64_t rep = a.own0 + i;
            const bool work = m0.ca != 0;
            // (a) DMA node i's own row and its first D sender rows
            if (work) {
                if (!(a.ablate & 4))
                    dma16((const void*)(a.base + rep * a.nwp + off), my + D * 1024);
#pragma unroll
                for (int b = 0; b < D; ++b) {
                    if (m0.p0 + b < m0.p1 && !(a.ablate & 2))
                        dma16((const void*)(a.F_prev + (uint64_t)(c0[b] & kColMask) * a.nwp + off), my + b * 1024);
                }
            }
            // (b) prefetch: columns of node i+stride, row pointers of node i+2*stride
            Meta m2;
            fetch_cols(m1, c1);
            fetch_meta(i + 2 * stride, m2);
            vm_drain();
            if (work) {
                const bool lag = false;  // lean rounds precede every sync timer: no LAG
                (void)lag;
                const ulonglong2 o = *reinterpret_cast<const ulonglong2*>(my + D * 1024 + lane16);
                Row<WPL> sp, S;
                sp.w[0] = o.x;
                sp.w[1] = o.y;
                S = sp;
                if (m0.ca & CA_INJ) {  // (1) client broadcasts of this round
                    uint32_t lo = 0, hi = a.n_inj;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (a.inj[2 * mid] < (uint32_t)i) lo = mid + 1;
                        else hi = mid;
                    }
                    for (uint32_t k = lo; k < a.n_inj && a.inj[2 * k] == (uint32_t)i; ++k) {
                        const uint32_t lane = a.inj[2 * k + 1];
                        const uint32_t word = lane >> 6;
                        if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
                    }
                }
                // (2) node broadcasts, ascending sender: first deliverer claims
                unsigned long long cl_recip = 0;
                auto claim = [&](uint64_t x0, uint64_t x1, uint32_t c) {
                    const uint64_t w0 = x0 & ~S.w[0], w1 = x1 & ~S.w[1];
                    S.w[0] |= w0;
                    S.w[1] |= w1;
                    if (c & kRecipBit) cl_recip += __popcll(w0) + __popcll(w1);
                };
#pragma unroll
                for (int b = 0; b < D; ++b) {
                    if (m0.p0 + b < m0.p1) {
                        const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(my + b * 1024 + lane16);
                        claim(x.x, x.y, c0[b]);
                    }
                }
                for (int64_t k = m0.p0 + D; k < m0.p1; k += D) {  // more than D senders
                    uint32_t cb[D];
#pragma unroll
                    for (int b = 0; b < D; ++b) {
                        cb[b] = k + b < m0.p1 ? a.in_col[k + b] : 0u;
                        if (k + b < m0.p1)
                            dma16((const void*)(a.F_prev + (uint64_t)(cb[b] & kColMask) * a.nwp + off), my + b * 1024);
                    }
                    vm_drain();
#pragma unroll
                    for (int b = 0; b < D; ++b) {
                        if (k + b < m0.p1) {
                            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(my + b * 1024 + lane16);
                            claim(x.x, x.y, cb[b]);
                        }
                    }
                }
                c_gathers += (lg == 0) ? (unsigned long long)(m0.p1 - m0.p0) : 0ull;
                // new state
                Row<WPL> F;
                unsigned long long T = 0;
                const uint64_t g = a.lo + i;
#pragma unroll
                for (int w = 0; w < WPL; ++w) {
                    F.w[w] = S.w[w] & ~sp.w[w];
                    T += __popcll(F.w[w]);
                    if (F.w[w] && !(a.ablate & 8)) {
                        const uint64_t idx = g * a.nw + off + w;
                        c_hash += gg_word_hash(idx, S.w[w]) - (sp.w[w] ? gg_word_hash(idx, sp.w[w]) : 0ull);
                    }
                }
                const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
                if (!(a.ablate & 1)) {
                    if (any || m0.zm) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
                    if (any) store_row<WPL>(a.base + rep * a.nwp + off, S);
                }
                if (lg == 0 && !(a.ablate & 16)) {
                    if (any) a.flg_cur[rep] = FL_ACT;
                    a.cand[rep] = 0;
                    if (m0.zm) a.zmark[rep] = 0;
                }
                const unsigned long long deg = a.symmetric ? (unsigned long long)(m0.p1 - m0.p0)
                                                           : (unsigned long long)(a.out_ptr[i + 1] - a.out_ptr[i]);
                c_new += T;
                c_fwd += deg * T - cl_recip;
                c_active += (lg == 0) ? 1ull : 0ull;
            } else if (m0.zm) {  // only a stale F row to clear
                if (!(a.ablate & 1)) {
                    Row<WPL> z;
                    z.w[0] = z.w[1] = 0;
                    store_row<WPL>(a.F_cur + rep * a.nwp + off, z);
                }
                if (lg == 0) a.zmark[rep] = 0;
            }
            m0 = m1;
            m1 = m2;
#pragma unroll
            for (int b = 0; b < D; ++b) c0[b] = c1[b];
        }
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_fwd;
    acc[C_FWD_DELIV] = c_fwd;
    acc[C_HASH] = c_hash;
    acc[C_NEXT_ACKS] = c_fwd;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers;
    flush_counters(a, acc, s_red, t_start);
}

// First-seen round of every new bit (GG_TRACK_DELIVERY only; observation).
__global__ void track_delivery(const uint64_t* F_cur, const uint8_t* flg_cur, int32_t* dr, uint64_t n_own,
                               uint64_t own0, uint32_t nwp, uint32_t nw, uint32_t W, int32_t round) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_own * nw) return;
    const uint64_t i = t / nw, j = t % nw;
    if (!(flg_cur[own0 + i] & FL_ACT)) return;
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
