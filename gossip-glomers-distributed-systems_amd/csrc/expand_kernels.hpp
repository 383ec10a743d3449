// expand_kernels.hpp — the per-round gossip kernels for gfx950 (CDNA4).
//
// One lockstep round is three launches on one stream (captured in a hipGraph):
//   round_prep    — one thread per node: the sync timer (`broadcast/main.go:42-51`,
//                   `SyncBroadcast` reads, `broadcast.go:119-121`), the read_oks
//                   that answer last round's reads (`HandleRead`, `:124-132`), and
//                   in sparse rounds *candidate marking*: a node can change this
//                   round only if a sender of its in-list was active (or pushed)
//                   last round, it has a deferred fold (LAG), a sync callback, or a
//                   client broadcast; active senders mark their out-lists.
//   expand_round  — the device form of HandleBroadcast (`:59-79`) +
//                   rebroadcastAllExcept (`:50-57`) + the SyncBroadcast callback
//                   (`:82-117`) for every candidate node, in the determinized
//                   order of DESIGN.md §2 (client broadcasts, node broadcasts by
//                   ascending sender, read_ok callbacks by ascending peer).
//   expand_stream — the same for *dense* lean rounds, over every node.
// Which of expand_round / expand_stream works (the other exits at once) is
// decided on the device from the number of nodes that became active in the
// previous round (dense_round), so one captured launch sequence serves every
// round shape.
//
// State: `base` holds every node's set *in place*; F[r&1] holds
// the bits a node learned in round r (what it forwards in r+1), valid only
// where flags[r&1] has ACT. A node whose set is read by a sync peer in round r
// (a read_ok payload or a push) keeps base = its round r-1 set and marks LAG;
// then its true set is base | F. So every reader computes
//     set(u) = base[u] | (LAG(u) ? F_prev[u] : 0)
// and idle nodes move no row.
//
// Work mapping of expand_round: tiles of NG = 256/G consecutive nodes; each
// block examines tiles blockIdx.x + k*gridDim.x 64 at a time (their candidate
// flags, set by round_prep / mark_injections), compacts the live ones with
// their edge ranges in LDS, and for each stages the CSR slice (row_ptr, col)
// plus per-sender flags in LDS with coalesced loads; a *node group* of G lanes
// owns one node, lane l holding words [l*WPL, l*WPL+WPL) of its set (16-byte
// accesses for WPL = 2). Pass 1 compacts the node's contributing senders in
// LDS; pass 2 gathers their rows 4 at a time and runs the claim chain (first
// deliverer, ascending sender) in registers. Counters are linear in per-lane
// popcounts: summed per lane, reduced once per block, added to one of 64
// counter slots.
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
// 4: the lean kernel fits 95 VGPRs (5 waves/SIMD) and the masked one 123 without
// spills (6: 103 / 128 + 28 B scratch); A/B at 2M nodes: C3 7.88 -> 6.97 ms per
// episode, C2 equal (its internal nodes take a second batch of one row)
#ifndef GG_STREAM_ROWS
#define GG_STREAM_ROWS 4
#endif
// 5 waves (round 6): expand_stream<32,2> (C4) fits 96 VGPRs + 12 B of scratch
// instead of 4 waves: the C4 leg 824 -> 813 ms/step, C2 / C3 / C5 equal
// (profiles/r6/ab_waves5/); 6 waves spill 76 B a lane and double C2's dense rounds
#ifndef GG_STREAM_WAVES_PER_EU
#define GG_STREAM_WAVES_PER_EU 5
#endif
constexpr int kStreamRows = GG_STREAM_ROWS;
// ... in the marking kernel: three rows keep it at 95 VGPRs, 5 waves/SIMD (four:
// 101, four waves). With three in both kernels C2 ran 1.613 -> 1.568 ms/step and
// C3 at 2M nodes 6.58 -> 6.82 ms (in-degree 8 wants four in the busy rounds)
#ifndef GG_MARK_ROWS
#define GG_MARK_ROWS 3
#endif
constexpr int kMarkRows = GG_MARK_ROWS;
constexpr uint32_t kBllMax = 4096;  // block lists: nodes of a block's slice (kBlock x 16 candidate bytes)
// Sender rows a lane of expand_stream1 (W = 64) keeps in flight.
#ifndef GG_STREAM1_ROWS
#define GG_STREAM1_ROWS 8
#endif
// ... and the waves per SIMD it is compiled for (A/B knob; the lean W >= 128
// kernels keep GG_STREAM_WAVES_PER_EU)
#ifndef GG_STREAM1_WAVES_PER_EU
#define GG_STREAM1_WAVES_PER_EU GG_STREAM_WAVES_PER_EU
#endif

// Sender (flag, row) pairs a lane keeps in flight in dense lean rounds.
#ifndef GG_SPEC_BATCH
#define GG_SPEC_BATCH 4
#endif

constexpr int kBlock = 256;
constexpr int kSlots = 64;       // counter slots
constexpr int kCounters = 32;    // per slot
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
    C_DROPPED, C_FIRED, C_HASH, C_NEXT_ACKS, C_NEXT_ACKDROP, C_ACTIVE, C_GATHERS,
    C_NACT,   // nodes that became active (ACT) this round: next round's dense/sparse choice
    C_BYTES,  // algorithmic bytes the launch had to move, per kernel kind
    C_NACTDEG,  // out-degree sum of those nodes: next round's flags-first choice
    C_NUM
};
// Kernel kinds with their own device clock stamps (s_memrealtime, 100 MHz) per
// counter slot: first block start (stored complemented, so a max over
// zero-initialised slots gives the min) and last block end. Every block of
// every launch stamps, no-op exits included, so a kind's time per round is
// comparable with rocprofv3's dispatch durations.
enum Kind : int { K_PREP = 0, K_EXPAND = 1, K_STREAM = 2, K_NKIND = 3 };
constexpr int kStamp0 = 20;  // stamps at kStamp0 + 2*kind (+0 start~, +1 end)
constexpr int kBytes0 = 26;  // C_BYTES of each kind lands at kBytes0 + kind
static_assert(C_NUM <= kStamp0 && kStamp0 + 2 * K_NKIND <= kBytes0 && kBytes0 + K_NKIND <= kCounters, "slot layout");

__device__ __forceinline__ unsigned long long clock100() { return __builtin_amdgcn_s_memrealtime(); }

struct TileWork {
    uint32_t tile;   // tile index (nodes tile*NG ..)
    uint32_t ne;     // in-edges of the tile
    int64_t eb;      // in_ptr of the tile's first node
};

// A contiguous piece of a hub node's in-list (or, for marking, of a high
// out-degree sender's out-list).
struct HubChunk {
    uint32_t node;   // local row
    uint32_t n;      // edges in the piece
    int64_t e0;      // first edge
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
    uint8_t* flg_prev_w;        // flg_prev, writable (marking rounds clear a processed node's byte)
    uint8_t* cand;              // [rows] candidate bytes of this round (cleared by expand); two
                                // arrays by round parity, so marks for round r+1 made during r
                                // (cand_next) never meet round r's reads and clears
    uint8_t* cand_next;         // [rows] candidate bytes of round r+1
    uint32_t mark_cand;         // marking lean rounds (double-buffered, single engine): the expand
                                // kernel marks round r+1's candidates itself — every node whose set
                                // changes, and its receivers — and clears the node's flag byte of
                                // r-1, so round r+1 needs no round_prep (prep_in_compact)
    uint32_t prep_in_compact;   // no round_prep this round: compact_round sums the rings of r-1
                                // (round r-1 was a marking round, or r is the first round)
    uint32_t block_lists;       // ... and no compact_round either: the marking kernel sums the
                                // rings itself and each of its blocks lists the candidates of
                                // its own granules of the owned nodes in LDS
    uint32_t solo;              // marking rounds: 0 = both expand kernels are launched and each exits
                                // when the round is the other's (busy or not, decided on the device);
                                // SOLO_MARK / SOLO_DB = the host launched only that one (its guess
                                // from the last run of this round: busy_count of its C_NACT), which
                                // then takes the round whatever it finds: the marking kernel visits
                                // every node when the round is busy, expand_stream_db every node
                                // always; either sums round r-1's rings itself
    uint32_t prev_mark;         // round r-1 was a solo marking round: 1 = its kernel marked round r's
                                // candidates, 2 = it marked nothing (expand_stream_db: round r is
                                // dense); 0 = the device decides from the act ring (busy_prev)
    uint32_t no_list;           // lean streaming round without compact_round (the host expects it busy,
                                // from the last run of this round): dense whatever the act ring says
    uint8_t* zmark;             // [rows] F row of this parity is stale (node active 2 rounds ago)
    uint8_t* tile_cand;         // [n_tiles rounded to 8] tile has a candidate (sparse rounds)
    struct TileWork* work;      // live tiles of a sparse round (compact_round; expand_round)
    uint32_t* n_work;           // [2]: live tiles, candidate nodes (two pairs by round parity)
    uint32_t* n_work_next;      // [2] round r+1's pair: zeroed by this round's compact_round
    uint32_t* bcount;           // [compact blocks + 1] split compaction (large graphs): per-block counts -> offsets
    uint32_t* nodes;            // candidate nodes of a sparse lean round (compact_round; expand_stream)
    uint32_t* act;              // [4] ring: nodes that became active in round r (slot r&3), summed by round_prep
    unsigned long long* act_deg;  // [4] ring: their out-degree sum (edges carrying F rows next round)
    // the same three rings spread over kSlots addresses per round ([4][kSlots]): the
    // kernels of round r add into slot r&3 (block % kSlots), round_prep of round r+1
    // sums them — one same-address atomic per block on a single word was a serial
    // tail at the end of every launch
    uint32_t* act_s;
    unsigned long long* act_deg_s;
    unsigned long long* tot_s;
    uint64_t* abits;            // [rows/64] bit u: sender u is ACT in round r-1 (pack_act_bits; flags-first)
    int32_t ff_ok;              // flags-first gathers allowed below ff_ok/16 of the in-edges carrying data (0: never)
    uint64_t ff_min;            // ... and from ff_min such edges on (the bitmap pass costs more in smaller rounds)
    int32_t prep_wide;          // round_prep: the 16-nodes-per-thread sparse scan whatever the size (A/B)
    unsigned long long* tot;    // [4] ring: new bits of the owned nodes in rounds <= r (slot r&3), or nullptr
    unsigned long long full_new;  // n_own x lanes injected in rounds <= r-1: tot of r-1 equal to it means
                                  // every owned set holds every injected lane (sets hold injected lanes only)
    uint32_t lanes_prev;        // lanes of this engine injected in rounds <= r-1 (0: none yet). A node whose
                                // set holds that many lanes is saturated: sender rows of r-1 carry only
                                // those lanes, so it has nothing to gather (expand_stream1)
    // hubs (lean rounds): owned nodes with in-degree > hub_deg skip expand_stream
    // and take hub_chunks + hub_finish; senders with out-degree > hub_deg are
    // marked by hub_mark instead of round_prep (0: no hubs)
    uint32_t hub_deg;
    const struct HubChunk* hchunks;  // in-edge chunks of the hubs, hub by hub
    uint64_t n_hchunks;
    const uint32_t* hubs;            // [n_hubs] hub local rows
    const uint32_t* hub_c0;          // [n_hubs+1] first chunk of each hub
    uint64_t n_hubs;
    uint64_t* hscratch;              // [n_hchunks][2][nwp] (union, first-claimer-recip) per chunk;
                                     // streamed sync engines: [n_hchunks][3][nwp], the third row the
                                     // chunk's callback prefix (hub_sync_*)
    uint32_t* hflag;                 // [n_hchunks] streamed sync rounds: HF_* of the chunk this round
    uint8_t* hlive;                  // [n_hubs] streamed sync rounds: the hub is processed this round
                                     // (its candidate byte, | CA_NODE; written by sync_records)
    const struct HubChunk* mchunks;  // out-edge chunks of high out-degree senders
    uint64_t n_mchunks;
    uint4* srec;                // [2 n_own] sync records (streamed sync rounds), or nullptr
    uint8_t* pushb;             // [out-edges] 1: the node's sync callback (round r-1 for a pusher
                                // of round r) pushed something to that peer (SyncBroadcast
                                // :104-108 sends nothing for an empty difference); or nullptr
    const uint32_t* rev;        // [in-edges] the sender's out-edge index of this edge (owned
                                // senders; streamed sync rounds), or nullptr
    uint8_t* sstate;            // [rows] sender state of round r (round_prep; streamed sync rounds)
    uint64_t* ibits;            // [rows/64] bit: sstate has FL_ACT, FL_LAG or SE_FM3 (a
                                // cache-resident filter in front of it; callbacks: fired_m2)
    uint8_t* pushany;           // [rows] the node's sync callback (streamed) pushed to some peer
    uint32_t push_marked;       // the streamed callbacks of r-1 marked their push receivers and
                                // wrote pushany: round_prep skips the pushers' out-lists
    uint32_t mark_next;         // this round's callbacks mark their push receivers for r+1
    uint64_t* pend;             // batched gossip: [rows][nwp] pending values (not yet sent)
    uint32_t* pend_src;         // batched gossip: [rows] kPendNone, kPendMixed, or the only
                                // sender's local row | in-edge reciprocal bit << 31
    uint32_t batch_tick;        // batched gossip: this round ends with a send
    const uint64_t* bset_prev;  // batched gossip with sync: [rows][nwp] every node's set after r-1
    uint64_t* bset_cur;         // (read by push receivers and callbacks), and after r (written by all)
    int32_t* dr;                // batched gossip: first-seen rounds [n_own][dr_w] (GG_TRACK_DELIVERY), or nullptr
    uint32_t dr_w;
    uint2* nmeta;               // streamed sync rounds: compact_round's node list as (node,
                                // cand | flg_cur << 8 | sstate << 16), cand cleared; or nullptr
    uint64_t* sat;              // [rows/64] saturation digest (streamed sync rounds, else nullptr):
                                // bit = the row's seen set was, after some round r' < r, every
                                // lane injected so far (|S| == usat) — exact: sets only grow
                                // and hold injected lanes only, so it stays true until a new
                                // lane is injected (sat_reset). Owned rows; ghosts stay 0.
    uint64_t* sat_new;          // [rows/64] bits found this round (merged by the next round_prep)
    uint8_t* lsat;              // [rows] lean rounds (W >= 128), or nullptr: 1 = the owned node's set
                                // held every lane injected through the round that set it (lusat then).
                                // Sets only grow and hold injected lanes only, and the host clears the
                                // digest after any later injection, so a set bit means the node's set
                                // of r-1 holds every lane any sender row of r-1 can carry: it gathers
                                // nothing (expand_stream, hub_chunks, hub_finish skip its in-edges)
    uint32_t lusat;             // lanes of this engine's range injected in rounds <= r
    uint32_t lmark;             // the digest's writers mark this round (0: read only)
    const uint32_t* lreach;     // [n_own] lanes broadcast into the node's component over the whole known
                                // schedule (symmetric graphs with several components: lreach_fill_tab),
                                // or nullptr: lusat for every node. A set never holds more (§4.2)
    uint32_t usat;              // lanes of this engine's range injected in rounds <= r
    uint32_t sat_reset;         // usat grew this round: every digest bit is void
    const uint64_t* fired_m1;   // sync-fired bitmaps of rounds r-1, r-2, r-3
    const uint64_t* fired_m2;
    const uint64_t* fired_m3;
    uint64_t* fired_cur;        // round r (written whole by round_prep)
    int32_t* sync_next;         // [rows] sync timers of the owned nodes and (sharded) of the
    uint32_t* sync_k;           // ghosts: every engine runs its ghosts' timers itself
    const uint8_t* grp[5];      // partition groups of rounds r-3..r+1 (nullptr: no window)
    const uint64_t* ebits[5];   // the same windows as in-edge bitmaps: bit e = the two ends of
                                // in-edge e are in different groups (masked streaming rounds),
                                // or the caller's per-edge mask (gg_set_partition windows)
    uint32_t ewin;              // bit k: window k is per-edge (ebits[k] decides, not grp[k])
    const uint32_t* inj;        // (local node, lane) pairs sorted by node (inj_tab: of the whole batch)
    uint32_t n_inj;             // host count (inj_tab == nullptr: the kernels' count)
    const uint32_t* inj_tab;    // this round's [first pair, end] in inj, in device memory (inj_p / inj_n): a
                                // captured batch then replays for any injections with the same rounds
    unsigned long long* counters;  // [kSlots][kCounters]
    uint64_t n_own, own0, lo;   // own rows are local rows own0 .. own0+n_own-1 (own0 = 0)
    const uint32_t* gid;        // [rows] original node id of each local row (sharded), or
                                // nullptr: original id = lo + row (single engine)
    uint64_t ghost0, n_ghost;   // sharded: ghost rows ghost0 .. ghost0+n_ghost-1
    const int64_t* gout_ptr;    // [n_ghost+1] per ghost: the owned nodes it sends to
    const uint32_t* gout_col;
    uint32_t nwp;               // words per local row (power of two >= this engine's lane words)
    uint32_t nw, word0;         // seen_hash index of local word j of node g: g * nw + word0 + j
                                // (nw = words per node of the whole job; word0 = this engine's
                                // first lane word: non-zero when ranks split the lanes)
    uint32_t count_nodes;       // count node-level events (reads, read_oks, their drops, timers):
                                // 1 on exactly one engine per node (lane group 0)
    uint32_t tile_nodes;        // NG of the expand kernel
    int32_t symmetric;          // out-lists == in-lists
    uint64_t n_edges;           // in_col entries of this engine
    uint64_t rows;              // replica rows
    int32_t db;                 // double-buffered lean round: sets of r-1 in base_prev,
                                // this round's sets into base (rows of nodes that changed in r or r-1),
                                // senders' sets gathered instead of F rows, no F rows written
    const uint64_t* base_prev;
    int32_t stream_ok;          // lean round (no sync events in expand, no masks) with nwp >= 2:
                                // expand_stream takes it when it is dense (dense_round)
    int64_t round;
    uint64_t seed;
    uint64_t sync_mix, sync_rcp;  // gg_sync_interval_rcp's constants (gg_mix64(seed ^ GG_TAG_SYNC), gg_sync_rcp)
    uint32_t sync_base, sync_jitter;
    int32_t enable_sync;
};

// This round's client broadcasts: from the batch's device-resident offset table
// when there is one (the launch sequence does not depend on the pairs), else
// from the host-set pointer and count.
__device__ __forceinline__ uint32_t inj_n(const RoundArgs& a) {
    return a.inj_tab ? a.inj_tab[1] - a.inj_tab[0] : a.n_inj;
}
__device__ __forceinline__ const uint32_t* inj_p(const RoundArgs& a) {
    return a.inj_tab ? a.inj + 2 * (size_t)a.inj_tab[0] : a.inj;
}

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
    if constexpr (WPL % 2 == 0) {
#pragma unroll
        for (int k = 0; k < WPL; k += 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p + k);
            r.w[k] = v.x;
            r.w[k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < WPL; ++k) r.w[k] = p[k];
    }
    return r;
}

template <int WPL>
__device__ __forceinline__ void store_row(uint64_t* p, const Row<WPL>& r) {
    if constexpr (WPL % 2 == 0) {
#pragma unroll
        for (int k = 0; k < WPL; k += 2) *reinterpret_cast<ulonglong2*>(p + k) = make_ulonglong2(r.w[k], r.w[k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < WPL; ++k) p[k] = r.w[k];
    }
}

// 16-byte non-temporal store of a lane's two words
__device__ __forceinline__ void store_row_nt(uint64_t* p, const Row<2>& r) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store((u64x2){r.w[0], r.w[1]}, reinterpret_cast<u64x2*>(p));
}

__device__ __forceinline__ bool bit_at(const uint64_t* bm, uint64_t row) {
    return (bm[row >> 6] >> (row & 63)) & 1ull;
}

// Most nodes are candidates this round: the nodes that became active in r-1
// (owned ones and, in sharded engines, ghosts) times the mean out-degree cover
// at least half of the owned nodes. Read from the act ring,
// which no kernel of round r writes, so every launch of the round agrees.
__device__ __forceinline__ bool busy_round(const RoundArgs& a) {
    const double act = (double)a.act[(a.round - 1) & 3];
    return 2.0 * act * (double)a.n_edges >= (double)a.n_own * (double)a.n_own;
}
// Round r-1's expand marked no candidates for round r: it was busy (the same
// test one round earlier, from the act ring: expand_stream_db took it), or the
// host launched only expand_stream_db in it (RoundArgs::solo).
__device__ __forceinline__ bool busy_prev(const RoundArgs& a) {
    if (a.prev_mark) return a.prev_mark == 2;
    const double act = (double)a.act[(a.round - 2) & 3];
    return 2.0 * act * (double)a.n_edges >= (double)a.n_own * (double)a.n_own;
}
// Dense lean round: expand_stream visits every node, round_prep marks nothing
// and expand_round exits. A round without round_prep (prep_in_compact) after a
// busy round is dense whatever its own count: a busy round's expand marks no
// candidates (expand_stream_db takes it, not the marking kernel), so the round
// after it visits every node and marks for the next one.
__device__ __forceinline__ bool dense_round(const RoundArgs& a) {
    return a.stream_ok && (a.no_list || busy_round(a) || (a.prep_in_compact && busy_prev(a)));
}

// Flags-first streaming round: fewer than half of the in-edges name a sender
// that was ACT last round (an F row that is not zero), so expand_stream looks
// each sender up in the abits bitmap first and gathers only the rows of active
// senders. Random row gathers of <= 128 B are capped by the memory system's
// request rate (~50 G rows/s, tools/gather_bench.hip), and the bitmap (one bit
// a node; in degree order its hub part stays in L2) replaces most of them: in
// C4's round 2 about 6% of the candidates' in-edges carry data.
__device__ __forceinline__ bool ff_round(const RoundArgs& a) {
    if (!(a.ff_ok && a.stream_ok && a.act_deg)) return false;
    const unsigned long long d = a.act_deg[(a.round - 1) & 3];
    return d >= a.ff_min && 16.0 * (double)d < (double)a.ff_ok * (double)a.n_edges;
}

// Every owned node already holds every lane injected so far and the round
// injects nothing: no set can change (e.g. the quiescence round that ends an
// episode), so a lean round gathers nothing; only stale F rows are cleared.
__device__ __forceinline__ bool all_full(const RoundArgs& a) {
    return a.tot && inj_n(a) == 0 && a.tot[(a.round - 1) & 3] == a.full_new;
}

// Original node id of local row i (hashes, sync timers, partition groups).
__device__ __forceinline__ uint64_t gid_of(const RoundArgs& a, uint64_t i) {
    return a.gid ? (uint64_t)a.gid[i] : a.lo + i;
}

// message from replica row ra to replica row rb in round (r-3+k) dropped? e:
// the edge between them (its position in rb's in-list or ra's out-list: the
// same list on the symmetric topologies per-edge windows require).
template <bool MASKW>
__device__ __forceinline__ bool masked(const RoundArgs& a, int k, uint64_t ra, uint64_t rb, uint64_t e) {
    if constexpr (!MASKW) {
        return false;
    } else {
        const uint8_t* g = a.grp[k];
        if (g == nullptr) return false;
        if ((a.ewin >> k) & 1u) return bit_at(a.ebits[k], e);  // gg_set_partition window
        return g[ra] != g[rb];
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
__device__ __forceinline__ bool is_push(const RoundArgs& a, uint8_t ef, uint64_t u, uint64_t v, uint64_t e) {
    if constexpr (!SYNCW) {
        return false;
    } else {
        return (ef & SE_FM3) && !masked<MASKW>(a, 0, u, v, e) && !masked<MASKW>(a, 1, v, u, e);
    }
}

// Saturation digest: the G lanes of a node group that changed its set this
// round count it; a full set (every lane injected so far) sets the node's bit
// for the next rounds. Group-uniform call (shuffles stay inside the group).
template <int G, int WPL>
__device__ __forceinline__ void sat_mark(const RoundArgs& a, const Row<WPL>& S, uint64_t rep, int lg) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < WPL; ++w) c += (uint32_t)__popcll(S.w[w]);
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lg == 0 && c == a.usat) atomicOr(a.sat_new + (rep >> 6), 1ull << (rep & 63));
}

// Lean saturation digest: a node group whose node's set changed this round
// counts it and sets the node's bit when it holds every lane injected so far.
// Group-uniform call.
// Sum over a node group of G lanes (G-aligned), every lane gets it: DPP moves
// inside 16-lane rows (quad swaps, half-row and row mirrors: VALU only), a
// cross-lane permute only past 16 lanes (ds_bpermute goes through the LDS unit
// and its counter; five of them per changed node cost C2's dense rounds ~10 %).
#ifndef GG_LSAT_DPP
#define GG_LSAT_DPP 1
#endif
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
#if GG_LSAT_DPP
    if constexpr (G >= 2) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
    if constexpr (G >= 4) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
    if constexpr (G >= 8) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    if constexpr (G >= 16) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false); // row_mirror
    if constexpr (G >= 32) x += (uint32_t)__shfl_xor((int)x, 16, 64);
    if constexpr (G >= 64) x += (uint32_t)__shfl_xor((int)x, 32, 64);
#else
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
#endif
    return x;
}

template <int G, int WPL>
__device__ __forceinline__ void lsat_mark(const RoundArgs& a, const Row<WPL>& S, uint64_t rep, int lg, uint32_t tgt) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < WPL; ++w) c += (uint32_t)__popcll(S.w[w]);
    c = group_sum<G>(c);
    // a plain byte store: a bitmap word took 64 same-address atomics when a run of
    // consecutive nodes saturated in one round (C2 +11 %)
    if (lg == 0 && c == tgt) a.lsat[rep] = 1;
}

// Component labels for the lean digest's targets (symmetric single engines, at
// topology install): min-label propagation pulled over the in-lists (= out-lists)
// with pointer jumping, until a pass changes nothing. Labels only decrease and
// stay inside the component, so in-place updates (and atomicMin for hubs) are safe.
__global__ void cc_init(uint32_t* lab, uint64_t n) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        lab[v] = (uint32_t)v;
}
// one thread per node of in-degree <= hub_deg (hubs: cc_hubs)
__global__ void cc_pass(const int64_t* in_ptr, const uint32_t* in_col, uint32_t* lab, uint64_t n, uint32_t hub_deg,
                        uint32_t* changed) {
    bool ch = false;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t p0 = in_ptr[v], p1 = in_ptr[v + 1];
        if (hub_deg && p1 - p0 > (int64_t)hub_deg) continue;
        const uint32_t l0 = lab[v];
        uint32_t m = l0;
        for (int64_t e = p0; e < p1; ++e) m = min(m, lab[in_col[e] & kColMask]);
        if (m < l0) {
            lab[v] = m;
            ch = true;
        }
    }
    if (ch) *changed = 1u;
}
// one wave per node of in-degree > deg_min (the whole graph of a vertex-part
// engine has no hub chunk list): lanes stride the in-list, a wave minimum
__global__ void cc_pass_wide(const int64_t* in_ptr, const uint32_t* in_col, uint32_t* lab, uint64_t n, uint32_t deg_min,
                             uint32_t* changed) {
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const int ln = threadIdx.x & 63;
    bool ch = false;
    for (uint64_t v = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; v < n; v += waves) {
        const int64_t p0 = in_ptr[v], p1 = in_ptr[v + 1];
        if (p1 - p0 <= (int64_t)deg_min) continue;  // wave-uniform
        uint32_t m = ~0u;
        for (int64_t e = p0 + ln; e < p1; e += 64) m = min(m, lab[in_col[e] & kColMask]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
        if (ln == 0 && m < atomicMin(lab + v, m)) ch = true;
    }
    if (ch) *changed = 1u;
}
// a block per hub in-edge chunk: the chunk's smallest label, atomicMin into the hub
__global__ __launch_bounds__(kBlock) void cc_hubs(const HubChunk* ch, uint64_t n_ch, const uint32_t* in_col,
                                                  uint32_t* lab, uint32_t* changed) {
    __shared__ uint32_t s_m[kBlock / 64];
    for (uint64_t c = blockIdx.x; c < n_ch; c += gridDim.x) {
        const HubChunk hc = ch[c];
        uint32_t m = ~0u;
        for (uint32_t k = threadIdx.x; k < hc.n; k += kBlock) m = min(m, lab[in_col[hc.e0 + k] & kColMask]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
        if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < kBlock / 64; ++w) m = min(m, s_m[w]);
            if (m < atomicMin(lab + hc.node, m)) *changed = 1u;
        }
        __syncthreads();
    }
}
__global__ void cc_jump(uint32_t* lab, uint64_t n, uint32_t* changed) {
    bool ch = false;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t l = lab[v], ll = lab[l];
        if (ll < l) {
            lab[v] = ll;
            ch = true;
        }
    }
    if (ch) *changed = 1u;
}
// components = nodes that are their own label
__global__ void cc_roots(const uint32_t* lab, uint64_t n, unsigned long long* roots) {
    unsigned long long c = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        c += lab[v] == (uint32_t)v ? 1u : 0u;
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(roots, c);
}

// A node of the lean digest gathers nothing this round: saturated and no client
// broadcast to it (one would change its set: forwards and marks need its degree)
__device__ __forceinline__ bool lsat_skip(const RoundArgs& a, uint64_t rep, uint8_t ca) {
    return a.lsat && !(ca & CA_INJ) && a.lsat[rep];
}

// The digest's first bits: one pass over every owned row at the start of the
// first streamed sync round r (lean rounds before it have no LAG rows, so the
// base row is the node's set after r-1, and they do not mark, keeping the
// dense loop lean). cpn 16-byte chunks per row, one per lane; a wave covers
// 64/cpn consecutive nodes, one word's worth of bits, and ORs them in at once.
__global__ __launch_bounds__(kBlock) void sat_scan(const uint64_t* base, uint64_t n_own, uint32_t nwp, uint32_t usat,
                                                   uint64_t* sat) {
    if (nwp == 1) {  // W = 64: one word per node, one node per lane, a wave = one digest word
        const uint64_t node = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        const bool full = node < n_own && (uint32_t)__popcll(base[node]) == usat;
        const unsigned long long m = __ballot(full);
        if ((threadIdx.x & 63) == 0 && m) atomicOr(sat + (node >> 6), m);
        return;
    }
    const uint32_t cpn = nwp / 2;
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t node = t / cpn;
    uint32_t c = 0;
    if (node < n_own) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(base + node * nwp + (t % cpn) * 2);
        c = (uint32_t)(__popcll(v.x) + __popcll(v.y));
    }
    for (uint32_t o = cpn / 2; o > 0; o >>= 1) c += __shfl_xor(c, (int)o, 64);
    const unsigned long long m = __ballot(node < n_own && t % cpn == 0 && c == usat);
    if ((threadIdx.x & 63) == 0) {
        uint64_t bits = 0;  // lane k*cpn -> node bit k
        for (uint32_t k = 0; k < 64 / cpn; ++k) bits |= ((m >> (k * cpn)) & 1ull) << k;
        const uint64_t n0 = t / cpn;  // first node of the wave
        if (bits) atomicOr(sat + (n0 >> 6), bits << (n0 & 63));
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

__device__ __forceinline__ void stamp(const RoundArgs& a, int kind, unsigned long long t_start) {
    unsigned long long* slot = a.counters + (blockIdx.x % kSlots) * kCounters + kStamp0 + 2 * kind;
    atomicMax(slot, ~t_start);
    atomicMax(slot + 1, clock100());
}

// A launch with nothing to do this round (the other kernel kind takes it).
__device__ __forceinline__ void noop_exit(const RoundArgs& a, int kind, unsigned long long t_start) {
    if (threadIdx.x == 0 && blockIdx.x == 0) stamp(a, kind, t_start);  // one block's stamps suffice
}

__device__ __forceinline__ void flush_counters(const RoundArgs& a, unsigned long long (&acc)[C_NUM],
                                               unsigned long long (*s_red)[C_NUM], unsigned long long t_start,
                                               int kind) {
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
        const int idx = threadIdx.x == C_BYTES ? kBytes0 + kind : (int)threadIdx.x;
        if (s) atomicAdd(&a.counters[(blockIdx.x % kSlots) * kCounters + idx], s);
        const int sl = (int)(a.round & 3) * kSlots + (int)(blockIdx.x % kSlots);
        if (threadIdx.x == C_NACT && s) atomicAdd(&a.act_s[sl], (uint32_t)s);
        if (threadIdx.x == C_NACTDEG && s && a.act_deg) atomicAdd(&a.act_deg_s[sl], s);
        if (threadIdx.x == C_NEW && s && a.tot) atomicAdd(&a.tot_s[sl], s);
    }
    if (threadIdx.x == 0) stamp(a, kind, t_start);
}

// Round r-1's rings (act, act_deg, tot) from their spread slots: every wave sums
// the act slots for its own dense/sparse choice; block 0 publishes the three
// sums for the round's later launches and clears round r's slots (nothing in
// the calling kernel adds to them). Returns this round's dense choice.
__device__ __forceinline__ bool rings_in(const RoundArgs& a) {
    const int lane = threadIdx.x & 63;
    const int pr = (int)((a.round - 1) & 3), cr = (int)(a.round & 3);
    const unsigned long long act_prev = wave_sum((unsigned long long)a.act_s[pr * kSlots + lane]);
    const bool dense = a.stream_ok &&
                       2.0 * (double)act_prev * (double)a.n_edges >= (double)a.n_own * (double)a.n_own;
    if (blockIdx.x == 0 && threadIdx.x < kSlots) {
        const unsigned long long d = wave_sum(a.act_deg_s[pr * kSlots + lane]);
        const unsigned long long n = wave_sum(a.tot_s[pr * kSlots + lane]);
        // round r's slots, and round r+1's: a round r+1 with block lists sums
        // its predecessor's slots while its own blocks add to its own, so it
        // finds them cleared and clears round r+2's (below)
        const int nr = (int)((a.round + 1) & 3);
        a.act_s[cr * kSlots + lane] = 0;
        a.act_deg_s[cr * kSlots + lane] = 0;
        a.tot_s[cr * kSlots + lane] = 0;
        a.act_s[nr * kSlots + lane] = 0;
        a.act_deg_s[nr * kSlots + lane] = 0;
        a.tot_s[nr * kSlots + lane] = 0;
        if (lane == 0) {
            a.act[pr] = (uint32_t)act_prev;
            a.act_deg[pr] = d;
            if (a.tot) a.tot[pr] = (a.round > 0 ? a.tot[(a.round - 2) & 3] : 0ull) + n;
        }
    }
    return dense;
}

constexpr uint32_t SOLO_MARK = 1, SOLO_DB = 2;

// Round r-1's rings as a kernel of round r sees them. Published (rings_in ran
// earlier in the round) or, in rounds with block lists, summed from r-1's slots
// by every wave, with block 0 publishing them for round r+1 and clearing round
// r+1's slots (round r's were cleared in round r-1; this round's blocks add to
// them). Both expand kernels of such a round publish the same values.
struct RingView {
    unsigned long long act, act_deg, tot;  // round r-1: nodes active, their degrees, cumulative new bits
    unsigned long long act_m2;             // round r-2: nodes active
};
template <bool SUM = true>
__device__ __forceinline__ RingView ring_view(const RoundArgs& a) {
    RingView v;
    const int pr = (int)((a.round - 1) & 3), p2 = (int)((a.round - 2) & 3);
    v.act_m2 = a.act[p2];
    if (!(SUM || a.solo) || !a.block_lists) {
        v.act = a.act[pr];
        v.act_deg = a.act_deg ? a.act_deg[pr] : 0ull;
        v.tot = a.tot ? a.tot[pr] : 0ull;
        return v;
    }
    const int lane = threadIdx.x & 63;
    v.act = wave_sum((unsigned long long)a.act_s[pr * kSlots + lane]);
    v.act_deg = a.act_deg ? wave_sum(a.act_deg_s[pr * kSlots + lane]) : 0ull;
    const unsigned long long n = a.tot ? wave_sum(a.tot_s[pr * kSlots + lane]) : 0ull;
    v.tot = a.tot ? (a.round > 0 ? a.tot[p2] : 0ull) + n : 0ull;
    if (blockIdx.x == 0 && threadIdx.x < kSlots) {
        const int nr = (int)((a.round + 1) & 3);
        a.act_s[nr * kSlots + lane] = 0;
        a.act_deg_s[nr * kSlots + lane] = 0;
        a.tot_s[nr * kSlots + lane] = 0;
        if (lane == 0) {
            a.act[pr] = (uint32_t)v.act;
            if (a.act_deg) a.act_deg[pr] = v.act_deg;
            if (a.tot) a.tot[pr] = v.tot;
            if (a.n_work_next) a.n_work_next[0] = a.n_work_next[1] = 0;
        }
    }
    return v;
}
__device__ __forceinline__ bool busy_count(const RoundArgs& a, unsigned long long act) {
    return 2.0 * (double)act * (double)a.n_edges >= (double)a.n_own * (double)a.n_own;
}
// ff_round() from a ring view
__device__ __forceinline__ bool ff_view(const RoundArgs& a, const RingView& rv) {
    return a.ff_ok && a.stream_ok && a.act_deg && rv.act_deg >= a.ff_min &&
           16.0 * (double)rv.act_deg < (double)a.ff_ok * (double)a.n_edges;
}

// ---------------------------------------------------------------------------
// round_prep: one thread per owned node (64 consecutive nodes per wave, so a
// wave owns whole words of the fired bitmap). In dense rounds the per-node
// flag/stale-row work moves into expand_stream and no candidates are marked,
// so without sync timers the launch is a no-op.
template <bool SYNCW, bool MASKW>
__global__ __launch_bounds__(kBlock) void round_prep(RoundArgs a) {
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    // Round r-1's rings from their spread slots (one slot per lane, summed per wave):
    // this kernel decides dense/sparse from its own sum, block 0 publishes the sums
    // for the round's later launches and clears round r's slots (nothing in this
    // kernel adds to them).
    const bool dense = rings_in(a);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.n_work[0] = a.n_work[1] = 0;  // compact_round runs after this kernel
    if (a.sat) {  // last round's digest bits in (readers of this round see rounds < r only)
        const uint64_t nw = (a.n_own + 63) / 64;
        for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < nw; t += (uint64_t)gridDim.x * kBlock) {
            const uint64_t w = (a.own0 >> 6) + t;
            a.sat[w] = a.sat_reset ? 0ull : (a.sat[w] | a.sat_new[w]);
            a.sat_new[w] = 0;
        }
    }
    if (!SYNCW && dense) {
        noop_exit(a, K_PREP, t_start);
        return;
    }
    unsigned long long c_reads = 0, c_read_oks = 0, c_dropped = 0, c_fired = 0, c_bytes = 0;
    const uint64_t nwords = (a.n_own + 63) / 64;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    if (!SYNCW && a.stream_ok && !a.n_ghost && (a.prep_wide || (a.n_own + 3) / 4 > stride)) {
        // sparse lean round without timers over more nodes than the capped grid
        // covers in four passes (the loop below, specialised): 16 nodes per
        // thread from one 16-byte load of each flag array (own0 % 64 == 0, rows
        // padded to 64), the next 16 loaded before these are handled (the stores
        // to cand keep the compiler from hoisting them), most of them idle; a node
        // whose F row of r-2 is stale in this round's buffer, or that was active
        // in r-1 (then also its receivers), becomes a candidate. C5 at 2^26 nodes:
        // sparse rounds 2.2x faster than the loop below with 4 nodes per thread,
        // and 16 with a load ahead keep enough bytes in flight to stream (4 nodes
        // per thread ran at ~1.4 TB/s); at C2's 2^20 the loop below is as fast
        // (all 179 GPU tests passed with this path taken for every size)
        const uint64_t nq = (a.n_own + 15) / 16;
        auto ld16 = [&](const uint8_t* f, uint64_t q) -> ulonglong2 {
            return q < nq ? *reinterpret_cast<const ulonglong2*>(f + a.own0 + 16 * q) : make_ulonglong2(0ull, 0ull);
        };
        // active senders come in clusters (a wave front), so a lane walking the
        // out-lists of its own up-to-16 active nodes one after another (dependent
        // row pointer -> column -> mark chains) set the pace; the wave instead lists
        // its active nodes in LDS and gives each lane one out-list at a time
        __shared__ uint32_t s_act[kBlock / 64][64 * 16];
        uint32_t* const L = s_act[threadIdx.x >> 6];
        const int ln = threadIdx.x & 63;
        uint64_t qb = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u);  // wave-uniform loop
        ulonglong2 fp = ld16(a.flg_prev, qb + ln), fc = ld16(a.flg_cur, qb + ln);
        for (; qb < nq; qb += stride) {
            const uint64_t q = qb + ln;
            const ulonglong2 np = ld16(a.flg_prev, q + stride), nc = ld16(a.flg_cur, q + stride);
            const uint64_t n16 = q >= nq ? 0 : (a.n_own - 16 * q < 16 ? a.n_own - 16 * q : 16);
            c_bytes += 2 * n16;
            uint32_t actm = 0;
            if (fp.x | fp.y | fc.x | fc.y) {
                for (uint32_t j = 0; j < (uint32_t)n16; ++j) {
                    const uint64_t wp = j < 8 ? fp.x : fp.y, wc = j < 8 ? fc.x : fc.y;
                    const uint8_t f = (uint8_t)(wp >> (8 * (j & 7))), fcj = (uint8_t)(wc >> (8 * (j & 7)));
                    if ((fcj & FL_ACT) || (f & FL_LAG) || (a.db && (f & FL_ACT))) a.cand[a.own0 + 16 * q + j] = CA_NODE;
                    if (f & FL_ACT) actm |= 1u << j;
                }
            }
            const uint32_t cnt = (uint32_t)__popc(actm);
            uint32_t incl = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (ln >= o) incl += y;
            }
            const uint32_t total = __shfl(incl, 63, 64);
            if (total) {
                uint32_t pos = incl - cnt;
                for (uint32_t m = actm; m; m &= m - 1) L[pos++] = (uint32_t)(16 * q) + (uint32_t)(__ffs(m) - 1);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (uint32_t k = ln; k < total; k += 64) {
                    const uint64_t i = L[k];
                    const int64_t o0 = a.out_ptr[i];
                    int64_t o1 = a.out_ptr[i + 1];
                    if (a.hub_deg && o1 - o0 > (int64_t)a.hub_deg) o1 = o0;  // hub_mark does it
                    c_bytes += 16 + 5 * (unsigned long long)(o1 - o0);
                    constexpr int B = 8;
                    for (int64_t e0 = o0; e0 < o1; e0 += B) {
                        uint64_t w[B];
#pragma unroll
                        for (int b = 0; b < B; ++b) w[b] = e0 + b < o1 ? (uint64_t)(a.out_col[e0 + b] & kColMask) : ~0ull;
#pragma unroll
                        for (int b = 0; b < B; ++b)
                            if (w[b] < a.n_own) a.cand[w[b]] = CA_NODE;
                    }
                }
                __builtin_amdgcn_wave_barrier();  // the list is rewritten next iteration
            }
            fp = np;
            fc = nc;
        }
        unsigned long long acc[C_NUM];
#pragma unroll
        for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
        acc[C_BYTES] = c_bytes;
        flush_counters(a, acc, s_red, t_start, K_PREP);
        return;
    }
    // the per-node bytes of the next node are loaded before this node's stores:
    // two nodes' worth of loads in flight per thread (the grid is capped)
    // (timer rounds: the out-list bounds and the timer count too, for every node —
    // 12 coalesced bytes a node — so a firing node or an answered read has no
    // dependent load: C2's timer rounds were three memory latencies per node)
    struct PrepIn {
        uint64_t w1, w2, w3;  // fired words of r-1, r-2, r-3
        int64_t o0, o1;       // out_ptr[i], out_ptr[i+1] (SYNCW)
        int32_t sn;           // sync_next
        uint32_t sk;          // sync_k (SYNCW)
        uint8_t f, fc, pa;    // flg_prev, flg_cur, pushany
    };
    auto load_in = [&](uint64_t i, PrepIn& p) {
        p = PrepIn{};
        if (i >= a.n_own) return;
        const uint64_t rp = a.own0 + i;
        p.f = a.flg_prev[rp];
        if (!dense) p.fc = a.flg_cur[rp];
        if constexpr (SYNCW) {
            p.w1 = a.fired_m1[rp >> 6];
            p.w2 = a.fired_m2[rp >> 6];
            p.w3 = a.fired_m3[rp >> 6];
            p.sn = a.sync_next[i];
            p.o0 = a.out_ptr[i];
            p.o1 = a.out_ptr[i + 1];
            p.sk = a.sync_k[i];
            if (a.push_marked) p.pa = a.pushany[rp];
        }
    };
    PrepIn cur, nxt;
    load_in((uint64_t)blockIdx.x * kBlock + threadIdx.x, cur);
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < nwords * 64; t += stride) {
        load_in(t + stride, nxt);
        const uint64_t i = t;
        const bool valid = i < a.n_own;
        const uint64_t rep = a.own0 + i;
        bool fire = false;
        uint8_t st = 0;  // sender state (SYNCW, streamed sync rounds)
        if (valid) {
            int64_t o0 = 0, o1 = 0;
            bool fm1 = false, fm2 = false, fm3 = false;
            if constexpr (SYNCW) {
                fm1 = (cur.w1 >> (rep & 63)) & 1;
                fm2 = (cur.w2 >> (rep & 63)) & 1;
                fm3 = (cur.w3 >> (rep & 63)) & 1;
                if (a.sstate)  // sender state for sync_records / expand_stream_sync (stored below)
                    st = (uint8_t)((cur.f & (FL_ACT | FL_LAG)) | (fm2 ? SE_FM2 : 0) | (fm3 ? SE_FM3 : 0));
            }
            if (!dense) {
                const uint8_t f = cur.f;
                // flg_cur still holds round r-2's flags: an F row written then is
                // stale in this round's F buffer; the expand kernel zeroes it unless
                // the node writes a new one, so F rows stay zero for inactive nodes.
                if (a.stream_ok) {
                    // sparse lean round: expand_stream takes the node (it reads and
                    // rewrites the old flag byte itself); no tile flags (node list)
                    // (double-buffered rounds: a node that changed in r-1 also moves its row forward)
                    if ((cur.fc & FL_ACT) || (a.db && (f & FL_ACT))) a.cand[rep] = CA_NODE;
                    c_bytes += 2;
                } else {
                    if (cur.fc & FL_ACT) {
                        a.zmark[rep] = 1;
                        a.tile_cand[i / a.tile_nodes] = 1;
                    }
                    a.flg_cur[rep] = 0;  // expand_round sets the flags of changed nodes
                    c_bytes += 3;
                }
                // candidates of this round
                if ((f & FL_LAG) || fm2) {
                    a.cand[rep] = CA_NODE;
                    if (!a.stream_ok) a.tile_cand[i / a.tile_nodes] = 1;
                }
                if (!(f & FL_ACT) && fm3 && a.push_marked) {
                    // the streamed callback of r-1 marked its push receivers itself
                    if (!cur.pa) st &= (uint8_t)~SE_FM3;
                    c_bytes += 1;
                } else if ((f & FL_ACT) || fm3) {  // senders mark their (owned) receivers
                    if constexpr (SYNCW) {
                        o0 = cur.o0;
                        o1 = cur.o1;
                    } else {
                        o0 = a.out_ptr[i];
                        o1 = a.out_ptr[i + 1];
                    }
                    const bool hub = a.hub_deg && o1 - o0 > (int64_t)a.hub_deg;
                    if (hub) o1 = o0;  // hub_mark does it
                    // a pusher that is not active reaches only the peers it pushed to
                    const bool only_pushed = !(f & FL_ACT) && a.pushb != nullptr;
                    c_bytes += 16 + (only_pushed ? 6 : 5) * (unsigned long long)(o1 - o0);
                    bool pushed = false;
                    constexpr int B = 8;  // a batch of columns and push bytes in flight together
                    for (int64_t e0 = o0; e0 < o1; e0 += B) {
                        uint64_t w[B];
                        uint8_t pb[B];
#pragma unroll
                        for (int b = 0; b < B; ++b) w[b] = e0 + b < o1 ? (uint64_t)(a.out_col[e0 + b] & kColMask) : ~0ull;
#pragma unroll
                        for (int b = 0; b < B; ++b) pb[b] = (only_pushed && e0 + b < o1) ? a.pushb[e0 + b] : (uint8_t)1;
#pragma unroll
                        for (int b = 0; b < B; ++b) {
                            if (e0 + b >= o1 || !pb[b]) continue;
                            pushed = true;
                            if (w[b] >= a.n_own) continue;  // a ghost: its owner marks it
                            a.cand[w[b]] = CA_NODE;
                            if (!a.stream_ok) a.tile_cand[w[b] / a.tile_nodes] = 1;
                        }
                    }
                    // a push that reached no peer with anything is no push: its
                    // receivers skip it, and nobody reads this node's set for it
                    if (only_pushed && !pushed && !hub) st &= (uint8_t)~SE_FM3;
                }
            }
            if constexpr (SYNCW) {
                if (a.sstate) a.sstate[rep] = st;
                o0 = cur.o0;
                o1 = cur.o1;
                // reads v sent in r-1 arrive now; each answered by a read_ok (:131)
                if (fm1) {
                    if constexpr (MASKW) {
                        for (int64_t e = o0; e < o1; ++e) {
                            const uint64_t w = a.out_col[e] & kColMask;
                            if (masked<MASKW>(a, 2, rep, w, e)) continue;
                            c_read_oks++;
                            if (masked<MASKW>(a, 3, w, rep, e)) c_dropped++;
                        }
                    } else {  // no window: every read arrives and is answered (a hub's list is long)
                        c_read_oks += (unsigned long long)(o1 - o0);
                    }
                }
                // (5) the sync timer (main.go:42-51): read RPC to every neighbour (:119-121)
                c_bytes += 4;
                if ((int64_t)cur.sn == a.round) {
                    fire = true;
                    c_fired++;
                    c_reads += (unsigned long long)(o1 - o0);
                    if constexpr (MASKW) {
                        for (int64_t e = o0; e < o1; ++e)
                            c_dropped += masked<MASKW>(a, 3, rep, a.out_col[e] & kColMask, e) ? 1 : 0;
                    }
                    const uint32_t kk = cur.sk + 1;
                    a.sync_k[i] = kk;
                    a.sync_next[i] = (int32_t)(a.round + gg_sync_interval_rcp(a.sync_mix, a.sync_rcp, gid_of(a, i), kk,
                                                                              a.sync_base, a.sync_jitter));
                }
            }
        }
        if constexpr (SYNCW) {  // before the first timer every fired word is still zero
            const unsigned long long word = __ballot(fire);
            if ((threadIdx.x & 63) == 0) a.fired_cur[(a.own0 + (i & ~63ull)) >> 6] = word;
            if (a.ibits) {
                const unsigned long long iw = __ballot((st & (FL_ACT | FL_LAG | SE_FM3)) != 0);
                if ((threadIdx.x & 63) == 0) a.ibits[(a.own0 + (i & ~63ull)) >> 6] = iw;
            }
        }
        cur = nxt;
    }
    if constexpr (SYNCW) {
        // ghost rows (sharded; whole waves over 64 consecutive ghost rows, ghost0 %
        // 64 == 0): the ghosts' own sync timers — the same pure function of (seed,
        // node id, k) their owner runs, so no fired bit crosses the exchange; not
        // counted here (the owner counts its reads) — and their sender states
        const uint64_t gw = (a.n_ghost + 63) / 64 * 64;
        for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < gw; g += stride) {
            const uint64_t row = a.ghost0 + g;
            uint8_t st = 0;
            bool fire = false;
            if (g < a.n_ghost) {
                if ((int64_t)a.sync_next[row] == a.round) {
                    fire = true;
                    const uint32_t kk = a.sync_k[row] + 1;
                    a.sync_k[row] = kk;
                    a.sync_next[row] = (int32_t)(a.round + gg_sync_interval_rcp(a.sync_mix, a.sync_rcp, gid_of(a, row), kk,
                                                                                a.sync_base, a.sync_jitter));
                }
                if (a.sstate) {
                    st = (uint8_t)((a.flg_prev[row] & (FL_ACT | FL_LAG)) | (bit_at(a.fired_m2, row) ? SE_FM2 : 0) |
                                   (bit_at(a.fired_m3, row) ? SE_FM3 : 0));
                    a.sstate[row] = st;
                }
            }
            const unsigned long long fw = __ballot(fire);
            if ((threadIdx.x & 63) == 0) a.fired_cur[row >> 6] = fw;
            if (a.sstate) {
                const unsigned long long iw = __ballot((st & (FL_ACT | FL_LAG | SE_FM3)) != 0);
                if ((threadIdx.x & 63) == 0) a.ibits[row >> 6] = iw;
            }
        }
    }
    // sharded: ghost senders (remote nodes, state from last round's exchange)
    // that were active or pushed mark their owned receivers
    if (!dense) {
        for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < a.n_ghost; g += stride) {
            const uint64_t row = a.ghost0 + g;
            bool fm3 = false;
            if constexpr (SYNCW) fm3 = bit_at(a.fired_m3, row);
            if (!((a.flg_prev[row] & FL_ACT) || fm3)) continue;
            for (int64_t e = a.gout_ptr[g]; e < a.gout_ptr[g + 1]; ++e) {
                const uint32_t w = a.gout_col[e];
                a.cand[w] = CA_NODE;
                if (!a.stream_ok) a.tile_cand[w / a.tile_nodes] = 1;
            }
        }
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    // node-level events happen once per node, not once per lane group
    acc[C_READS] = a.count_nodes ? c_reads : 0;
    acc[C_READ_OKS] = a.count_nodes ? c_read_oks : 0;
    acc[C_DROPPED] = a.count_nodes ? c_dropped : 0;
    acc[C_FIRED] = a.count_nodes ? c_fired : 0;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_PREP);
}

// Client broadcasts of this round mark their nodes (after round_prep).
// Grid-stride over a count read on the device (the grid does not depend on it).
__global__ void mark_injections(RoundArgs a) {
    const uint32_t n = inj_n(a);
    const uint32_t* p = inj_p(a);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const uint64_t i = p[2 * k];
        a.cand[a.own0 + i] |= CA_NODE | CA_INJ;  // same value from every thread of a node
        if (!a.stream_ok) a.tile_cand[i / a.tile_nodes] = 1;  // lean rounds use the node list
    }
}

// The lean digest's per-node targets: lreach[v] = the count of v's component
// label in tab = {n, then n (label, count) pairs by ascending label; n =
// kTabOverflow: too many labels, no target is reachable}. Labels absent from
// the table have no broadcast: target 0, which no changed set equals.
constexpr uint32_t kTabOverflow = ~0u;
__global__ void lreach_fill_tab(const uint32_t* lab, const uint32_t* tab, uint32_t* lreach, uint64_t n) {
    const uint32_t m = tab[0];
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t c = ~0u;
        if (m != kTabOverflow) {
            const uint32_t l = lab[v];
            uint32_t lo = 0, hi = m;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (tab[1 + 2 * mid] < l) lo = mid + 1;
                else hi = mid;
            }
            c = (lo < m && tab[1 + 2 * lo] == l) ? tab[2 + 2 * lo] : 0u;
        }
        lreach[v] = c;
    }
}
// owned rows' labels from the global label array (vertex parts: row -> id map)
__global__ void llab_gather(const uint32_t* glab, const uint32_t* gid, uint32_t* llab, uint64_t n) {
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        llab[v] = glab[gid[v]];
}
constexpr unsigned kMarkInjBlocks = 16;

// Sparse rounds: the candidate nodes -> node list (lean rounds, expand_stream;
// node-granular, so every node group gets the same share; kCompactQ groups of 8
// candidate bytes per thread, a coalesced pass over them), or the live tiles ->
// work list (expand_round; 8 tile flags per group, cleared for the next round).
// One atomic per block reserves the block's slots: same-address atomics are
// serialised in L2, so blocks cover 8 KB of candidate bytes each. Order is
// irrelevant: nodes/tiles are independent within a round and the counters are sums.
// Large graphs (more than kCompactSplit blocks) split it in three launches: the
// one same-address atomic per block serialises in L2 (~12 ns each), and once a
// sparse round's candidates are spread over most of the blocks — C5 at 2^26
// nodes: 8192 blocks, from round 3 on — compact_round took ~100 us whatever the
// count. PH 1 writes each block's count, compact_scan turns the counts into
// offsets (and the list length), PH 2 writes the list from them (blocks with
// nothing exit after one load). PH 0: the single launch with the atomic.
#ifndef GG_COMPACT_Q
#define GG_COMPACT_Q 4
#endif
constexpr int kCompactQ = GG_COMPACT_Q;
constexpr uint64_t kCompactSplit = 1024;
template <int PH>
__global__ __launch_bounds__(kBlock) void compact_round(RoundArgs a) {
    __shared__ uint32_t s_cnt[kBlock / 64];
    __shared__ uint32_t s_base;
    const unsigned long long t_start = clock100();
    // a round without round_prep: the first compaction launch sums the rings
    // (the split path's later launches read what it published)
    const bool dense = (a.prep_in_compact && PH != 2) ? (rings_in(a) || busy_prev(a)) : dense_round(a);
    // round r+1's counts start from zero (round r-1, their last user, is done)
    if (PH != 2 && blockIdx.x == 0 && threadIdx.x == 0 && a.n_work_next) a.n_work_next[0] = a.n_work_next[1] = 0;
    if (dense) {
        noop_exit(a, K_PREP, t_start);
        return;
    }
    if (PH == 2 && a.bcount[blockIdx.x + 1] == a.bcount[blockIdx.x]) {  // no candidate in this block
        if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
        return;
    }
    const bool nodes = a.stream_ok != 0;
    const uint64_t NG = a.tile_nodes;
    const uint64_t ntiles = (a.n_own + NG - 1) / NG;
    const uint64_t q0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * kCompactQ;  // first 8-byte group
    unsigned long long x[kCompactQ];  // 8 candidate bytes (nodes) or 8 tile flags (tiles) per group
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kCompactQ; ++j) {
        const uint64_t q = q0 + j;
        x[j] = 0;
        if (nodes) {
            const uint64_t n = q * 8;
            if (n + 8 <= a.n_own) {  // own0 is a multiple of 64: aligned
                x[j] = *reinterpret_cast<const unsigned long long*>(a.cand + a.own0 + n);
            } else {
                for (uint64_t k = n; k < a.n_own; ++k) x[j] |= (unsigned long long)a.cand[a.own0 + k] << (8 * (k - n));
            }
        } else if (q * 8 < ntiles) {
            x[j] = *reinterpret_cast<const unsigned long long*>(a.tile_cand + q * 8);
        }
    }
#pragma unroll
    for (int j = 0; j < kCompactQ; ++j) {
        const uint64_t q = q0 + j;
        if (!x[j]) continue;
        if (PH == 1) {
        } else if (!nodes) {
            *reinterpret_cast<unsigned long long*>(a.tile_cand + q * 8) = 0ull;
        } else if (a.nmeta) {  // streamed sync rounds: sync_records does not touch the bytes
            if (q * 8 + 8 <= a.n_own) *reinterpret_cast<unsigned long long*>(a.cand + a.own0 + q * 8) = 0ull;
            else
                for (uint64_t k = q * 8; k < a.n_own; ++k) a.cand[a.own0 + k] = 0;
        }
        const unsigned long long lo7 = 0x7f7f7f7f7f7f7f7full;
        c += (uint32_t)__popcll((((x[j] & lo7) + lo7) | x[j]) & ~lo7);  // non-zero bytes
    }
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
            const uint32_t v = s_cnt[w];
            s_cnt[w] = tot;
            tot += v;
        }
        if (PH == 0) s_base = tot ? atomicAdd(&a.n_work[nodes ? 1 : 0], tot) : 0u;
        else if (PH == 1) a.bcount[blockIdx.x] = tot;
        else s_base = a.bcount[blockIdx.x];
    }
    if (PH == 1) {
        if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
        return;
    }
    __syncthreads();
    uint32_t pos = s_base + s_cnt[wave] + incl - c;
    for (int j = 0; j < kCompactQ; ++j) {
        const uint64_t q = q0 + j;
        for (int t = 0; t < 8; ++t) {
            const uint32_t byte = (uint32_t)((x[j] >> (8 * t)) & 0xff);
            if (!byte) continue;
            if (nodes) {
                const uint32_t node = (uint32_t)(q * 8 + t);
                if (a.nmeta) {
                    const uint64_t rep = a.own0 + node;
                    a.nmeta[pos] = make_uint2(node, byte | ((uint32_t)a.flg_cur[rep] << 8) |
                                                        ((uint32_t)a.sstate[rep] << 16));
                }
                a.nodes[pos++] = node;
            } else {
                const uint64_t tile = q * 8 + t;
                const uint64_t n0 = tile * NG;
                const uint64_t n1 = n0 + NG < a.n_own ? n0 + NG : a.n_own;
                TileWork w;
                w.tile = (uint32_t)tile;
                w.eb = a.in_ptr[n0];
                w.ne = (uint32_t)(a.in_ptr[n1] - w.eb);
                a.work[pos++] = w;
            }
        }
    }
    if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
}

// Split compaction, middle launch: the nb per-block counts of compact_round<1>
// -> exclusive offsets in place, bcount[nb] = the list length (one block; each
// thread sums a contiguous run, a block scan, then the run is rewritten).
__global__ __launch_bounds__(1024) void compact_scan(RoundArgs a, uint32_t nb) {
    __shared__ uint32_t s_w[16];
    const unsigned long long t_start = clock100();
    if (dense_round(a)) {
        noop_exit(a, K_PREP, t_start);
        return;
    }
    const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    // 16-byte loads, four in flight, when a thread's run is 16-byte aligned (C5 at
    // 2^30 nodes: 128 counts a thread; one count per load made the pass latency-bound, ~200 us)
    const bool vec = (per & 3u) == 0;
    uint32_t sum = 0;
    uint32_t b = b0;
    if (vec) {
        const uint4* v4 = reinterpret_cast<const uint4*>(a.bcount);
        for (; b + 16 <= b1; b += 16) {
            const uint4 x0 = v4[b / 4], x1 = v4[b / 4 + 1], x2 = v4[b / 4 + 2], x3 = v4[b / 4 + 3];
            sum += x0.x + x0.y + x0.z + x0.w + x1.x + x1.y + x1.z + x1.w + x2.x + x2.y + x2.z + x2.w + x3.x + x3.y +
                   x3.z + x3.w;
        }
        for (; b + 4 <= b1; b += 4) {
            const uint4 x = v4[b / 4];
            sum += x.x + x.y + x.z + x.w;
        }
    }
    for (; b < b1; ++b) sum += a.bcount[b];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; ++w) {
            const uint32_t v = s_w[w];
            s_w[w] = t;
            t += v;
        }
        a.bcount[nb] = t;
        a.n_work[a.stream_ok ? 1 : 0] = t;
    }
    __syncthreads();
    uint32_t off = s_w[wave] + incl - sum;
    b = b0;
    if (vec) {
        uint4* v4 = reinterpret_cast<uint4*>(a.bcount);
        for (; b + 16 <= b1; b += 16) {
            uint4 x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = v4[b / 4 + q];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = x[q];
                x[q] = make_uint4(off, off + v.x, off + v.x + v.y, off + v.x + v.y + v.z);
                off += v.x + v.y + v.z + v.w;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) v4[b / 4 + q] = x[q];
        }
        for (; b + 4 <= b1; b += 4) {
            const uint4 v = v4[b / 4];
            v4[b / 4] = make_uint4(off, off + v.x, off + v.x + v.y, off + v.x + v.y + v.z);
            off += v.x + v.y + v.z + v.w;
        }
    }
    for (; b < b1; ++b) {
        const uint32_t v = a.bcount[b];
        a.bcount[b] = off;
        off += v;
    }
    if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
}

// ---------------------------------------------------------------------------
// expand_round. G lanes per node, WPL words per lane; SYNCW: sync events
// possible in r-3..r (timers fire from r >= sync_base); MASKW: some partition
// window covers r-3..r+1.
template <int G, int WPL, bool SYNCW, bool MASKW>
__device__ __forceinline__ void expand_body(const RoundArgs& a) {
    constexpr int NG = kBlock / G;  // nodes per tile
    constexpr int kBatch = 4;       // flags-first: contributing rows in flight per lane
    constexpr int kSpec = GG_SPEC_BATCH;  // busy lean rounds (W = 64): (flag, row) pairs in flight per lane
    constexpr int kPre = 64;        // worklist entries preloaded per chunk
    constexpr bool LEAN = !SYNCW && !MASKW;
    constexpr uint8_t L_PUSH = 1, L_LAG = 2, L_M3 = 4, L_M4 = 8;  // compacted-list flags (L_M3/L_M4: the
                                                                  // windows of r, r+1 cut the edge)
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
    unsigned long long c_new = 0, c_fwd = 0, c_hash = 0, c_active = 0, c_gathers = 0, c_nact = 0, c_bytes = 0;
    unsigned long long c_nactdeg = 0;
    // MASKW-only
    unsigned long long c_fwd_deliv = 0, c_push_deliv = 0, c_dropped = 0, c_next_ackdrop = 0;
    // SYNCW-only
    unsigned long long c_push = 0;

    if (LEAN && a.stream_ok) {  // expand_stream takes every lean round with nwp >= 2
        noop_exit(a, K_EXPAND, t_start);
        return;
    }
    // busy lean round (W = 64): load sender flags together with their rows
    // (speculative gathers; a row of an inactive sender is zero) instead of flags first
    const bool dense = LEAN && busy_round(a);

    const uint64_t n_work = *a.n_work;
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
            // row_ptr + col (+ one sender flag byte per edge) + per-node cand/zmark/flag bytes
            if (threadIdx.x == 0) c_bytes += 8ull * (NG + 1) + (dense ? 4ull : 5ull) * tw.ne + 3ull * NG;
            lds_barrier();

            if (zm && !ca) {  // only the stale F row to clear
                {
                    Row<WPL> z;
#pragma unroll
                    for (int w = 0; w < WPL; ++w) z.w[w] = 0;
                    store_row<WPL>(a.F_cur + rep * a.nwp + off, z);
                }
                if (lg == 0) {
                    a.zmark[rep] = 0;
                    c_bytes += 8ull * a.nwp;
                }
            }
            if (ca) {
                unsigned long long nrows = 0, nextra = 0;  // rows moved / other bytes for this node
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
                    sp = load_row<WPL>(a.base + rep * a.nwp + off);
                    if (lag) {
                        const Row<WPL> f = load_row<WPL>(a.F_prev + rep * a.nwp + off);
#pragma unroll
                        for (int w = 0; w < WPL; ++w) sp.w[w] |= f.w[w];
                    }
                    S = sp;
                    nrows += lag ? 2 : 1;
                    // (1) client broadcasts of this round
                    if (has_inj) {
                        uint32_t lo = 0, hi = inj_n(a);
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (inj_p(a)[2 * mid] < (uint32_t)i) lo = mid + 1;
                            else hi = mid;
                        }
                        for (uint32_t k = lo; k < inj_n(a) && inj_p(a)[2 * k] == (uint32_t)i; ++k) {
                            const uint32_t lane = inj_p(a)[2 * k + 1];
                            const uint32_t word = lane >> 6;
                            if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
                        }
                    }
                };
                // (2) first deliverer claims, ascending sender
                // mb: bit 0 = v's forward of round r to u dropped, bit 1 = u's ack of r+1 dropped
                auto claim = [&](const Row<WPL>& src, uint32_t c, uint32_t mb) {
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
                            if (!(mb & 1u)) {
                                cl_deliv += pc;
                                if (mb & 2u) cl_ackdrop += pc;
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
                    nrows += (unsigned long long)(k1 - k0);  // every sender row and flag byte
                    nextra += (unsigned long long)(k1 - k0);
                    {
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
                                    claim(src[b], cb[b], 0u);
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
                        const uint64_t ei = (uint64_t)(eb + k);
                        const bool drop = masked<MASKW>(a, 2, u, rep, ei);  // sent in r-1
                        if constexpr (SYNCW) keep |= (ef & SE_FM2) != 0;  // u's callback reads v now
                        const bool p = !drop && is_push<SYNCW, MASKW>(a, ef, u, rep, ei);
                        if (!drop && ((ef & SE_ACT) || p)) {
                            need = true;
                            if (staged) {  // every lane of the group writes the same entry
                                s_col[k0 + m] = c;
                                s_ef[k0 + m] = (p ? L_PUSH : 0) | ((ef & SE_LAG) ? L_LAG : 0) |
                                               (masked<MASKW>(a, 3, rep, u, ei) ? L_M3 : 0) |
                                               (masked<MASKW>(a, 4, u, rep, ei) ? L_M4 : 0);
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
                            nrows += (unsigned long long)m;
                            for (int b0 = 0; b0 < m; b0 += kBatch) {
                                uint32_t cb[kBatch];
                                uint8_t lfs[kBatch];
                                Row<WPL> src[kBatch];
#pragma unroll
                                for (int b = 0; b < kBatch; ++b) {
                                    const bool v = b0 + b < m;
                                    cb[b] = v ? s_col[k0 + b0 + b] : 0u;
                                    const uint8_t lf = v ? s_ef[k0 + b0 + b] : 0;
                                    lfs[b] = lf;
                                    if (v) {
                                        src[b] = sender_row(cb[b], lf & L_PUSH, lf & L_LAG);
                                    } else {
#pragma unroll
                                        for (int w = 0; w < WPL; ++w) src[b].w[w] = 0;
                                    }
                                }
#pragma unroll
                                for (int b = 0; b < kBatch; ++b) claim(src[b], cb[b], (uint32_t)(lfs[b] >> 2));
                            }
                        } else {
                            for (int64_t k = k0; k < k1; ++k) {  // hub slow path
                                const uint32_t c = a.in_col[eb + k];
                                const uint64_t u = c & kColMask;
                                const uint8_t ef = sender_flags<SYNCW>(a, u);
                                const uint64_t ei = (uint64_t)(eb + k);
                                if (masked<MASKW>(a, 2, u, rep, ei)) continue;
                                const bool p = is_push<SYNCW, MASKW>(a, ef, u, rep, ei);
                                if (!(ef & SE_ACT) && !p) continue;
                                c_gathers += (lg == 0) ? 1ull : 0ull;
                                nrows++;
                                claim(sender_row(c, p, (ef & SE_LAG) != 0), c,
                                      (masked<MASKW>(a, 3, rep, u, ei) ? 1u : 0u) |
                                          (masked<MASKW>(a, 4, u, rep, ei) ? 2u : 0u));
                            }
                        }
                        // (3) sync callback: v fired in r-2, read_oks of peers in ascending order
                        if constexpr (SYNCW) {
                            if (callback) {
                                const int64_t o0 = a.out_ptr[i], o1 = a.out_ptr[i + 1];
                                for (int64_t e = o0; e < o1; ++e) {
                                    const uint64_t w = a.out_col[e] & kColMask;
                                    if (masked<MASKW>(a, 1, rep, w, e) || masked<MASKW>(a, 2, w, rep, e)) {
                                        if (a.pushb && lg == 0) a.pushb[e] = 0;  // no callback: no push
                                        continue;
                                    }
                                    const Row<WPL> R =
                                        sender_row((uint32_t)w, true, (a.flg_prev[w] & FL_LAG) != 0);
                                    nrows++;
                                    nextra += 13;  // out_col + flag
                                    unsigned long long pn = 0, pp = 0;
#pragma unroll
                                    for (int q2 = 0; q2 < WPL; ++q2) {
                                        pn += __popcll(R.w[q2] & ~S.w[q2]);
                                        pp += __popcll(S.w[q2] & ~R.w[q2]);
                                        S.w[q2] |= R.w[q2];
                                    }
                                    if (a.pushb) {  // did this peer get any push (next round's receivers)
                                        const bool nz = ((__ballot(pp != 0) >> gshift) & gmask) != 0;
                                        if (lg == 0) a.pushb[e] = nz ? 1 : 0;
                                    }
                                    cb_new += pn;
                                    push_sent += pp;
                                    if (!masked<MASKW>(a, 3, rep, w, e)) {
                                        cb_new_deliv += pn;
                                        push_deliv += pp;
                                        if (masked<MASKW>(a, 4, w, rep, e)) {
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
                    const uint64_t g = gid_of(a, i);
#pragma unroll
                    for (int w = 0; w < WPL; ++w) {
                        F.w[w] = S.w[w] & ~sp.w[w];
                        T += __popcll(F.w[w]);
                        if (F.w[w]) {  // seen_hash: the round's new bits of a word
                            const uint64_t idx = g * a.nw + a.word0 + off + w;
                            c_hash += gg_word_hash(idx, F.w[w]);
                        }
                    }
                    const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
                    if (any || zm) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
                    if (zm && lg == 0) a.zmark[rep] = 0;
                    nrows += (any || zm) ? 1 : 0;
                    if (keep) {
                        if (lag) store_row<WPL>(a.base + rep * a.nwp + off, sp);
                        nrows += lag ? 1 : 0;
                    } else if (any || lag) {
                        store_row<WPL>(a.base + rep * a.nwp + off, S);
                        nrows++;
                    }
                    if (lg == 0 && any) a.flg_cur[rep] = (uint8_t)(FL_ACT | (keep ? FL_LAG : 0));
                    c_nact += (lg == 0 && any) ? 1ull : 0ull;
                    c_nactdeg += (lg == 0 && any) ? deg : 0ull;

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
                                if (!masked<MASKW>(a, 3, rep, w, e)) {
                                    U++;
                                    if (masked<MASKW>(a, 4, w, rep, e)) AD++;
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
                if (!work && zm) {  // a candidate whose senders were all dropped: still
                    Row<WPL> z;     // clear its stale F row (rows of inactive nodes are zero)
#pragma unroll
                    for (int w = 0; w < WPL; ++w) z.w[w] = 0;
                    store_row<WPL>(a.F_cur + rep * a.nwp + off, z);
                    if (lg == 0) a.zmark[rep] = 0;
                    nrows++;
                }
                if (lg == 0) c_bytes += nrows * 8ull * a.nwp + nextra + 16;  // + out_ptr
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
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_EXPAND);
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
// expand_stream: every lean round (no sync events in expand, no masks) with
// nwp >= 2 (expand_stream1 below: nwp = 1). Dense rounds (dense_round) visit EVERY node; sparse ones the
// candidate-node list of compact_round. No tiles, no barriers: node group q (G
// lanes) walks items q, q + n_groups, ... with a software pipeline — while
// item k's own row and sender rows land in its wave's LDS slots by DMA, item
// k+1's column list, item k+2's row pointers and bytes and item k+3's list
// entry are already in flight — so each node costs about one memory round
// trip. F rows of inactive senders are zero, so every sender row is claimed
// without looking at sender flags, and a node nobody reached finds no new
// bits. The node-local part of round_prep (stale F row of round r-2, flag
// reset) is done here from the node's old flag byte.
// Which of a batch's D senders (columns c, the first n valid) were ACT last
// round (flags-first rounds): lane lg of the node group looks up senders lg,
// lg + G, ... in the abits bitmap and a ballot assembles the group's D-bit
// mask, which every lane of the group gets. All lanes of a group call it.
template <int G, int D>
__device__ __forceinline__ uint32_t active_senders(const uint64_t* abits, const uint32_t (&c)[D], uint32_t n, int lg,
                                                   int gbase) {
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < (D + G - 1) / G; ++q) {
        const int b = lg + q * G;
        uint32_t col = 0;
#pragma unroll
        for (int bb = 0; bb < D; ++bb) col = (bb == b) ? c[bb] : col;
        const bool act = b < D && (uint32_t)b < n && bit_at(abits, col & kColMask);
        const unsigned long long w = __ballot(act);
        const unsigned long long gm = (G >= 64) ? ~0ull : ((1ull << G) - 1ull);
        m |= (uint32_t)((w >> gbase) & gm) << (q * G);
    }
    return m & ((1u << D) - 1u);
}

template <int G, int WPL, bool MASKW, bool DB = false, bool MARK = false, int D = kStreamRows>
__device__ __forceinline__ void stream_body(RoundArgs a) {
    static_assert(WPL == 2, "DMA slots hold 16 bytes per lane");
    constexpr int NGB = kBlock / G;  // node groups per block
    // D: sender rows per DMA batch
    __shared__ __attribute__((aligned(16))) uint8_t s_slots[(kBlock / 64) * (D + 1) * 1024];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    // round r-1's rings: summed by the marking kernel in rounds with block lists
    // (launched first: the other kernel reads what its block 0 published)
    const RingView rv = ring_view<MARK>(a);
    const bool busy = busy_count(a, rv.act);
    // marking rounds launch two kernels: expand_stream_db takes the busy ones
    // (every node, nothing marked) and expand_stream_db_mark the others (the
    // candidate list, or every node after a busy round; the next round's
    // candidates marked) — or only the one the host expects (solo), which then
    // takes the round whatever it finds
    if (!a.stream_ok || (!a.solo && (MARK ? busy : (DB && a.mark_cand && !busy)))) {
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    // dense_round(): a round without round_prep after a round whose expand marked
    // nothing (busy, or a solo expand_stream_db) is dense too; a solo
    // expand_stream_db round is dense (it has no candidate list)
    const bool prev_unmarked = a.prev_mark ? a.prev_mark == 2 : busy_count(a, rv.act_m2);  // busy_prev()
    const bool dense = busy || a.no_list || (DB && !MARK && a.solo) || (a.prep_in_compact && prev_unmarked);
    // block lists (sparse rounds without compact_round): thread t of block b
    // takes the 16 nodes of granule t * grid + b (one 16-byte load of candidate
    // bytes; the host sizes the grid so 256 granules a block cover every node),
    // the block lists their candidates in LDS by a block scan and its node
    // groups walk that list. Granules interleaved over the blocks: the wave
    // fronts of sparse rounds are runs of consecutive nodes (C2, a tree in BFS
    // order: subtrees), which contiguous slices left to a few blocks (rounds
    // 4-9 took 2x as long)
    // (marking kernel only: the host sets block_lists in marking rounds, where the
    // other kernel takes only busy, dense rounds)
    const bool bl = MARK && a.block_lists && !dense;
    __shared__ uint16_t s_list[kBllMax];
    __shared__ uint32_t s_lcnt[kBlock / 64];
    uint32_t n_items = dense ? (uint32_t)a.n_own : 0u;
    if (bl) {
        const uint64_t n16 = ((uint64_t)threadIdx.x * gridDim.x + blockIdx.x) * 16;  // rows: a multiple of 64
        const uint32_t t16 = threadIdx.x * 16;
        ulonglong2 x = make_ulonglong2(0ull, 0ull);
        if (n16 < a.n_own) x = *reinterpret_cast<const ulonglong2*>(a.cand + a.own0 + n16);
        const unsigned long long lo7 = 0x7f7f7f7f7f7f7f7full;
        unsigned long long m0 = (((x.x & lo7) + lo7) | x.x) & ~lo7, m1 = (((x.y & lo7) + lo7) | x.y) & ~lo7;
        const uint32_t c = (uint32_t)(__popcll(m0) + __popcll(m1));
        const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (ln >= o) incl += y;
        }
        if (ln == 63) s_lcnt[wv] = incl;
        __syncthreads();
        uint32_t pos = incl - c, tot = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            const uint32_t v = s_lcnt[w];
            pos += w < wv ? v : 0u;
            tot += v;
        }
        for (; m0; m0 &= m0 - 1) s_list[pos++] = (uint16_t)(t16 + (__ffsll(m0) - 1) / 8);
        for (; m1; m1 &= m1 - 1) s_list[pos++] = (uint16_t)(t16 + 8 + (__ffsll(m1) - 1) / 8);
        __syncthreads();
        n_items = tot;
    } else if (!dense) {
        n_items = a.n_work[1];
    }
    // list entry t * 16 + j: node j of thread t's granule
    auto bl_node = [&](uint32_t x) -> uint32_t { return ((x >> 4) * gridDim.x + blockIdx.x) * 16u + (x & 15u); };
    if (bl ? n_items == 0 : (uint64_t)blockIdx.x * NGB >= n_items) {  // sparse round: no item reaches this block
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    const bool ff = !MASKW && ff_view(a, rv);  // flags-first gathers (block-uniform)
    // nothing can arrive (all_full()): no gathers, no own rows
    const bool full = !MASKW && a.tot && inj_n(a) == 0 && rv.tot == a.full_new;
    if (DB && !MASKW && full) {
        // an all-full double-buffered round (e.g. the quiescence round that ends an
        // episode): every owned set is the universe, row 0's, so nothing arrives
        // and a node's only work is moving that row forward if its row in this
        // buffer is two rounds old (ACT in r-1), and its flag and candidate bytes.
        // No gathers: U nodes a group per iteration, their bytes loaded together
        // (the general loop below pays a memory round trip per node)
        const int lg = threadIdx.x % G;
        const uint32_t off = (uint32_t)lg * WPL, stride = bl ? (uint32_t)NGB : gridDim.x * NGB;
        const uint32_t k = (bl ? 0u : blockIdx.x * NGB) + threadIdx.x / G;
        auto node_of = [&](uint32_t q) -> uint32_t {
            return q < n_items ? (dense ? q : (bl ? bl_node(s_list[q]) : a.nodes[q])) : ~0u;
        };
        Row<WPL> U0;
        {
            const ulonglong2 u = *reinterpret_cast<const ulonglong2*>(a.base_prev + a.own0 * a.nwp + off);
            U0.w[0] = u.x;
            U0.w[1] = u.y;
        }
        constexpr int U = 4;
        uint32_t c_act = 0;
        unsigned long long c_by = 0;
        for (uint32_t kk = k; kk < n_items; kk += U * stride) {
            uint32_t nd[U];
            uint8_t fl[U], ca[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nd[u] = node_of(kk + u * stride);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                fl[u] = ca[u] = 0;
                if (nd[u] != ~0u) {
                    fl[u] = a.flg_prev[a.own0 + nd[u]];
                    ca[u] = a.cand[a.own0 + nd[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (nd[u] == ~0u) continue;
                const uint64_t rep = a.own0 + nd[u];
                if (fl[u] & FL_ACT) {
                    store_row_nt(a.base + rep * a.nwp + off, U0);
                    c_by += 16;
                }
                if (lg == 0) {
                    a.flg_cur[rep] = 0;
                    if (ca[u]) a.cand[rep] = 0;
                    if (MARK && fl[u]) a.flg_prev_w[rep] = 0;
                    c_act += 1;
                    c_by += (dense ? 0 : 4) + 8 + 2 + 1;
                }
            }
        }
        unsigned long long acc[C_NUM];
#pragma unroll
        for (int q = 0; q < C_NUM; ++q) acc[q] = 0;
        acc[C_ACTIVE] = c_act;
        acc[C_BYTES] = c_by;
        flush_counters(a, acc, s_red, t_start, K_STREAM);
        return;
    }
    // double-buffered round: own and sender rows are sets of r-1 (base_prev); in a
    // lean round without a dropped message so far a sender's set holds nothing new
    // for v beyond its F row (it forwarded every older value to v), so claims are
    // unchanged, and no F row is written
    constexpr bool db = DB && !MASKW;  // a kernel of its own: the F-row kernel keeps its registers
    const uint64_t* const rows_in = db ? a.base_prev : a.F_prev;
    constexpr uint32_t kAllD = (1u << D) - 1u;
    // per-lane counts that fit 32 bits stay 32-bit (register budget)
    uint32_t c_new = 0, c_active = 0, c_gathers = 0, c_nact = 0, c_nactdeg = 0;
    unsigned long long c_fwd = 0, c_hash = 0, c_bytes = 0;
    unsigned long long c_fwd_deliv = 0, c_dropped = 0, c_next_ackdrop = 0;  // MASKW
    const int lg = threadIdx.x % G;
    const uint32_t off = (uint32_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const int gbase = (int)(threadIdx.x & 63) - lg;  // the node group's first lane in the wave
    // sharded engines: a ghost sender's row is its F row either way (the exchange
    // ships F rows), so the sender row's buffer is chosen per sender
    auto sender_row = [&](uint32_t c) -> const uint64_t* {
        const uint64_t u = c & kColMask;
        return ((db && u >= a.ghost0 && a.n_ghost) ? a.F_prev : rows_in) + u * a.nwp + off;
    };
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    uint8_t* const my = &s_slots[(threadIdx.x >> 6) * (D + 1) * 1024];
    const uint32_t lane16 = (threadIdx.x & 63) * 16;
    const uint32_t stride = bl ? (uint32_t)NGB : gridDim.x * NGB;
    const unsigned long long rowb = 8ull * a.nwp;

    // node ids are < 2^31 (gg_create), so 32-bit ids and in-degrees keep the
    // three in-flight items within the 5-waves/SIMD register budget
    struct Meta {
        int64_t p0;
        uint32_t deg, node;
        uint8_t ca, fl;
    };
    constexpr uint32_t kNone = ~0u;
    constexpr uint32_t kHubBit = 0x80000000u;  // node ids < 2^31
    auto node_of = [&](uint32_t k) -> uint32_t {
        return k < n_items ? (dense ? (uint32_t)k : (bl ? bl_node(s_list[k]) : a.nodes[k])) : kNone;
    };
    auto fetch_meta = [&](uint32_t n, Meta& m) {
        m.node = n;
        if (n < a.n_own) {
            m.p0 = a.in_ptr[n];
            m.deg = (uint32_t)(a.in_ptr[n + 1] - m.p0);
            m.ca = a.cand[a.own0 + n];      // CA_INJ: client broadcasts this round
            // flags of round r-2 (ACT: stale F row), or in double-buffered rounds of
            // r-1 (ACT: the row in this round's set buffer is two rounds old)
            m.fl = (db ? a.flg_prev : a.flg_cur)[a.own0 + n];
            if (full) m.deg = 0;
            if (a.hub_deg && m.deg > a.hub_deg) {  // a hub: hub_chunks/hub_finish take it
                m.node |= kHubBit;
                m.deg = 0;
            }
        } else {
            m.p0 = 0;
            m.deg = 0;
            m.ca = m.fl = 0;
        }
    };
    auto fetch_cols = [&](const Meta& m, uint32_t (&c)[D]) {
#pragma unroll
        for (int b = 0; b < D; ++b)
            c[b] = ((uint32_t)b < m.deg) ? a.in_col[m.p0 + b] : 0u;
    };
    // the lean digest's byte of an item, loaded with its columns one stage
    // ahead (a load in fetch_meta made it wait for the candidate byte early: +5 %
    // on C4's dense rounds); applied before the item's row DMAs
    auto fetch_sat = [&](const Meta& m) -> uint32_t {
        if constexpr (MASKW) return 0u;
        return (a.lsat && !(m.node & kHubBit) && m.node < a.n_own) ? (uint32_t)a.lsat[a.own0 + m.node] : 0u;
    };

    uint32_t k = (bl ? 0u : blockIdx.x * NGB) + threadIdx.x / G;
    // an all-full double-buffered round: every owned set is row 0's, so each lane
    // puts its chunk of it in its own-row LDS slot once (no own-row DMA overwrites
    // it) instead of every node DMA-ing the same row, and the loop only writes the
    // rows moving forward
    if (db && full)
        *reinterpret_cast<ulonglong2*>(my + D * 1024 + lane16) =
            *reinterpret_cast<const ulonglong2*>(a.base_prev + a.own0 * a.nwp + off);
    Meta m0, m1;
    uint32_t c0[D], c1[D];
    const uint32_t n0 = node_of(k), n1 = node_of(k + stride);
    uint32_t n2 = node_of(k + 2 * stride);
    vm_drain();
    fetch_meta(n0, m0);
    fetch_meta(n1, m1);
    vm_drain();
    fetch_cols(m0, c0);
    uint32_t s0 = fetch_sat(m0), s1 = 0;
    vm_drain();  // nothing pending at the loop head: no compiler drains inside
    for (; k < n_items; k += stride) {
        // saturated (lsat_skip) and no client broadcast: no gathers, no forwards, marks nobody
        if (s0 && !(m0.ca & CA_INJ)) m0.deg = 0;
        const bool hub = (m0.node & kHubBit) != 0;
        const uint64_t i = m0.node & ~kHubBit;
        const uint64_t rep = a.own0 + i;
        // (a) DMA node i's own row and its first D sender rows (masked rounds:
        // and the words of the window bitmaps covering its first D in-edges)
        // (an all-full double-buffered round: every owned set is the same, row 0's)
        if (!hub && !full) dma16((const void*)((db ? a.base_prev : a.base) + rep * a.nwp + off), my + D * 1024);
        // the lean digest's target, loaded with the DMAs (waited for with them)
        const uint32_t tgt = (!MASKW && a.lreach && a.lmark && !hub) ? a.lreach[rep] : a.lusat;
        uint64_t mw[3][2];
        if constexpr (MASKW) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const uint64_t* eb = a.ebits[2 + q];
                mw[q][0] = (eb && m0.deg) ? eb[m0.p0 >> 6] : 0ull;
                mw[q][1] = (eb && m0.deg) ? eb[(m0.p0 + D - 1) >> 6] : 0ull;
            }
        }
        const uint32_t am0 = ff ? active_senders<G, D>(a.abits, c0, m0.deg, lg, gbase) : kAllD;
#pragma unroll
        for (int b = 0; b < D; ++b) {
            if ((uint32_t)b < m0.deg && ((am0 >> b) & 1u))
                dma16((const void*)sender_row(c0[b]), my + b * 1024);
        }
        // (b) prefetch: columns of item k+stride, row pointers of item k+2*stride,
        // list entry of item k+3*stride
        Meta m2;
        fetch_cols(m1, c1);
        s1 = fetch_sat(m1);
        fetch_meta(n2, m2);
        const uint32_t n3 = node_of(k + 3 * stride);
        vm_drain();
        if (!hub) {
        Row<WPL> sp, S;
        sp.w[0] = sp.w[1] = 0;
        if (!full || db) {
            const ulonglong2 o = *reinterpret_cast<const ulonglong2*>(my + D * 1024 + lane16);
            sp.w[0] = o.x;  // lean rounds precede every sync timer: no LAG
            sp.w[1] = o.y;
        }
        S = sp;
        if (m0.ca & CA_INJ) {  // (1) client broadcasts of this round
            uint32_t lo = 0, hi = inj_n(a);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (inj_p(a)[2 * mid] < (uint32_t)i) lo = mid + 1;
                else hi = mid;
            }
            for (uint32_t q = lo; q < inj_n(a) && inj_p(a)[2 * q] == (uint32_t)i; ++q) {
                const uint32_t lane = inj_p(a)[2 * q + 1];
                const uint32_t word = lane >> 6;
                if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
            }
        }
        // (2) node broadcasts, ascending sender: first deliverer claims.
        // Masked rounds: a sender whose message of r-1 was dropped is skipped;
        // claims of reciprocal senders count as delivered forwards unless v's
        // own forwards to them in r are dropped (bit in window r), and their
        // acks in r+1 as dropped when window r+1 separates them.
        unsigned long long cl_recip = 0, cl_deliv = 0, cl_ackdrop = 0;
        uint32_t n_m3 = 0, n_ad = 0;  // out-neighbours (= in, symmetric) cut in r; of the rest, cut in r+1
        auto claim = [&](uint64_t x0, uint64_t x1, uint32_t c, uint32_t mb) {
            if constexpr (MASKW) {
                if (mb & 1) return;  // dropped in flight
                const uint64_t w0 = x0 & ~S.w[0], w1 = x1 & ~S.w[1];
                S.w[0] |= w0;
                S.w[1] |= w1;
                if (c & kRecipBit) {
                    const unsigned long long pc = __popcll(w0) + __popcll(w1);
                    cl_recip += pc;
                    if (!(mb & 2)) {
                        cl_deliv += pc;
                        if (mb & 4) cl_ackdrop += pc;
                    }
                }
            } else {
                const uint64_t w0 = x0 & ~S.w[0], w1 = x1 & ~S.w[1];
                S.w[0] |= w0;
                S.w[1] |= w1;
                if (c & kRecipBit) cl_recip += __popcll(w0) + __popcll(w1);
            }
        };
        // bit b of the three window masks (r-1, r, r+1) for sender slot b of a batch at edge e0
        auto mask_bits = [&](uint64_t (&w)[3][2], int64_t e0, int b) -> uint32_t {
            uint32_t mb = 0;
            if constexpr (MASKW) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const uint64_t e = (uint64_t)(e0 + b);
                    const uint64_t word = ((e >> 6) == ((uint64_t)e0 >> 6)) ? w[q][0] : w[q][1];
                    mb |= (uint32_t)((word >> (e & 63)) & 1ull) << q;
                }
            }
            return mb;
        };
#pragma unroll
        for (int b = 0; b < D; ++b) {
            if ((uint32_t)b < m0.deg && ((am0 >> b) & 1u)) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(my + b * 1024 + lane16);
                uint32_t mb = 0;
                if constexpr (MASKW) {
                    mb = mask_bits(mw, m0.p0, b);
                    n_m3 += (mb >> 1) & 1;
                    n_ad += ((mb >> 1) & 1) ? 0u : ((mb >> 2) & 1);
                }
                claim(x.x, x.y, c0[b], mb);
            }
        }
        const int64_t p1 = m0.p0 + m0.deg;
        if (MASKW) {
            if (lg == 0) c_gathers += m0.deg;  // every sender row
        } else if (lg == 0) {
            c_gathers += __popc(am0 & (m0.deg >= (uint32_t)D ? kAllD : ((1u << m0.deg) - 1u)));
        }
        for (int64_t e = m0.p0 + D; e < p1; e += D) {  // more than D senders
            uint32_t cb[D];
#pragma unroll
            for (int b = 0; b < D; ++b) cb[b] = e + b < p1 ? a.in_col[e + b] : 0u;
            // one wait for the columns: the compiler cannot see the DMAs below, so
            // without it each DMA would get a vmcnt(0) of its own (serialising them)
            vm_drain();
            // flags-first: only the active senders' rows (bits looked up first)
            const uint32_t am = ff ? active_senders<G, D>(a.abits, cb, (uint32_t)(p1 - e), lg, gbase) : kAllD;
#pragma unroll
            for (int b = 0; b < D; ++b) {
                if (e + b < p1 && ((am >> b) & 1u))
                    dma16((const void*)sender_row(cb[b]), my + b * 1024);
            }
            uint64_t ew[3][2];
            if constexpr (MASKW) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const uint64_t* eb = a.ebits[2 + q];
                    ew[q][0] = eb ? eb[e >> 6] : 0ull;
                    ew[q][1] = eb ? eb[(e + D - 1) >> 6] : 0ull;
                }
            }
            vm_drain();
#pragma unroll
            for (int b = 0; b < D; ++b) {
                if (e + b < p1 && ((am >> b) & 1u)) {
                    const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(my + b * 1024 + lane16);
                    uint32_t mb = 0;
                    if constexpr (MASKW) {
                        mb = mask_bits(ew, e, b);
                        n_m3 += (mb >> 1) & 1;
                        n_ad += ((mb >> 1) & 1) ? 0u : ((mb >> 2) & 1);
                    }
                    claim(x.x, x.y, cb[b], mb);
                }
            }
            if (!MASKW && lg == 0) c_gathers += __popc(am & ((p1 - e >= D) ? kAllD : ((1u << (uint32_t)(p1 - e)) - 1u)));
        }
        const unsigned long long nin = m0.deg;
        // new state
        Row<WPL> F;
        uint32_t T = 0;
        const uint64_t g = gid_of(a, i);
#pragma unroll
        for (int w = 0; w < WPL; ++w) {
            F.w[w] = S.w[w] & ~sp.w[w];
            T += __popcll(F.w[w]);
            if (F.w[w]) {
                const uint64_t idx = g * a.nw + a.word0 + off + w;
                c_hash += gg_word_hash(idx, F.w[w]);
            }
        }
        const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
        if (!MASKW && any && a.lsat && a.lmark) lsat_mark<G, WPL>(a, S, rep, lg, tgt);
        const bool zm = !db && (m0.fl & FL_ACT) != 0;  // F row of round r-2 in this buffer
        // rows written this round are read next round from HBM anyway (F by
        // other nodes' gathers, base by this node): streamed past the caches,
        // they leave L2 to the gathers (C2 -2.5%, C3 -1.4% kernel time)
        // per lane, only the 16-byte chunks that changed: a chunk without new bits
        // keeps its base bytes, and its F bytes are already zero unless the node's
        // F row of round r-2 sits in this buffer (zm: then every chunk is written).
        // While most nodes learn a few of W values (C2 rounds 10-13: 15-66 % of
        // the chunks change) this drops most of the row stores of a dense round
        const bool lane_new = (F.w[0] | F.w[1]) != 0;
        const bool cp = db && (m0.fl & FL_ACT) != 0;  // db: this buffer's row is two rounds old
        if (db) {
            if (lane_new || cp) store_row_nt(a.base + rep * a.nwp + off, S);
        } else {
            if (lane_new || zm) store_row_nt(a.F_cur + rep * a.nwp + off, F);
            if (lane_new) store_row_nt(a.base + rep * a.nwp + off, S);
        }
        if (lg == 0) {
            // (double-buffered: the flag byte of r-2 is not known here, so always)
            if (any || db || m0.fl) a.flg_cur[rep] = any ? FL_ACT : 0;
            if (m0.ca) a.cand[rep] = 0;
        }
        const unsigned long long deg = a.symmetric ? nin : (unsigned long long)(a.out_ptr[i + 1] - a.out_ptr[i]);
        if constexpr (db && MARK) {
            {
                // round r+1's candidates, marked here instead of by a round_prep pass
                // over every flag byte: a node whose set changed moves its row forward
                // and is a sender (its receivers). Its flag byte of r-1 was read above
                // (m0.fl) and is not read again: cleared, so no stale ACT byte waits
                // for round r+1 to clear it (that round's round_prep would mark it)
                if (lg == 0 && m0.fl) a.flg_prev_w[rep] = 0;
                if (any) {  // (symmetric: mark_ok) the out-list is the in-list
                    if (lg == 0) a.cand_next[rep] = CA_NODE;
                    const uint32_t* oc = a.in_col + m0.p0;
                    for (uint32_t e = (uint32_t)lg; e < m0.deg; e += G) a.cand_next[oc[e] & kColMask] = CA_NODE;
                }
            }
        }
        c_new += T;
        const unsigned long long fs = deg * (unsigned long long)T - cl_recip;
        c_fwd += fs;
        if constexpr (MASKW) {  // symmetric only (host): out-neighbours = in-neighbours
            const unsigned long long fd = (deg - n_m3) * (unsigned long long)T - cl_deliv;
            c_fwd_deliv += fd;
            c_dropped += fs - fd;
            c_next_ackdrop += (unsigned long long)n_ad * T - cl_ackdrop;
        }
        if (lg == 0) {
            c_active += 1;
            c_nact += any ? 1 : 0;
            if constexpr (!MASKW) c_nactdeg += any ? (uint32_t)deg : 0u;  // masked rounds: no flags-first next
            // row_ptr + cand + flag bytes + col (+ a sender bit, flags-first), own row + gathered
            // sender rows, F / base / flag writes
            c_bytes += (dense ? 0 : 4) + 8 + 2 + (db ? 1 : 0) + 4 * nin + (ff ? (nin + 7) / 8 : 0) +
                       (full ? 0 : rowb) + (any ? 1 : 0) + ((MARK && any) ? nin + 1 : 0);
        }
        // this lane's F / base chunk stores
        c_bytes += db ? ((lane_new || cp) ? 16 : 0) : ((lane_new || zm) ? 16 : 0) + (lane_new ? 16 : 0);
        }  // !hub
        m0 = m1;
        s0 = s1;
        m1 = m2;
        n2 = n3;
#pragma unroll
        for (int b = 0; b < D; ++b) c0[b] = c1[b];
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    if constexpr (!MASKW) c_fwd_deliv = c_fwd;
    c_bytes += (unsigned long long)c_gathers * rowb;  // the gathered sender rows
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_fwd;
    acc[C_FWD_DELIV] = c_fwd_deliv;
    acc[C_DROPPED] = c_dropped;
    acc[C_HASH] = c_hash;
    acc[C_NEXT_ACKS] = c_fwd_deliv;
    acc[C_NEXT_ACKDROP] = c_next_ackdrop;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers;
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_STREAM_WAVES_PER_EU)))
void expand_stream(RoundArgs a) {
    stream_body<G, WPL, false>(a);
}

// Partition-window rounds: the mask bookkeeping needs more registers (4 waves/SIMD).
#ifndef GG_MASKED_WAVES_PER_EU
#define GG_MASKED_WAVES_PER_EU 4
#endif
template <int G, int WPL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_MASKED_WAVES_PER_EU)))
void expand_stream_masked(RoundArgs a) {
    stream_body<G, WPL, true>(a);
}

// Double-buffered lean rounds (RoundArgs::db): sets of r-1 in, sets of r out.
// D = 3 sender rows per batch on graphs with a mean in-degree below 4 (the host
// picks: C2 1.60 -> 1.56 ms/step), 4 above (C3 at 2M nodes: 6.58 vs 6.80 ms).
template <int G, int WPL, int D = kStreamRows>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_STREAM_WAVES_PER_EU)))
void expand_stream_db(RoundArgs a) {
    stream_body<G, WPL, false, true, false, D>(a);
}

// ... of marking rounds (RoundArgs::mark_cand) that are not busy: the same, and
// each node whose set changes marks itself and its receivers as candidates of
// round r+1 (the marking needs four more registers: a kernel of its own, so the
// busy rounds keep 5 waves/SIMD; with kMarkRows = 3 sender rows per batch it
// fits 5 waves too).
template <int G, int WPL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void expand_stream_db_mark(RoundArgs a) {
    stream_body<G, WPL, false, true, true, kMarkRows>(a);
}

// Which of a lane's D senders (columns c, the first n valid) were ACT last round
// (flags-first rounds of expand_stream1: one lane per node, so no ballot).
template <int D>
__device__ __forceinline__ uint32_t active_mask1(const uint64_t* abits, const uint32_t (&c)[D], uint32_t n) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(abits);
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < D; ++b) {
        const uint32_t col = c[b] & kColMask;
        if ((uint32_t)b < n && ((w[col >> 5] >> (col & 31)) & 1u)) m |= 1u << b;
    }
    return m;
}

// ---------------------------------------------------------------------------
// expand_stream1: expand_stream for W = 64 (one u64 per node). One lane per
// node, plain 8-byte loads (LDS-DMA has no 8-byte width) into registers; the
// same three-stage pipeline (list entry k+3, row pointers k+2, columns k+1)
// keeps each node to about one memory round trip. Same semantics and counters
// as expand_stream.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GG_STREAM1_WAVES_PER_EU)))
void expand_stream1(RoundArgs a) {
    constexpr int D = GG_STREAM1_ROWS;  // sender rows in flight per lane
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    if (!a.stream_ok) {
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    const bool dense = dense_round(a);
    const uint32_t n_items = dense ? (uint32_t)a.n_own : a.n_work[1];
    if ((uint64_t)blockIdx.x * kBlock >= n_items) {  // sparse round: no item reaches this block
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    uint32_t c_new = 0, c_active = 0, c_gathers = 0, c_nact = 0;
    unsigned long long c_fwd = 0, c_hash = 0, c_bytes = 0, c_nactdeg = 0;
    const uint32_t stride = gridDim.x * kBlock;
    const bool full = all_full(a);  // nothing can arrive: no gathers, no own rows
    const bool ff = ff_round(a);     // flags-first gathers (grid-uniform)
    constexpr uint32_t kAllD = (1u << D) - 1u;

    // the own row rides with the row pointers, two items ahead: a saturated node
    // (its set holds every lane injected through r-1) gathers nothing and reads no
    // columns. C5's last dense rounds deliver a few bits to few nodes while most
    // sets are already full (2^26 nodes: 19·10^6 and 44 new bits in rounds 14 and
    // 15, each a full 3.2 ms pass before)
    struct Meta {
        int64_t p0;
        uint64_t own;
        uint32_t deg, node;
        uint8_t ca, fl;
    };
    constexpr uint32_t kNone = ~0u;
    constexpr uint32_t kHubBit = 0x80000000u;
    auto node_of = [&](uint32_t k) -> uint32_t {
        return k < n_items ? (dense ? (uint32_t)k : a.nodes[k]) : kNone;
    };
    auto fetch_meta = [&](uint32_t n, Meta& m) {
        m.node = n;
        if (n < a.n_own) {
            m.p0 = a.in_ptr[n];
            m.deg = (uint32_t)(a.in_ptr[n + 1] - m.p0);
            m.ca = a.cand[a.own0 + n];
            m.fl = a.flg_cur[a.own0 + n];
            m.own = full ? 0ull : a.base[a.own0 + n];
            if (full) m.deg = 0;
            if (a.hub_deg && m.deg > a.hub_deg) {  // hub_chunks / hub_finish take it
                m.node |= kHubBit;
                m.deg = 0;
            }
            if (a.lanes_prev && (uint32_t)__popcll(m.own) == a.lanes_prev) m.deg = 0;  // saturated
        } else {
            m.p0 = 0;
            m.own = 0;
            m.deg = 0;
            m.ca = m.fl = 0;
        }
    };
    auto fetch_cols = [&](const Meta& m, uint32_t (&c)[D]) {
#pragma unroll
        for (int b = 0; b < D; ++b) c[b] = ((uint32_t)b < m.deg) ? a.in_col[m.p0 + b] : 0u;
    };

    uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    Meta m0, m1;
    uint32_t c0[D], c1[D];
    const uint32_t n0 = node_of(k), n1 = node_of(k + stride);
    uint32_t n2 = node_of(k + 2 * stride);
    fetch_meta(n0, m0);
    fetch_meta(n1, m1);
    fetch_cols(m0, c0);
    for (; k < n_items; k += stride) {
        const bool hub = (m0.node & kHubBit) != 0;
        const uint64_t i = m0.node & ~kHubBit;
        const uint64_t rep = a.own0 + i;
        // (a) own row and the first D sender rows
        const uint64_t sp = m0.own;
        uint64_t src[D];
        // flags-first round: look each sender up in the ACT bitmap (cache-resident:
        // V/8 bytes) and gather only the F words of senders active in r-1
        const uint32_t am0 = ff ? active_mask1<D>(a.abits, c0, m0.deg) : kAllD;
#pragma unroll
        for (int b = 0; b < D; ++b)
            src[b] = ((uint32_t)b < m0.deg && ((am0 >> b) & 1u)) ? a.F_prev[c0[b] & kColMask] : 0ull;
        // (b) prefetch the next items' columns, row pointers and list entry
        Meta m2;
        fetch_cols(m1, c1);
        fetch_meta(n2, m2);
        const uint32_t n3 = node_of(k + 3 * stride);
        if (!hub) {
            uint64_t S = sp;
            if (m0.ca & CA_INJ) {  // (1) client broadcasts of this round
                uint32_t lo = 0, hi = inj_n(a);
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (inj_p(a)[2 * mid] < (uint32_t)i) lo = mid + 1;
                    else hi = mid;
                }
                for (uint32_t q = lo; q < inj_n(a) && inj_p(a)[2 * q] == (uint32_t)i; ++q)
                    S |= 1ull << (inj_p(a)[2 * q + 1] & 63);
            }
            // (2) node broadcasts, ascending sender: first deliverer claims
            unsigned long long cl_recip = 0;
#pragma unroll
            for (int b = 0; b < D; ++b) {
                const uint64_t cw = src[b] & ~S;
                S |= cw;
                if (c0[b] & kRecipBit) cl_recip += __popcll(cw);
            }
            const int64_t p1 = m0.p0 + m0.deg;
            uint32_t ng = __popc(am0 & (m0.deg >= (uint32_t)D ? kAllD : ((1u << m0.deg) - 1u)));  // rows gathered
            for (int64_t e = m0.p0 + D; e < p1; e += D) {  // more than D senders
                uint32_t cb[D];
                uint64_t xb[D];
#pragma unroll
                for (int b = 0; b < D; ++b) cb[b] = e + b < p1 ? a.in_col[e + b] : 0u;
                const uint32_t am = ff ? active_mask1<D>(a.abits, cb, (uint32_t)(p1 - e)) : kAllD;
#pragma unroll
                for (int b = 0; b < D; ++b) xb[b] = (e + b < p1 && ((am >> b) & 1u)) ? a.F_prev[cb[b] & kColMask] : 0ull;
                ng += __popc(am & ((p1 - e >= D) ? kAllD : ((1u << (uint32_t)(p1 - e)) - 1u)));
#pragma unroll
                for (int b = 0; b < D; ++b) {
                    const uint64_t cw = xb[b] & ~S;
                    S |= cw;
                    if (cb[b] & kRecipBit) cl_recip += __popcll(cw);
                }
            }
            const uint32_t nin = m0.deg;
            c_gathers += ng;
            const uint64_t F = S & ~sp;
            const uint32_t T = (uint32_t)__popcll(F);
            if (F) {
                const uint64_t idx = gid_of(a, i) * a.nw + a.word0;
                c_hash += gg_word_hash(idx, F);
            }
            const bool any = F != 0;
            const bool zm = (m0.fl & FL_ACT) != 0;
            if (any || zm) a.F_cur[rep] = F;
            if (any) a.base[rep] = S;
            if (any || m0.fl) a.flg_cur[rep] = any ? FL_ACT : 0;
            if (m0.ca) a.cand[rep] = 0;
            // forward recipients: nin is 0 for a saturated node (no gathers), which can
            // still learn a client broadcast of this round: then the out-list length
            const unsigned long long deg =
                T == 0 ? 0ull : ((a.symmetric && nin) ? nin : (unsigned long long)(a.out_ptr[i + 1] - a.out_ptr[i]));
            c_new += T;
            c_fwd += deg * (unsigned long long)T - cl_recip;
            c_active += 1;
            c_nact += any ? 1 : 0;
            c_nactdeg += any ? deg : 0;
            c_bytes += (dense ? 0 : 4) + 8 + 2 + 4ull * nin + (ff ? (nin + 7) / 8 : 0) + 8ull * ((full ? 0 : 1) + ng) +
                       ((any || zm) ? 8 : 0) +
                       (any ? 9 : 0);
        }
        m0 = m1;
        m1 = m2;
        n2 = n3;
#pragma unroll
        for (int b = 0; b < D; ++b) c0[b] = c1[b];
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int q = 0; q < C_NUM; ++q) acc[q] = 0;
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_fwd;
    acc[C_FWD_DELIV] = c_fwd;
    acc[C_HASH] = c_hash;
    acc[C_NEXT_ACKS] = c_fwd;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers;
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

// ---------------------------------------------------------------------------
// Sync rounds, streamed (no partition masks, no in-hubs, nwp >= 2). After the
// timers start most senders are idle and a few push their whole set
// (SyncBroadcast callback, `broadcast.go:98-110`), so gathering every sender's
// F row the way expand_stream does would move mostly zero rows. Instead:
//   round_prep         writes each node's sender-state byte sstate (FL_ACT,
//                      FL_LAG of r-1, SE_FM2, SE_FM3): one lookup per edge below
//                      instead of a flag byte and two bitmap words.
//   sync_records       one thread per item (dense: every node; sparse: the node
//                      list): walks the in-list once (sender states), and for a
//                      callback node its out-list, and writes a 32-byte record:
//                      the node's own bits, up to three contributing senders
//                      (active last round, or pushing) with push/LAG bits, the
//                      out-list offset and its peers' LAG mask. Clears the
//                      candidate byte.
//   expand_stream_sync G lanes per node, records one item ahead: the own row,
//                      the recorded senders' rows and the first callback peers'
//                      columns are in flight together; nodes with more
//                      contributing senders walk their in-list, callback nodes
//                      their out-list, in batches.
// A node's whole set is base | F_prev, and base alone unless it is LAG (F rows
// are zero for idle nodes, and folded into base unless LAG); nodes whose sets
// are pushed or read keep base this round.
constexpr uint32_t SR_DEG = 0x000fffffu;       // forward recipients (out-degree)
constexpr int SR_NC = 20;                      // bits 20-21: recorded contributing senders
constexpr uint32_t SR_SLOW = 1u << 22;         // more than 3 of them (or a huge degree): walk the in-list
constexpr uint32_t SR_QUIET = 1u << 23;        // saturated, nothing arrives, every callback peer saturated:
                                               // the set cannot change and no push has content
constexpr uint32_t SR_SATV = 1u << 24;         // the node's set is saturated (sat digest)
constexpr uint32_t SR_KEEP = 1u << 26;         // the node's set is read this round: base stays
constexpr uint32_t SR_CB = 1u << 27;           // sync callback (fired in r-2)
constexpr uint32_t SR_LAG = 1u << 28;          // base lacks F_prev
constexpr uint32_t SR_STALE = 1u << 29;        // F row of round r-2 in this round's F buffer
constexpr uint32_t SR_INJ = 1u << 30;          // client broadcasts this round
constexpr uint32_t SR_HUB = 1u << 31;          // in-degree above hub_deg: hub_sync_chunks / hub_sync_finish /
                                               // hub_sync_push take the node (its cand byte is left set)
// second word: .x/.y out_ptr[i] (callback), .z peers' LAG mask (first 32 peers),
// .w bits 0-2: recorded sender j pushes, bits 3-5: recorded sender j is LAG

// Index of hub node i in the ascending hub list.
__device__ __forceinline__ uint32_t hub_index(const RoundArgs& a, uint32_t i) {
    uint32_t lo = 0, hi = (uint32_t)a.n_hubs;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.hubs[mid] < i) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void sync_records(RoundArgs a) {
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    const bool dense = dense_round(a);
    const uint32_t n_items = dense ? (uint32_t)a.n_own : a.n_work[1];
    // symmetric topology: the out-list is the in-list (same array), so a
    // callback's peer checks ride on the in-list walk
    const bool sym = a.out_col == a.in_col && a.out_ptr == a.in_ptr;
    unsigned long long c_bytes = 0;
    constexpr int B = 8;
    for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < n_items; k += gridDim.x * kBlock) {
        uint32_t i;
        uint8_t ca, fo, st;
        if (dense) {
            i = k;
            ca = a.cand[a.own0 + i];
            fo = a.flg_cur[a.own0 + i];
            st = a.sstate[a.own0 + i];
            if (ca) a.cand[a.own0 + i] = 0;
        } else {  // compact_round packed the node's bytes and cleared its candidate byte
            const uint2 m = a.nmeta[k];
            i = m.x;
            ca = (uint8_t)m.y;
            fo = (uint8_t)(m.y >> 8);
            st = (uint8_t)(m.y >> 16);
        }
        const uint64_t rep = a.own0 + i;
        const int64_t p0 = a.in_ptr[i], p1 = a.in_ptr[i + 1];
        if (a.hub_deg && p1 - p0 > (int64_t)a.hub_deg) {
            // a hub: the hub_sync kernels take it (its candidate byte moves to hlive;
            // the byte itself may be marked for the next round meanwhile)
            a.hlive[hub_index(a, i)] = (uint8_t)(ca | CA_NODE);
            a.srec[2 * (uint64_t)i] = make_uint4(SR_HUB, 0, 0, 0);
            c_bytes += 16 + 16 + 1;
            continue;
        }
        const int64_t o0 = sym ? p0 : a.out_ptr[i], o1 = sym ? p1 : a.out_ptr[i + 1];
        const uint64_t dout = (uint64_t)(o1 - o0);
        const bool cbk = (st & SE_FM2) != 0;
        const bool satv = a.sat && bit_at(a.sat, rep);
        bool keep = (st & SE_FM3) != 0;
        uint32_t nc = 0, sbits = 0, col0 = 0, col1 = 0, col2 = 0, lagm = 0;
        bool quiet = false;
        if (satv) {
            // saturated: S is every lane injected so far and nothing that arrives
            // (senders' sets are subsets of it) can change it, so senders are not
            // looked up and keep does not matter (the base write is S either way).
            // A callback still answers each peer: peers saturated too need nothing,
            // the others are gathered for the push difference (and their LAG bit).
            keep = false;
            quiet = !(st & FL_LAG) && !(fo & FL_ACT) && !(ca & CA_INJ);
            if (cbk) {
                bool allsat = true;
                for (int64_t e0 = o0; e0 < o1; e0 += B) {
                    uint32_t w[B];
                    bool sb[B];
#pragma unroll
                    for (int b = 0; b < B; ++b) w[b] = e0 + b < o1 ? (a.out_col[e0 + b] & kColMask) : 0u;
#pragma unroll
                    for (int b = 0; b < B; ++b) sb[b] = e0 + b >= o1 || bit_at(a.sat, w[b]);
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        allsat &= sb[b];
                        const int64_t pos = e0 - o0 + b;
                        if (!sb[b] && pos < 32 && bit_at(a.ibits, w[b]) && (a.sstate[w[b]] & FL_LAG)) lagm |= 1u << pos;
                    }
                }
                quiet = quiet && allsat;
                c_bytes += 4ull * dout;
            }
        } else {
            for (int64_t e0 = p0; e0 < p1; e0 += B) {
                uint32_t cb[B];
                uint8_t f[B];
#pragma unroll
                for (int b = 0; b < B; ++b) cb[b] = e0 + b < p1 ? a.in_col[e0 + b] : 0u;
                // in-neighbour u is a callback of this round (fired in r-2): it reads this set
#pragma unroll
                for (int b = 0; b < B; ++b) keep |= e0 + b < p1 && bit_at(a.fired_m2, cb[b] & kColMask);
                // ibits: ACT, LAG or pushing senders only (sparse once sync rounds settle)
#pragma unroll
                for (int b = 0; b < B; ++b) f[b] = e0 + b < p1 ? (uint8_t)bit_at(a.ibits, cb[b] & kColMask) : (uint8_t)0;
#pragma unroll
                for (int b = 0; b < B; ++b) f[b] = f[b] ? a.sstate[cb[b] & kColMask] : (uint8_t)0;
#pragma unroll
                for (int b = 0; b < B; ++b) {  // a push from an owned sender that sent nothing is no push
                    if ((f[b] & SE_FM3) && a.rev && (cb[b] & kColMask) < a.n_own && !a.pushb[a.rev[e0 + b]])
                        f[b] &= (uint8_t)~SE_FM3;
                }
                if (sym && cbk) {  // the out-list is this list: the peers' LAG bits
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        const int64_t pos = e0 - p0 + b;
                        if (e0 + b < p1 && pos < 32 && (f[b] & FL_LAG)) lagm |= 1u << pos;
                    }
                }
#pragma unroll
                for (int b = 0; b < B; ++b) {
                    if (f[b] & (FL_ACT | SE_FM3)) {
                        if (nc == 0) col0 = cb[b];
                        else if (nc == 1) col1 = cb[b];
                        else if (nc == 2) col2 = cb[b];
                        if (nc < 3)
                            sbits |= ((f[b] & SE_FM3) ? 1u << nc : 0u) | ((f[b] & FL_LAG) ? 8u << nc : 0u);
                        ++nc;
                    }
                }
            }
            c_bytes += 5ull * (uint64_t)(p1 - p0);
            if (cbk && !sym) {  // which peers' base rows lag their F rows
                const int64_t oe = o1 < o0 + 32 ? o1 : o0 + 32;
                for (int64_t e0 = o0; e0 < oe; e0 += B) {
                    uint8_t f[B];
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        const uint64_t w = e0 + b < oe ? (uint64_t)(a.out_col[e0 + b] & kColMask) : 0ull;
                        f[b] = (e0 + b < oe && bit_at(a.ibits, w)) ? a.sstate[w] : (uint8_t)0;
                    }
#pragma unroll
                    for (int b = 0; b < B; ++b) lagm |= (f[b] & FL_LAG) ? 1u << (e0 - o0 + b) : 0u;
                }
                c_bytes += 5ull * (uint64_t)(oe - o0);
            }
        }
        uint32_t x = (uint32_t)(dout < SR_DEG ? dout : SR_DEG);
        if (nc > 3 || dout >= SR_DEG) x |= SR_SLOW;
        else x |= nc << SR_NC;
        if (keep) x |= SR_KEEP;
        if (quiet) x |= SR_QUIET;
        if (satv) x |= SR_SATV;
        if (cbk) x |= SR_CB;
        if (st & FL_LAG) x |= SR_LAG;
        if (fo & FL_ACT) x |= SR_STALE;
        if (ca & CA_INJ) x |= SR_INJ;
        a.srec[2 * (uint64_t)i] = make_uint4(x, col0, col1, col2);
        a.srec[2 * (uint64_t)i + 1] = make_uint4((uint32_t)o0, (uint32_t)((uint64_t)o0 >> 32), lagm, sbits);
        // row_ptr (+ out_ptr), the node's bytes, the record
        c_bytes += (sym ? 16 : 32) + (dense ? 3 + (ca ? 1 : 0) : 8) + 32;
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int q = 0; q < C_NUM; ++q) acc[q] = 0;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_PREP);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void expand_stream_sync(RoundArgs a) {
    constexpr int kCb = 4;  // callback peers / in-list senders per batch
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    const bool dense = dense_round(a);
    const uint32_t n_items = dense ? (uint32_t)a.n_own : a.n_work[1];
    uint32_t c_new = 0, c_active = 0, c_gathers = 0, c_nact = 0;
    unsigned long long c_fwd = 0, c_push = 0, c_hash = 0, c_bytes = 0, c_nactdeg = 0;
    const int lg = threadIdx.x % G;
    const uint32_t off = (uint32_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    const uint32_t stride = gridDim.x * (kBlock / G);
    const unsigned long long rowb = 8ull * a.nwp;
    constexpr uint32_t kNone = ~0u;
    auto node_of = [&](uint32_t k) -> uint32_t {
        return k < n_items ? (dense ? k : a.nodes[k]) : kNone;
    };
    auto zero = []() {
        Row<WPL> z;
#pragma unroll
        for (int w = 0; w < WPL; ++w) z.w[w] = 0;
        return z;
    };
    auto or_in = [](Row<WPL>& d, const Row<WPL>& x) {
#pragma unroll
        for (int w = 0; w < WPL; ++w) d.w[w] |= x.w[w];
    };
    auto row_at = [&](const uint64_t* arr, uint64_t u) { return load_row<WPL>(arr + u * a.nwp + off); };

    uint32_t k = blockIdx.x * (kBlock / G) + threadIdx.x / G;
    uint32_t n0 = node_of(k), n1 = node_of(k + stride);
    uint4 r0 = make_uint4(0, 0, 0, 0), q0 = r0;
    if (n0 < a.n_own) {
        r0 = a.srec[2 * (uint64_t)n0];
        q0 = a.srec[2 * (uint64_t)n0 + 1];
    }
    for (; k < n_items; k += stride) {
        const uint64_t i = n0;
        const uint64_t rep = a.own0 + i;
        const uint32_t x = r0.x;
        if (x & SR_HUB) {  // the hub_sync kernels take it
            const uint32_t n2 = node_of(k + 2 * stride);
            r0 = make_uint4(0, 0, 0, 0);
            q0 = r0;
            if (n1 < a.n_own) {
                r0 = a.srec[2 * (uint64_t)n1];
                q0 = a.srec[2 * (uint64_t)n1 + 1];
            }
            n0 = n1;
            n1 = n2;
            continue;
        }
        const bool lag = (x & SR_LAG) != 0, slow = (x & SR_SLOW) != 0, cbk = (x & SR_CB) != 0;
        const bool quiet = (x & SR_QUIET) != 0, satv = (x & SR_SATV) != 0;
        const uint32_t nc = slow ? 0u : (x >> SR_NC) & 3u;
        const uint32_t sb = q0.w;
        const int64_t o0 = (int64_t)(((uint64_t)q0.y << 32) | q0.x);
        uint64_t dout = x & SR_DEG;
        if (dout == SR_DEG) dout = (uint64_t)(a.out_ptr[i + 1] - a.out_ptr[i]);
        // own row (+ its F row when base lags), the recorded senders' rows (F,
        // or base for pushes, + F when that base lags), the first callback
        // peers' columns: one round trip
        Row<WPL> sp = quiet ? zero() : row_at(a.base, rep);
        const Row<WPL> of = lag ? row_at(a.F_prev, rep) : zero();
        const uint32_t cs[3] = {r0.y, r0.z, r0.w};
        Row<WPL> fr[3], br[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t u = cs[j] & kColMask;
            const bool v = (uint32_t)j < nc, push = (sb >> j) & 1u, slag = (sb >> (3 + j)) & 1u;
            fr[j] = (v && (!push || slag)) ? row_at(a.F_prev, u) : zero();
            br[j] = (v && push) ? row_at(a.base, u) : zero();
        }
        uint64_t pw[kCb];
#pragma unroll
        for (int b = 0; b < kCb; ++b)
            pw[b] = (cbk && !quiet && (uint64_t)b < dout) ? (uint64_t)(a.out_col[o0 + b] & kColMask) : 0ull;
        // next item's record, the item after's list entry
        const uint32_t n2 = node_of(k + 2 * stride);
        uint4 r1 = make_uint4(0, 0, 0, 0), q1 = r1;
        if (n1 < a.n_own) {
            r1 = a.srec[2 * (uint64_t)n1];
            q1 = a.srec[2 * (uint64_t)n1 + 1];
        }
        if (quiet) {  // nothing arrives, every read_ok equals the node's set: no change, no push
            if (cbk && a.pushb && lg == 0) {
                for (uint64_t e = 0; e < dout; ++e) a.pushb[o0 + e] = 0;
                if (a.pushany) a.pushany[rep] = 0;
            }
            if (lg == 0) {
                c_active += 1;
                c_bytes += 32 + (cbk ? dout : 0);
            }
            n0 = n1;
            n1 = n2;
            r0 = r1;
            q0 = q1;
            continue;
        }

        or_in(sp, of);
        Row<WPL> S = sp;
        if (x & SR_INJ) {  // (1) client broadcasts of this round
            uint32_t lo = 0, hi = inj_n(a);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (inj_p(a)[2 * mid] < (uint32_t)i) lo = mid + 1;
                else hi = mid;
            }
            for (uint32_t q = lo; q < inj_n(a) && inj_p(a)[2 * q] == (uint32_t)i; ++q) {
                const uint32_t lane = inj_p(a)[2 * q + 1];
                const uint32_t word = lane >> 6;
                if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
            }
        }
        // (2) node broadcasts and pushes, ascending sender: first deliverer claims
        unsigned long long cl_recip = 0;
        auto claim = [&](const Row<WPL>& src, uint32_t c) {
            unsigned long long n = 0;
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                const uint64_t cw = src.w[w] & ~S.w[w];
                S.w[w] |= cw;
                n += __popcll(cw);
            }
            if (c & kRecipBit) cl_recip += n;
        };
        unsigned long long nrows = 1 + (lag ? 1 : 0), nextra = 32;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if ((uint32_t)j < nc) {
                Row<WPL> r = fr[j];
                or_in(r, br[j]);
                claim(r, cs[j]);
                const bool push = (sb >> j) & 1u, slag = (sb >> (3 + j)) & 1u;
                nrows += (push ? 1 : 0) + ((!push || slag) ? 1 : 0);
            }
        }
        if (slow) {  // walk the in-list: sender states, then the contributing rows
            const int64_t p0 = a.in_ptr[i], p1 = a.in_ptr[i + 1];
            nextra += 16 + 5ull * (uint64_t)(p1 - p0);
            for (int64_t e0 = p0; e0 < p1; e0 += kCb) {
                uint32_t cb[kCb];
                uint8_t f[kCb];
                Row<WPL> r[kCb];
#pragma unroll
                for (int b = 0; b < kCb; ++b) cb[b] = e0 + b < p1 ? a.in_col[e0 + b] : 0u;
#pragma unroll
                for (int b = 0; b < kCb; ++b) f[b] = e0 + b < p1 ? a.sstate[cb[b] & kColMask] : (uint8_t)0;
#pragma unroll
                for (int b = 0; b < kCb; ++b) {  // as sync_records: empty pushes are no pushes
                    if ((f[b] & SE_FM3) && a.rev && (cb[b] & kColMask) < a.n_own && !a.pushb[a.rev[e0 + b]])
                        f[b] &= (uint8_t)~SE_FM3;
                }
#pragma unroll
                for (int b = 0; b < kCb; ++b) {
                    const uint64_t u = cb[b] & kColMask;
                    const bool push = f[b] & SE_FM3, con = f[b] & (FL_ACT | SE_FM3), slag = f[b] & FL_LAG;
                    const Row<WPL> fb = (con && (!push || slag)) ? row_at(a.F_prev, u) : zero();
                    r[b] = push ? row_at(a.base, u) : zero();
                    or_in(r[b], fb);
                    nrows += (push ? 1 : 0) + ((con && (!push || slag)) ? 1 : 0);
                    c_gathers += (lg == 0 && con) ? 1u : 0u;
                }
#pragma unroll
                for (int b = 0; b < kCb; ++b)
                    if (f[b] & (FL_ACT | SE_FM3)) claim(r[b], cb[b]);
            }
        }
        // (3) sync callback: v fired in r-2; read_oks of its peers, ascending peer
        unsigned long long cb_new = 0, push_sent = 0;
        bool pushed = false;
        if (cbk) {
            const uint32_t lagm = q0.z;
            nextra += 16 + 4 * dout;
            for (uint64_t e0 = 0; e0 < dout; e0 += kCb) {
                Row<WPL> R[kCb];
                bool same[kCb];  // both sets saturated: the read_ok equals S, no row needed
#pragma unroll
                for (int b = 0; b < kCb; ++b) {
                    const uint64_t e = e0 + b;
                    same[b] = satv && e < dout && bit_at(a.sat, pw[b]);
                    const bool slag = e >= 32 || ((lagm >> e) & 1u);
                    R[b] = (e < dout && !same[b]) ? row_at(a.base, pw[b]) : zero();
                    const Row<WPL> f = (e < dout && !same[b] && slag) ? row_at(a.F_prev, pw[b]) : zero();
                    or_in(R[b], f);
                    nrows += (e < dout && !same[b]) ? (slag ? 2 : 1) : 0;
                }
                // columns of the next batch, in flight with these rows
                uint64_t pc[kCb];
#pragma unroll
                for (int b = 0; b < kCb; ++b) {
                    const uint64_t e = e0 + kCb + b;
                    pc[b] = pw[b];
                    pw[b] = e < dout ? (uint64_t)(a.out_col[o0 + e] & kColMask) : 0ull;
                }
#pragma unroll
                for (int b = 0; b < kCb; ++b) {
                    if (e0 + b >= dout) continue;
                    if (same[b]) R[b] = S;  // S is the saturated set throughout (only sets <= it arrive)
                    unsigned long long pn = 0, pp = 0;
#pragma unroll
                    for (int q = 0; q < WPL; ++q) {
                        pn += __popcll(R[b].w[q] & ~S.w[q]);
                        pp += __popcll(S.w[q] & ~R[b].w[q]);
                        S.w[q] |= R[b].w[q];
                    }
                    if (a.pushb) {  // did this peer get any push (next round's receivers)
                        const bool nz = ((__ballot(pp != 0) >> gshift) & gmask) != 0;
                        if (lg == 0) {
                            a.pushb[o0 + e0 + b] = nz ? 1 : 0;
                            pushed |= nz;
                            // the receiver's candidate byte for round r+1 (round_prep skips the walk)
                            if (nz && a.mark_next && pc[b] < a.n_own) a.cand_next[a.own0 + pc[b]] = CA_NODE;
                        }
                    }
                    cb_new += pn;
                    push_sent += pp;
                }
            }
        }
        if (cbk && lg == 0 && a.pushany) a.pushany[rep] = pushed ? 1 : 0;
        // new state (as expand_round)
        Row<WPL> F;
        uint32_t T = 0;
        const uint64_t g = gid_of(a, i);
#pragma unroll
        for (int w = 0; w < WPL; ++w) {
            F.w[w] = S.w[w] & ~sp.w[w];
            T += __popcll(F.w[w]);
            if (F.w[w]) {
                const uint64_t idx = g * a.nw + a.word0 + off + w;
                c_hash += gg_word_hash(idx, F.w[w]);
            }
        }
        const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
        const bool zm = (x & SR_STALE) != 0, keep = (x & SR_KEEP) != 0;
        if (any || zm) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
        nrows += (any || zm) ? 1 : 0;
        if (keep) {
            if (lag) store_row<WPL>(a.base + rep * a.nwp + off, sp);
            nrows += lag ? 1 : 0;
        } else if (any || lag) {
            store_row<WPL>(a.base + rep * a.nwp + off, S);
            nrows++;
        }
        if (lg == 0 && (any || zm)) a.flg_cur[rep] = any ? (uint8_t)(FL_ACT | (keep ? FL_LAG : 0)) : (uint8_t)0;
        if (any && a.sat_new) sat_mark<G, WPL>(a, S, rep, lg);
        c_new += T;
        c_fwd += dout * (unsigned long long)T - cl_recip - cb_new;
        c_push += push_sent;
        if (lg == 0) {
            c_active += 1;
            c_gathers += nc;
            c_nact += any ? 1u : 0u;
            c_nactdeg += any ? dout : 0ull;
            c_bytes += nrows * rowb + nextra + ((any || zm) ? 1 : 0);
        }
        n0 = n1;
        n1 = n2;
        r0 = r1;
        q0 = q1;
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int q = 0; q < C_NUM; ++q) acc[q] = 0;
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_fwd;
    acc[C_FWD_DELIV] = c_fwd;
    acc[C_PUSH] = c_push;
    acc[C_PUSH_DELIV] = c_push;
    acc[C_HASH] = c_hash;
    acc[C_NEXT_ACKS] = c_fwd + c_push;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers;
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

// ---------------------------------------------------------------------------
// Batched gossip (gg_config.batch_ticks; new semantics, DESIGN.md §2b — not the
// parity path; message-level restatement oracle/o1_batched.py, bitset one
// O2 compute_round_batched): every node, every round. G lanes per node: own set,
// client broadcasts, the messages its in-neighbours sent last round and no
// partition window dropped (their batch = F row, and on a push edge their whole
// set of r-1: the push carried every value the sender held that this node's
// read_ok lacked, ascending sender), the read_oks of a sync callback (peers'
// sets of r-1, ascending) followed by one push per such peer when S & ~R is not
// empty; new values into the pending row; the sync timer; at a send tick the
// pending row becomes the node's F row (its batch, read by its out-neighbours
// next round) and one message per out-neighbour is counted, except to the one
// neighbour that delivered every pending value (the message to it would be
// empty). F rows are rewritten only when they change (flags: a batch sent two
// rounds ago in this buffer). With sync, sets are also double-buffered
// (bset_prev / bset_cur): pushes and read_oks carry sets of r-1 while nodes
// update theirs in place.
constexpr uint32_t kPendNone = ~0u, kPendMixed = ~0u - 1;
template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void expand_batched(RoundArgs a) {
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    const int lg = threadIdx.x % G;
    const uint32_t off = (uint32_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    auto group_any = [&](bool x) { return ((__ballot(x) >> gshift) & gmask) != 0; };
    const bool sync = a.enable_sync && a.bset_prev != nullptr;
    bool win = false;  // some partition window covers r-3 .. r+1
#pragma unroll
    for (int k = 0; k < 5; ++k) win |= a.grp[k] != nullptr;
    uint32_t c_new = 0, c_active = 0, c_nact = 0;
    unsigned long long c_msgs = 0, c_deliv = 0, c_hash = 0, c_bytes = 0, c_gathers = 0;
    unsigned long long c_push = 0, c_push_deliv = 0, c_ackdrop = 0, c_dropped = 0;
    unsigned long long c_reads = 0, c_read_oks = 0, c_fired = 0;
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / G);
    const uint64_t first = (uint64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G;
    const unsigned long long rowb = 8ull * a.nwp;
    // whole groups run the loop together (the group's node, or past the end)
    const uint64_t bound = (a.n_own + ngroups - 1) / ngroups * ngroups;  // same trip count for every group
    for (uint64_t i = first; i < bound; i += ngroups) {
        const bool valid = i < a.n_own;
        const uint64_t rep = a.own0 + (valid ? i : 0);
        Row<WPL> S, sp, P;
        uint32_t src = kPendNone;
        if (valid) {
            S = load_row<WPL>(a.base + rep * a.nwp + off);
            P = load_row<WPL>(a.pend + rep * a.nwp + off);
            src = a.pend_src[rep];
        } else {
#pragma unroll
            for (int w = 0; w < WPL; ++w) S.w[w] = P.w[w] = 0;
        }
        sp = S;
        auto deliver = [&](uint32_t d) {  // d: local row | kRecipBit when d is an out-neighbour
            src = src == kPendNone ? d : ((src != kPendMixed && (src & kColMask) == (d & kColMask)) ? src : kPendMixed);
        };
        // (1) client broadcasts: a new client value goes to every neighbour
        bool inj_new = false;
        if (valid && (a.cand[rep] & CA_INJ)) {
            uint32_t lo = 0, hi = inj_n(a);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (inj_p(a)[2 * mid] < (uint32_t)i) lo = mid + 1;
                else hi = mid;
            }
            for (uint32_t q = lo; q < inj_n(a) && inj_p(a)[2 * q] == (uint32_t)i; ++q) {
                const uint32_t ln = inj_p(a)[2 * q + 1];
                const uint32_t word = ln >> 6;
                if (word / WPL == (uint32_t)lg) {
                    Row<WPL> b;
#pragma unroll
                    for (int w = 0; w < WPL; ++w) b.w[w] = 0;
                    set_lane_bit<WPL>(b, word % WPL, ln & 63);
#pragma unroll
                    for (int w = 0; w < WPL; ++w) {
                        inj_new |= (b.w[w] & ~S.w[w]) != 0;
                        S.w[w] |= b.w[w];
                    }
                }
            }
        }
        if (group_any(inj_new)) src = kPendMixed;
        // (2) last round's batches and pushes, ascending sender
        const int64_t p0 = valid ? a.in_ptr[i] : 0, p1 = valid ? a.in_ptr[i + 1] : 0;
        for (int64_t e = p0; e < p1; ++e) {
            const uint32_t c = a.in_col[e];
            const uint64_t u = c & kColMask;
            if (sync && bit_at(a.fired_m1, u) && !masked<true>(a, 2, u, rep, e)) {  // u's read, answered now
                c_read_oks++;
                if (masked<true>(a, 3, rep, u, e)) c_dropped++;
            }
            if (win && masked<true>(a, 2, u, rep, e)) continue;  // dropped in flight (r-1)
            const bool push = sync && bit_at(a.fired_m3, u) && !masked<true>(a, 0, u, rep, e) &&
                              !masked<true>(a, 1, rep, u, e);
            Row<WPL> x = load_row<WPL>(a.F_prev + u * a.nwp + off);
            if (push) {
                const Row<WPL> y = load_row<WPL>(a.bset_prev + u * a.nwp + off);
#pragma unroll
                for (int w = 0; w < WPL; ++w) x.w[w] |= y.w[w];
            }
            bool got = false;
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                const uint64_t cw = x.w[w] & ~S.w[w];
                S.w[w] |= cw;
                got |= cw != 0;
            }
            if (group_any(got)) deliver((uint32_t)u | (c & kRecipBit));
            c_gathers += push ? 2 : 1;
        }
        // (3) sync callback (fired in r-2): read_oks of the peers ascending, then one push each
        const int64_t o0 = valid ? a.out_ptr[i] : 0, o1 = valid ? a.out_ptr[i + 1] : 0;
        if (sync && valid && bit_at(a.fired_m2, rep)) {
            for (int pass = 0; pass < 2; ++pass) {
                for (int64_t e = o0; e < o1; ++e) {
                    const uint64_t w = a.out_col[e] & kColMask;
                    if (masked<true>(a, 1, rep, w, e) || masked<true>(a, 2, w, rep, e)) continue;
                    const Row<WPL> R = load_row<WPL>(a.bset_prev + w * a.nwp + off);
                    c_gathers++;
                    if (pass == 0) {
                        bool got = false;
#pragma unroll
                        for (int q = 0; q < WPL; ++q) {
                            got |= (R.w[q] & ~S.w[q]) != 0;
                            S.w[q] |= R.w[q];
                        }
                        if (group_any(got)) deliver((uint32_t)w | kRecipBit);
                    } else {
                        bool any = false;
#pragma unroll
                        for (int q = 0; q < WPL; ++q) any |= (S.w[q] & ~R.w[q]) != 0;
                        if (!group_any(any)) continue;
                        c_push++;
                        if (masked<true>(a, 3, rep, w, e)) {
                            c_dropped++;
                        } else {
                            c_push_deliv++;
                            if (masked<true>(a, 4, w, rep, e)) c_ackdrop++;
                        }
                    }
                }
            }
        }
        // new state
        Row<WPL> F;
        uint32_t T = 0;
        bool pend_any = false;
        const uint64_t g = gid_of(a, i);
#pragma unroll
        for (int w = 0; w < WPL; ++w) {
            F.w[w] = S.w[w] & ~sp.w[w];
            T += __popcll(F.w[w]);
            if (F.w[w]) c_hash += gg_word_hash(g * a.nw + a.word0 + off + w, F.w[w]);
            if (a.dr && valid && off + w < a.dr_w / 64) {
                uint64_t y = F.w[w];
                while (y) {
                    const int b = __builtin_ctzll(y);
                    y &= y - 1;
                    a.dr[i * a.dr_w + (off + w) * 64 + b] = (int32_t)a.round;
                }
            }
            P.w[w] |= F.w[w];
            pend_any |= P.w[w] != 0;
        }
        const bool any = group_any(T != 0);
        const bool send = a.batch_tick && group_any(pend_any);
        if (valid) {
            if (any) store_row<WPL>(a.base + rep * a.nwp + off, S);
            if (sync) store_row<WPL>(a.bset_cur + rep * a.nwp + off, S);
            const uint8_t fl = a.flg_cur[rep];  // a batch of round r-2 in this F buffer
            if (send || (fl & FL_ACT)) {
                Row<WPL> out;
#pragma unroll
                for (int w = 0; w < WPL; ++w) out.w[w] = send ? P.w[w] : 0ull;
                store_row<WPL>(a.F_cur + rep * a.nwp + off, out);
            }
            if (send) {
#pragma unroll
                for (int w = 0; w < WPL; ++w) P.w[w] = 0;
            }
            if (any || send) store_row<WPL>(a.pend + rep * a.nwp + off, P);
            if (lg == 0) {
                if (send || fl) a.flg_cur[rep] = send ? FL_ACT : 0;
                if (a.cand[rep]) a.cand[rep] = 0;
                const uint64_t deg = (uint64_t)(o1 - o0);
                // (5) the sync timer (main.go:42-51): a read to every neighbour
                if (sync && (int64_t)a.sync_next[i] == a.round) {
                    c_fired++;
                    c_reads += deg;
                    if (win)
                        for (int64_t e = o0; e < o1; ++e)
                            if (masked<true>(a, 3, rep, a.out_col[e] & kColMask, e)) c_dropped++;
                    atomicOr(a.fired_cur + (rep >> 6), 1ull << (rep & 63));
                    const uint32_t kk = a.sync_k[i] + 1;
                    a.sync_k[i] = kk;
                    a.sync_next[i] = (int32_t)(a.round + gg_sync_interval_rcp(a.sync_mix, a.sync_rcp, g, kk, a.sync_base, a.sync_jitter));
                }
                // (6) the batch: one message per out-neighbour but the single deliverer
                const bool single = src != kPendMixed && src != kPendNone;
                if (send && !win) {
                    const unsigned long long msgs = deg - ((single && (src & kRecipBit)) ? 1 : 0);
                    c_msgs += msgs;
                    c_deliv += msgs;
                } else if (send) {
                    for (int64_t e = o0; e < o1; ++e) {
                        const uint64_t w = a.out_col[e] & kColMask;
                        if (single && (src & kColMask) == (uint32_t)w) continue;
                        c_msgs++;
                        if (masked<true>(a, 3, rep, w, e)) {
                            c_dropped++;
                        } else {
                            c_deliv++;
                            if (masked<true>(a, 4, w, rep, e)) c_ackdrop++;
                        }
                    }
                }
                const uint32_t nsrc = a.batch_tick ? kPendNone : src;
                if (nsrc != a.pend_src[rep]) a.pend_src[rep] = nsrc;
                c_active += 1;
                c_nact += send ? 1u : 0u;
                c_bytes += 16 + 4ull * (p1 - p0) + rowb * 2 + (any ? rowb : 0) + (sync ? rowb : 0) +
                           ((send || (fl & FL_ACT)) ? rowb : 0) + ((any || send) ? rowb : 0);
            }
            c_new += T;
        }
    }
    // sharded: the ghosts' sync timers (the same pure function of seed, node id and
    // k their owner runs), so their fired bits (reads answered here, pushes, the
    // sets the exchange ships) are known without crossing the exchange
    if (sync && a.n_ghost) {
        for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < a.n_ghost; g += (uint64_t)gridDim.x * kBlock) {
            const uint64_t row = a.ghost0 + g;
            if ((int64_t)a.sync_next[row] != a.round) continue;
            atomicOr(a.fired_cur + (row >> 6), 1ull << (row & 63));
            const uint32_t kk = a.sync_k[row] + 1;
            a.sync_k[row] = kk;
            a.sync_next[row] =
                (int32_t)(a.round + gg_sync_interval_rcp(a.sync_mix, a.sync_rcp, gid_of(a, row), kk, a.sync_base, a.sync_jitter));
        }
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    if (lg != 0) {  // per-message counts were taken once per node group (lane 0) or by every lane
        c_push = c_push_deliv = c_ackdrop = c_dropped = c_read_oks = 0;
    }
    acc[C_NEW] = c_new;
    acc[C_FWD_SENT] = c_msgs;
    acc[C_FWD_DELIV] = c_deliv;
    acc[C_PUSH] = c_push;
    acc[C_PUSH_DELIV] = c_push_deliv;
    acc[C_NEXT_ACKS] = c_deliv + c_push_deliv;
    acc[C_NEXT_ACKDROP] = c_ackdrop;
    acc[C_DROPPED] = c_dropped;
    acc[C_READS] = c_reads;
    acc[C_READ_OKS] = c_read_oks;
    acc[C_FIRED] = c_fired;
    acc[C_HASH] = c_hash;
    acc[C_ACTIVE] = c_active;
    acc[C_GATHERS] = c_gathers * (lg == 0 ? 1 : 0);
    acc[C_NACT] = c_nact;
    acc[C_BYTES] = c_bytes + (lg == 0 ? c_gathers * rowb : 0);
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

// rev[k] for in-edge k (sender u -> v): the position of v in u's out-list, for
// owned senders (streamed sync rounds read pushb through it); ~0u for ghosts.
// Out-lists ascend by node id (gid), so a binary search by id.
__global__ void build_rev(const int64_t* in_ptr, const uint32_t* in_col, const int64_t* out_ptr,
                          const uint32_t* out_col, const uint32_t* gid, uint64_t n_own, uint64_t n_edges,
                          uint32_t* rev) {
    // edge-parallel (a hub's in-list is no single thread's serial walk): each
    // thread takes a slice of consecutive in-edges, finds the slice's first row
    // by binary search in in_ptr, and for each edge v <- u binary-searches v in
    // u's out-list (ascending by original id)
    constexpr uint64_t kSlice = 8;
    const uint64_t slices = (n_edges + kSlice - 1) / kSlice;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < slices; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k0 = s * kSlice, k1 = k0 + kSlice < n_edges ? k0 + kSlice : n_edges;
        uint64_t lo = 0, hi = n_own - 1;  // largest v with in_ptr[v] <= k0
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if ((uint64_t)in_ptr[mid] <= k0) lo = mid;
            else hi = mid - 1;
        }
        uint64_t v = lo;
        for (uint64_t k = k0; k < k1; ++k) {
            while ((uint64_t)in_ptr[v + 1] <= k) ++v;  // empty rows in between
            const uint64_t gv = gid ? gid[v] : v;
            const uint32_t u = in_col[k] & kColMask;
            uint32_t r = ~0u;
            if (u < n_own) {
                int64_t a = out_ptr[u], b = out_ptr[u + 1];
                while (a < b) {
                    const int64_t mid = (a + b) >> 1;
                    const uint32_t w = out_col[mid] & kColMask;
                    if ((gid ? (uint64_t)gid[w] : (uint64_t)w) < gv) a = mid + 1;
                    else b = mid;
                }
                r = (uint32_t)a;
            }
            rev[k] = r;
        }
    }
}

// Flags-first rounds: the ACT bits of round r-1 (every local row: owned nodes
// and ghosts) packed into abits (rows is a multiple of 64). A thread turns 16
// flag bytes into 16 bits (FL_ACT is bit 0: a multiply gathers the eight bit-0s
// of a word into its top byte); one 16-byte load and a 2-byte store per lane
// keep the pass at streaming rate (one byte per lane ran at ~1 TB/s).
__global__ __launch_bounds__(kBlock) void pack_act_bits(RoundArgs a) {
    static_assert(FL_ACT == 1, "the bit gather assumes FL_ACT is bit 0");
    const unsigned long long t_start = clock100();
    if (!ff_view(a, ring_view(a))) {
        noop_exit(a, K_PREP, t_start);
        return;
    }
    const ulonglong2* fl = reinterpret_cast<const ulonglong2*>(a.flg_prev);
    uint16_t* out = reinterpret_cast<uint16_t*>(a.abits);
    constexpr unsigned long long kB0 = 0x0101010101010101ull, kGather = 0x0102040810204080ull;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < a.rows / 16; t += (uint64_t)gridDim.x * kBlock) {
        const ulonglong2 v = fl[t];
        const uint32_t lo = (uint32_t)(((v.x & kB0) * kGather) >> 56), hi = (uint32_t)(((v.y & kB0) * kGather) >> 56);
        out[t] = (uint16_t)(lo | (hi << 8));
    }
    if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
}

// ---------------------------------------------------------------------------
// Hubs (power-law graphs, lean rounds). The claim chain of a node is an ordered
// scan, and its result is all the counters need: the union O of the sender rows
// and, per bit, whether the first sender holding it (ascending id) is
// reciprocal (mask R). Pieces combine associatively in sender order:
//     (O1, R1) . (O2, R2) = (O1 | O2, R1 | (R2 & ~O1))
// and with the node's own row (+ client broadcasts) S0: new bits = O & ~S0,
// reciprocal claims = popcount(O & ~S0 & R). hub_chunks reduces each in-edge
// chunk of a hub with one block (its node groups take consecutive slices and
// combine in order in LDS) into hscratch; hub_finish combines a hub's chunks
// the same way and writes the node like expand_stream does.
template <int WPL>
__device__ __forceinline__ void hub_combine(Row<WPL>& O, Row<WPL>& R, const Row<WPL>& O2, const Row<WPL>& R2) {
#pragma unroll
    for (int w = 0; w < WPL; ++w) {
        R.w[w] |= R2.w[w] & ~O.w[w];
        O.w[w] |= O2.w[w];
    }
}

// Ordered tree reduction of the NGB node-group partials of a block in LDS;
// node group 0 ends with the combined (O, R). s_or/s_rc: [NGB][G*WPL] words.
template <int G, int WPL>
__device__ __forceinline__ void hub_block_reduce(Row<WPL>& O, Row<WPL>& R, uint64_t* s_or, uint64_t* s_rc) {
    constexpr int NGB = kBlock / G;
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
#pragma unroll
    for (int w = 0; w < WPL; ++w) {
        s_or[j * G * WPL + lg * WPL + w] = O.w[w];
        s_rc[j * G * WPL + lg * WPL + w] = R.w[w];
    }
    __syncthreads();
    for (int st = 1; st < NGB; st <<= 1) {
        if (j % (2 * st) == 0 && j + st < NGB) {
            Row<WPL> O2, R2;
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                O2.w[w] = s_or[(j + st) * G * WPL + lg * WPL + w];
                R2.w[w] = s_rc[(j + st) * G * WPL + lg * WPL + w];
            }
            hub_combine<WPL>(O, R, O2, R2);
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                s_or[j * G * WPL + lg * WPL + w] = O.w[w];
                s_rc[j * G * WPL + lg * WPL + w] = R.w[w];
            }
        }
        __syncthreads();
    }
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void hub_chunks(RoundArgs a) {
    constexpr int NGB = kBlock / G;
    constexpr int D = 4;  // sender rows in flight per lane
    __shared__ uint64_t s_or[NGB * G * WPL], s_rc[NGB * G * WPL];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    if (!a.stream_ok || !a.n_hchunks) {
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    const bool dense = dense_round(a);
    const bool ff = ff_round(a);  // flags-first: only active senders' rows
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    unsigned long long c_bytes = 0;
    for (uint64_t c = blockIdx.x; c < a.n_hchunks; c += gridDim.x) {
        const HubChunk hc = a.hchunks[c];
        const uint8_t hca = a.cand[a.own0 + hc.node];
        if (!dense && !hca) continue;  // block-uniform
        if (lsat_skip(a, a.own0 + hc.node, hca)) continue;  // saturated hub (hub_finish skips its chunks)
        const uint32_t per = (hc.n + NGB - 1) / NGB;
        const int64_t e0 = hc.e0 + (int64_t)j * per;
        const int64_t e1 = min(hc.e0 + (int64_t)hc.n, e0 + (int64_t)per);
        Row<WPL> O, R;
#pragma unroll
        for (int w = 0; w < WPL; ++w) O.w[w] = R.w[w] = 0;
        for (int64_t e = e0; e < e1; e += D) {
            uint32_t cb[D];
            Row<WPL> src[D];
#pragma unroll
            for (int b = 0; b < D; ++b) cb[b] = e + b < e1 ? a.in_col[e + b] : 0u;
            bool act[D];
#pragma unroll
            for (int b = 0; b < D; ++b) act[b] = e + b < e1 && (!ff || bit_at(a.abits, cb[b] & kColMask));
#pragma unroll
            for (int b = 0; b < D; ++b) {
                if (act[b]) {
                    // double-buffered rounds: the sender's set of r-1 (same claims, §3)
                    const uint64_t u = cb[b] & kColMask;
                    const uint64_t* rows = (a.db && !(a.n_ghost && u >= a.ghost0)) ? a.base_prev : a.F_prev;
                    src[b] = load_row<WPL>(rows + u * a.nwp + off);
                    if (lg == 0) c_bytes += 8ull * a.nwp;
                } else {
#pragma unroll
                    for (int w = 0; w < WPL; ++w) src[b].w[w] = 0;
                }
            }
#pragma unroll
            for (int b = 0; b < D; ++b) {
#pragma unroll
                for (int w = 0; w < WPL; ++w) {
                    const uint64_t cw = src[b].w[w] & ~O.w[w];
                    O.w[w] |= cw;
                    if (cb[b] & kRecipBit) R.w[w] |= cw;
                }
            }
        }
        if (lg == 0 && e1 > e0) c_bytes += (unsigned long long)(e1 - e0) * 4 + (ff ? (e1 - e0 + 7) / 8 : 0);
        hub_block_reduce<G, WPL>(O, R, s_or, s_rc);
        if (j == 0) {
            uint64_t* dst = a.hscratch + c * 2 * a.nwp;
            store_row<WPL>(dst + off, O);
            store_row<WPL>(dst + a.nwp + off, R);
            if (lg == 0) c_bytes += 16ull * a.nwp;
        }
        __syncthreads();  // LDS reuse
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void hub_finish(RoundArgs a) {
    constexpr int NGB = kBlock / G;
    __shared__ uint64_t s_or[NGB * G * WPL], s_rc[NGB * G * WPL];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    const unsigned long long t_start = clock100();
    if (!a.stream_ok || !a.n_hubs) {
        noop_exit(a, K_STREAM, t_start);
        return;
    }
    const bool dense = dense_round(a);
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    unsigned long long c_new = 0, c_fwd = 0, c_hash = 0, c_active = 0, c_gathers = 0, c_nact = 0, c_bytes = 0;
    unsigned long long c_nactdeg = 0;
    for (uint64_t h = blockIdx.x; h < a.n_hubs; h += gridDim.x) {
        const uint32_t i = a.hubs[h];
        const uint8_t ca = a.cand[i];
        if (!dense && !ca) continue;  // block-uniform
        const bool hsat = lsat_skip(a, a.own0 + i, ca);  // hub_chunks skipped its chunks (stale hscratch)
        const uint32_t c0 = a.hub_c0[h], c1 = hsat ? c0 : a.hub_c0[h + 1];
        const uint32_t per = (c1 - c0 + NGB - 1) / NGB;
        const uint32_t q0 = c0 + j * per, q1 = min(c1, q0 + per);
        Row<WPL> O, R;
#pragma unroll
        for (int w = 0; w < WPL; ++w) O.w[w] = R.w[w] = 0;
        for (uint32_t q = q0; q < q1; ++q) {
            const uint64_t* src = a.hscratch + (uint64_t)q * 2 * a.nwp;
            hub_combine<WPL>(O, R, load_row<WPL>(src + off), load_row<WPL>(src + a.nwp + off));
        }
        hub_block_reduce<G, WPL>(O, R, s_or, s_rc);
        if (j == 0) {
            const uint64_t rep = a.own0 + i;
            Row<WPL> sp = load_row<WPL>((a.db ? a.base_prev : a.base) + rep * a.nwp + off), S = sp;  // lean: no LAG
            if (ca & CA_INJ) {  // (1) client broadcasts of this round
                uint32_t lo = 0, hi = inj_n(a);
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (inj_p(a)[2 * mid] < i) lo = mid + 1;
                    else hi = mid;
                }
                for (uint32_t k = lo; k < inj_n(a) && inj_p(a)[2 * k] == i; ++k) {
                    const uint32_t lane = inj_p(a)[2 * k + 1];
                    const uint32_t word = lane >> 6;
                    if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
                }
            }
            // (2) node broadcasts: every new bit's first deliverer claims it
            unsigned long long cl_recip = 0;
            Row<WPL> F;
            unsigned long long T = 0;
            const uint64_t g = gid_of(a, i);
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                const uint64_t claim = O.w[w] & ~S.w[w];
                cl_recip += __popcll(claim & R.w[w]);
                S.w[w] |= claim;
                F.w[w] = S.w[w] & ~sp.w[w];
                T += __popcll(F.w[w]);
                if (F.w[w]) {
                    const uint64_t idx = g * a.nw + a.word0 + off + w;
                    c_hash += gg_word_hash(idx, F.w[w]);
                }
            }
            const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
            if (any && a.lsat && a.lmark) lsat_mark<G, WPL>(a, S, rep, lg, a.lreach ? a.lreach[rep] : a.lusat);
            const uint8_t fl = a.db ? a.flg_prev[rep] : a.flg_cur[rep];  // (db: r-1, else r-2)
            const bool zm = !a.db && (fl & FL_ACT) != 0;
            const bool lane_new = [&] {
                bool x = false;
#pragma unroll
                for (int w = 0; w < WPL; ++w) x |= F.w[w] != 0;
                return x;
            }();
            if (a.db) {  // chunks that changed now, whole row if it changed in r-1 (§3)
                if (lane_new || (fl & FL_ACT)) store_row<WPL>(a.base + rep * a.nwp + off, S);
            } else {
                if (any || zm) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
                if (any) store_row<WPL>(a.base + rep * a.nwp + off, S);
            }
            const uint64_t nin = (uint64_t)(a.in_ptr[i + 1] - a.in_ptr[i]);
            const unsigned long long deg = a.symmetric ? nin : (unsigned long long)(a.out_ptr[i + 1] - a.out_ptr[i]);
            c_new += T;
            c_fwd += deg * T - cl_recip;
            if (lg == 0) {
                if (any || fl || a.db) a.flg_cur[rep] = any ? FL_ACT : 0;
                if (ca) a.cand[rep] = 0;
                c_active += 1;
                c_gathers += hsat ? 0 : nin;
                c_nact += any ? 1 : 0;
                c_nactdeg += any ? deg : 0;
                c_bytes += 16 + 2 + (hsat ? 1 : 0) + (uint64_t)(c1 - c0) * 16 * a.nwp + 8 * a.nwp +
                           ((any || zm) ? 8 * a.nwp : 0) + (any ? 8 * a.nwp + 1 : 0);
            }
        }
        __syncthreads();  // LDS reuse
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
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

// ---------------------------------------------------------------------------
// Streamed sync rounds on graphs with hubs (symmetric topologies: a hub's
// out-list is its in-list, so one chunk list serves both directions). A hub
// takes three launches instead of one node group walking its whole list:
//   hub_sync_chunks  one block per edge chunk of a live hub: the chunk's senders
//                    under expand_stream_sync's rules (an ACT sender contributes
//                    its F row; a pusher — fired in r-3, pushb says it sent this
//                    hub something — its set base | (LAG ? F)), reduced in sender
//                    order to (union, first-claimer-reciprocal); whether a sender
//                    is a callback of this round (it reads the hub's set: keep);
//                    and, when the hub is a callback itself (fired in r-2), the OR
//                    of the chunk's peers' sets (their read_ok payloads).
//   hub_sync_finish  one block per live hub: its chunks combined in order with
//                    its own set and client broadcasts (the claims); a callback
//                    hub turns the chunk ORs into each chunk's exclusive prefix
//                    (its running set before the chunk's first peer,
//                    broadcast.go:110-114) and takes every peer's set; the node is
//                    written as expand_stream_sync writes it.
//   hub_sync_push    one block per chunk of a live callback hub: an ordered
//                    prefix OR over the chunk's peers gives each peer's push
//                    S_{i-1} & ~R_i (broadcast.go:104-108): push counts, pushb,
//                    the receivers' candidate bytes for the next round.
// Liveness: hlive (sync_records' copy of the hub's candidate byte, cleared by
// hub_sync_finish); hflag carries it from the chunks to the push launch.
constexpr uint32_t HF_KEEP = 1, HF_LIVE = 2, HF_CB = 4;

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void hub_sync_chunks(RoundArgs a) {
    constexpr int NGB = kBlock / G;
    constexpr int D = 4;  // senders in flight per lane
    __shared__ uint64_t s_or[NGB * G * WPL], s_rc[NGB * G * WPL];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    __shared__ uint32_t s_keep;
    const unsigned long long t_start = clock100();
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    unsigned long long c_bytes = 0, c_gathers = 0;
    for (uint64_t c = blockIdx.x; c < a.n_hchunks; c += gridDim.x) {
        const HubChunk hc = a.hchunks[c];
        const uint64_t rep = a.own0 + hc.node;
        if (!a.hlive[hub_index(a, hc.node)]) {  // block-uniform
            if (threadIdx.x == 0) a.hflag[c] = 0;
            continue;
        }
        const bool cbk = bit_at(a.fired_m2, rep);
        if (threadIdx.x == 0) s_keep = 0;
        __syncthreads();
        const uint32_t per = (hc.n + NGB - 1) / NGB;
        const int64_t e0 = hc.e0 + (int64_t)j * per;
        const int64_t e1 = min(hc.e0 + (int64_t)hc.n, e0 + (int64_t)per);
        Row<WPL> O, R, Q, Z;
#pragma unroll
        for (int w = 0; w < WPL; ++w) O.w[w] = R.w[w] = Q.w[w] = Z.w[w] = 0;
        bool keep = false;
        for (int64_t e = e0; e < e1; e += D) {
            uint32_t cb[D];
            uint8_t f[D];
#pragma unroll
            for (int b = 0; b < D; ++b) cb[b] = e + b < e1 ? a.in_col[e + b] : 0u;
#pragma unroll
            for (int b = 0; b < D; ++b) keep |= e + b < e1 && bit_at(a.fired_m2, cb[b] & kColMask);
#pragma unroll
            for (int b = 0; b < D; ++b)
                f[b] = (e + b < e1 && bit_at(a.ibits, cb[b] & kColMask)) ? a.sstate[cb[b] & kColMask] : (uint8_t)0;
#pragma unroll
            for (int b = 0; b < D; ++b) {  // a push from an owned sender that sent nothing is no push
                if ((f[b] & SE_FM3) && a.rev && (cb[b] & kColMask) < a.n_own && !a.pushb[a.rev[e + b]])
                    f[b] &= (uint8_t)~SE_FM3;
            }
            Row<WPL> r[D], fb[D], sb[D];
#pragma unroll
            for (int b = 0; b < D; ++b) {
                const uint64_t u = cb[b] & kColMask;
                const bool push = f[b] & SE_FM3, con = f[b] & (FL_ACT | SE_FM3), slag = f[b] & FL_LAG;
                const bool needf = (con && (!push || slag)) || (cbk && slag && e + b < e1);
                const bool needb = push || (cbk && e + b < e1);
#pragma unroll
                for (int w = 0; w < WPL; ++w) fb[b].w[w] = sb[b].w[w] = 0;
                if (needf) fb[b] = load_row<WPL>(a.F_prev + u * a.nwp + off);
                if (needb) sb[b] = load_row<WPL>(a.base + u * a.nwp + off);
                if (lg == 0) c_bytes += 8ull * a.nwp * ((needf ? 1 : 0) + (needb ? 1 : 0));
#pragma unroll
                for (int w = 0; w < WPL; ++w) r[b].w[w] = (con && (!push || slag) ? fb[b].w[w] : 0) | (push ? sb[b].w[w] : 0);
                c_gathers += (lg == 0 && con) ? 1u : 0u;
            }
#pragma unroll
            for (int b = 0; b < D; ++b) {
                if (f[b] & (FL_ACT | SE_FM3)) {
#pragma unroll
                    for (int w = 0; w < WPL; ++w) {
                        const uint64_t cw = r[b].w[w] & ~O.w[w];
                        O.w[w] |= cw;
                        if (cb[b] & kRecipBit) R.w[w] |= cw;
                    }
                }
                if (cbk && e + b < e1) {  // the peer's read_ok payload: its whole set
#pragma unroll
                    for (int w = 0; w < WPL; ++w) Q.w[w] |= sb[b].w[w] | ((f[b] & FL_LAG) ? fb[b].w[w] : 0);
                }
            }
        }
        if (lg == 0 && e1 > e0) c_bytes += (unsigned long long)(e1 - e0) * 6;
        if (keep) atomicOr(&s_keep, 1u);
        hub_block_reduce<G, WPL>(O, R, s_or, s_rc);
        if (j == 0) {
            uint64_t* dst = a.hscratch + c * 3 * a.nwp;
            store_row<WPL>(dst + off, O);
            store_row<WPL>(dst + a.nwp + off, R);
        }
        __syncthreads();  // LDS reuse
        if (cbk) {
            hub_block_reduce<G, WPL>(Q, Z, s_or, s_rc);  // an OR: the order does not matter
            if (j == 0) store_row<WPL>(a.hscratch + c * 3 * a.nwp + 2 * a.nwp + off, Q);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            a.hflag[c] = (s_keep ? HF_KEEP : 0u) | HF_LIVE | (cbk ? HF_CB : 0u);
            c_bytes += 16 + 16ull * a.nwp + (cbk ? 8ull * a.nwp : 0);
        }
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_GATHERS] = c_gathers;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void hub_sync_finish(RoundArgs a) {
    constexpr int NGB = kBlock / G;
    __shared__ uint64_t s_or[NGB * G * WPL], s_rc[NGB * G * WPL];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    __shared__ uint32_t s_keep;
    const unsigned long long t_start = clock100();
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    unsigned long long c_new = 0, c_fwd = 0, c_hash = 0, c_active = 0, c_nact = 0, c_bytes = 0, c_nactdeg = 0;
    for (uint64_t h = blockIdx.x; h < a.n_hubs; h += gridDim.x) {
        const uint32_t i = a.hubs[h];
        const uint64_t rep = a.own0 + i;
        const uint8_t ca = a.hlive[h];
        if (!ca) continue;  // block-uniform
        if (threadIdx.x == 0) s_keep = 0;
        __syncthreads();
        const uint32_t c0 = a.hub_c0[h], c1 = a.hub_c0[h + 1];
        const uint32_t per = (c1 - c0 + NGB - 1) / NGB;
        const uint32_t q0 = c0 + j * per, q1 = min(c1, q0 + per);
        Row<WPL> O, R;
#pragma unroll
        for (int w = 0; w < WPL; ++w) O.w[w] = R.w[w] = 0;
        bool keep = false;
        for (uint32_t q = q0; q < q1; ++q) {
            const uint64_t* src = a.hscratch + (uint64_t)q * 3 * a.nwp;
            hub_combine<WPL>(O, R, load_row<WPL>(src + off), load_row<WPL>(src + a.nwp + off));
            keep |= (a.hflag[q] & HF_KEEP) != 0;
        }
        if (keep) atomicOr(&s_keep, 1u);
        hub_block_reduce<G, WPL>(O, R, s_or, s_rc);
        if (j == 0) {
            const uint8_t st = a.sstate[rep], fo = a.flg_cur[rep];
            const bool lag = (st & FL_LAG) != 0, cbk = (st & SE_FM2) != 0;
            const bool keep_all = s_keep || (st & SE_FM3);  // read by a callback, or pushed by this node
            Row<WPL> sp = load_row<WPL>(a.base + rep * a.nwp + off);
            if (lag) {
                const Row<WPL> of = load_row<WPL>(a.F_prev + rep * a.nwp + off);
#pragma unroll
                for (int w = 0; w < WPL; ++w) sp.w[w] |= of.w[w];
            }
            Row<WPL> S = sp;
            if (ca & CA_INJ) {  // (1) client broadcasts of this round
                uint32_t lo = 0, hi = inj_n(a);
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (inj_p(a)[2 * mid] < i) lo = mid + 1;
                    else hi = mid;
                }
                for (uint32_t k = lo; k < inj_n(a) && inj_p(a)[2 * k] == i; ++k) {
                    const uint32_t lane = inj_p(a)[2 * k + 1];
                    const uint32_t word = lane >> 6;
                    if (word / WPL == (uint32_t)lg) set_lane_bit<WPL>(S, word % WPL, lane & 63);
                }
            }
            // (2) node broadcasts and pushes: every new bit's first deliverer claims it
            unsigned long long cl_recip = 0, cb_new = 0;
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                const uint64_t claim = O.w[w] & ~S.w[w];
                cl_recip += __popcll(claim & R.w[w]);
                S.w[w] |= claim;
            }
            // (3) its callback: each chunk's exclusive prefix, then every peer's set
            if (cbk) {
                Row<WPL> P = S;
                for (uint32_t q = c0; q < c1; ++q) {
                    uint64_t* qr = a.hscratch + (uint64_t)q * 3 * a.nwp + 2 * a.nwp + off;
                    const Row<WPL> Qc = load_row<WPL>(qr);
                    store_row<WPL>(qr, P);
#pragma unroll
                    for (int w = 0; w < WPL; ++w) P.w[w] |= Qc.w[w];
                }
#pragma unroll
                for (int w = 0; w < WPL; ++w) {
                    cb_new += __popcll(P.w[w] & ~S.w[w]);
                    S.w[w] = P.w[w];
                }
                if (lg == 0 && a.pushany) a.pushany[rep] = 0;  // hub_sync_push sets it where a push had content
            }
            Row<WPL> F;
            unsigned long long T = 0;
            const uint64_t g = gid_of(a, i);
#pragma unroll
            for (int w = 0; w < WPL; ++w) {
                F.w[w] = S.w[w] & ~sp.w[w];
                T += __popcll(F.w[w]);
                if (F.w[w]) {
                    const uint64_t idx = g * a.nw + a.word0 + off + w;
                    c_hash += gg_word_hash(idx, F.w[w]);
                }
            }
            const bool any = ((__ballot(T != 0) >> gshift) & gmask) != 0;
            const bool zm = (fo & FL_ACT) != 0;
            if (any || zm) store_row<WPL>(a.F_cur + rep * a.nwp + off, F);
            if (keep_all) {
                if (lag) store_row<WPL>(a.base + rep * a.nwp + off, sp);
            } else if (any || lag) {
                store_row<WPL>(a.base + rep * a.nwp + off, S);
            }
            if (any && a.sat_new) sat_mark<G, WPL>(a, S, rep, lg);
            const uint64_t dout = (uint64_t)(a.in_ptr[i + 1] - a.in_ptr[i]);
            c_new += T;
            c_fwd += dout * T - cl_recip - cb_new;
            if (lg == 0) {
                if (any || zm) a.flg_cur[rep] = any ? (uint8_t)(FL_ACT | (keep_all ? FL_LAG : 0)) : (uint8_t)0;
                a.hlive[h] = 0;
                c_active += 1;
                c_nact += any ? 1 : 0;
                c_nactdeg += any ? dout : 0;
                c_bytes += 16 + 3 + (uint64_t)(c1 - c0) * (4 + 16ull * a.nwp + (cbk ? 16ull * a.nwp : 0)) +
                           8ull * a.nwp * (1 + (lag ? 1 : 0) + ((any || zm) ? 1 : 0) + ((keep_all ? lag : any || lag) ? 1 : 0));
            }
        }
        __syncthreads();  // LDS reuse
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
    acc[C_NACT] = c_nact;
    acc[C_NACTDEG] = c_nactdeg;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

template <int G, int WPL>
__global__ __launch_bounds__(kBlock) void hub_sync_push(RoundArgs a) {
    constexpr int NGB = kBlock / G;
    __shared__ uint64_t s_q[NGB * G * WPL];
    __shared__ unsigned long long s_red[kBlock / 64][C_NUM];
    __shared__ uint32_t s_any;
    const unsigned long long t_start = clock100();
    const int j = threadIdx.x / G, lg = threadIdx.x % G;
    const uint64_t off = (uint64_t)lg * WPL;
    const int gshift = (threadIdx.x & 63) / G * G;
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
    unsigned long long c_push = 0, c_bytes = 0;
    for (uint64_t c = blockIdx.x; c < a.n_hchunks; c += gridDim.x) {
        const uint32_t fl = a.hflag[c];
        if ((fl & (HF_LIVE | HF_CB)) != (HF_LIVE | HF_CB)) continue;  // block-uniform
        const HubChunk hc = a.hchunks[c];
        if (threadIdx.x == 0) s_any = 0;
        const uint32_t per = (hc.n + NGB - 1) / NGB;
        const int64_t e0 = hc.e0 + (int64_t)j * per;
        const int64_t e1 = min(hc.e0 + (int64_t)hc.n, e0 + (int64_t)per);
        auto peer_set = [&](int64_t e, uint32_t& w) {
            w = a.in_col[e] & kColMask;
            Row<WPL> r = load_row<WPL>(a.base + (uint64_t)w * a.nwp + off);
            if (bit_at(a.ibits, w) && (a.sstate[w] & FL_LAG)) {
                const Row<WPL> f = load_row<WPL>(a.F_prev + (uint64_t)w * a.nwp + off);
#pragma unroll
                for (int q = 0; q < WPL; ++q) r.w[q] |= f.w[q];
            }
            return r;
        };
        // the OR of each node group's slice, then every slice's exclusive prefix in order
        Row<WPL> X;
#pragma unroll
        for (int q = 0; q < WPL; ++q) X.w[q] = 0;
        for (int64_t e = e0; e < e1; ++e) {
            uint32_t w;
            const Row<WPL> r = peer_set(e, w);
#pragma unroll
            for (int q = 0; q < WPL; ++q) X.w[q] |= r.w[q];
        }
#pragma unroll
        for (int q = 0; q < WPL; ++q) s_q[j * G * WPL + lg * WPL + q] = X.w[q];
        __syncthreads();
        Row<WPL> P = load_row<WPL>(a.hscratch + c * 3 * a.nwp + 2 * a.nwp + off);  // S before the chunk
        for (int jj = 0; jj < j; ++jj) {
#pragma unroll
            for (int q = 0; q < WPL; ++q) P.w[q] |= s_q[jj * G * WPL + lg * WPL + q];
        }
        bool pushed = false;
        for (int64_t e = e0; e < e1; ++e) {
            uint32_t w;
            const Row<WPL> r = peer_set(e, w);
            unsigned long long pp = 0;
#pragma unroll
            for (int q = 0; q < WPL; ++q) {
                pp += __popcll(P.w[q] & ~r.w[q]);
                P.w[q] |= r.w[q];
            }
            c_push += pp;
            const bool nz = ((__ballot(pp != 0) >> gshift) & gmask) != 0;
            if (lg == 0) {
                if (a.pushb) a.pushb[e] = nz ? 1 : 0;
                pushed |= nz;
                if (nz && a.mark_next && w < a.n_own) a.cand_next[a.own0 + w] = CA_NODE;
            }
        }
        if (lg == 0 && e1 > e0) c_bytes += (uint64_t)(e1 - e0) * (8 + 2 * 8ull * a.nwp + 1);
        if (pushed) atomicOr(&s_any, 1u);
        __syncthreads();
        if (threadIdx.x == 0 && s_any && a.pushany) a.pushany[a.own0 + hc.node] = 1;
        __syncthreads();  // LDS reuse
    }
    unsigned long long acc[C_NUM];
#pragma unroll
    for (int k = 0; k < C_NUM; ++k) acc[k] = 0;
    acc[C_PUSH] = c_push;
    acc[C_PUSH_DELIV] = c_push;
    acc[C_NEXT_ACKS] = c_push;
    acc[C_BYTES] = c_bytes;
    flush_counters(a, acc, s_red, t_start, K_STREAM);
}

// Senders with out-degree > hub_deg that were active (or pushed) last round
// mark their owned receivers; one block per out-edge chunk (sparse rounds).
__global__ __launch_bounds__(kBlock) void hub_mark(RoundArgs a) {
    const unsigned long long t_start = clock100();
    if (dense_round(a)) {
        noop_exit(a, K_PREP, t_start);
        return;
    }
    for (uint64_t c = blockIdx.x; c < a.n_mchunks; c += gridDim.x) {
        const HubChunk hc = a.mchunks[c];
        const uint64_t u = a.own0 + hc.node;
        if (!((a.flg_prev[u] & FL_ACT) || bit_at(a.fired_m3, u))) continue;
        for (uint32_t t = threadIdx.x; t < hc.n; t += kBlock) {
            const uint64_t w = a.out_col[hc.e0 + t] & kColMask;
            if (w >= a.n_own) continue;
            a.cand[w] = CA_NODE;
            if (!a.stream_ok) a.tile_cand[w / a.tile_nodes] = 1;
        }
    }
    if (threadIdx.x == 0) stamp(a, K_PREP, t_start);
}

// Host reads (gg_read_bits, gg_delivery_rounds): rows gathered by local row;
// a set is base | F of the last round where that round's flag says LAG.
__global__ void gather_sets(const uint32_t* rows, uint64_t n, const uint64_t* base, const uint64_t* F_last,
                            const uint8_t* flg_last, uint32_t nwp, uint64_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * nwp) return;
    const uint64_t k = t / nwp, j = t % nwp, r = rows[k];
    uint64_t w = base[r * nwp + j];
    if (flg_last && (flg_last[r] & FL_LAG)) w |= F_last[r * nwp + j];
    out[t] = w;
}

__global__ void gather_rounds(const uint32_t* rows, uint64_t n, const int32_t* dr, uint32_t W, int32_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * W) return;
    out[t] = dr[(uint64_t)rows[t / W] * W + t % W];
}

// First-seen round of every new bit (GG_TRACK_DELIVERY only; observation).
// F_cur: the new bits of round r, or (prev != nullptr, double-buffered rounds) the sets of r
__global__ void track_delivery(const uint64_t* F_cur, const uint8_t* flg_cur, int32_t* dr, uint64_t n_own,
                               uint64_t own0, uint32_t nwp, uint32_t nw, uint32_t W, int32_t round,
                               const uint64_t* prev) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_own * nw) return;
    const uint64_t i = t / nw, j = t % nw;
    if (!(flg_cur[own0 + i] & FL_ACT)) return;
    uint64_t x = F_cur[(own0 + i) * nwp + j];
    if (prev) x &= ~prev[(own0 + i) * nwp + j];
    while (x) {
        const int b = __builtin_ctzll(x);
        x &= x - 1;
        dr[i * W + j * 64 + b] = round;
    }
}

// Sum a round's 64 counter slots into one (stamps: max, see kStamp0). One block
// per round, one thread per counter.
// The F rows of round q, the last double-buffered round, for the F-row rounds
// that follow it: F = set(q) & ~set(q-1) for the nodes flagged ACT in q (every
// other F row is still zero: double-buffered rounds write none).
__global__ void materialize_F(const uint64_t* set_q, const uint64_t* set_qm1, const uint8_t* flg_q, uint64_t* F_q,
                              uint64_t n_own, uint32_t nwp) {
    const uint64_t n = n_own * nwp;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        if (!(flg_q[t / nwp] & FL_ACT)) continue;
        F_q[t] = set_q[t] & ~set_qm1[t];
    }
}

// Zero n 8-byte words (16-byte stores, an 8-byte tail). Used instead of
// hipMemsetAsync inside captured launch sequences: replays of a graph whose
// memset node was captured in an engine's first batch were seen to fill the
// counter slots with pointer-like words (16-byte pattern) instead of zeros,
// depending on the process's other allocations (round 5, 2 ranks on one GPU).
__global__ void zero_words(uint64_t* p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n2 = n / 2;
    ulonglong2* q = reinterpret_cast<ulonglong2*>(p);
    for (uint64_t k = i; k < n2; k += stride) q[k] = make_ulonglong2(0ull, 0ull);
    if (i == 0 && (n & 1)) p[n - 1] = 0;
}

// (clear: zero the slots read, so the next batch needs no zeroing launch)
__global__ void fold_slots(unsigned long long* ctr, unsigned long long* out, uint32_t clear) {
    const int j = threadIdx.x;
    unsigned long long* c = ctr + (size_t)blockIdx.x * kSlots * kCounters;
    const bool stampj = j >= kStamp0 && j < kStamp0 + 2 * K_NKIND;
    unsigned long long v = 0;
    for (int k = 0; k < kSlots; ++k) {
        const unsigned long long x = c[k * kCounters + j];
        v = stampj ? (x > v ? x : v) : v + x;
    }
    out[(size_t)blockIdx.x * kCounters + j] = v;
    if (clear)
        for (int k = 0; k < kSlots; ++k) c[k * kCounters + j] = 0;
}

// Episode reset: fill up to kResetSegs arrays (8-byte words) and start the
// sync timers, in one launch.
constexpr int kResetSegs = 32;
struct ResetSeg {
    uint64_t* p;
    uint64_t n;    // 8-byte words
    uint64_t val;
};
struct ResetArgs {
    ResetSeg seg[kResetSegs];
    int n_seg;
    int32_t* sync_next;
    uint32_t* sync_k;
    uint64_t n_own, ghost0, n_ghost;  // timers: owned rows and ghost rows
    const uint32_t* gid;
    uint64_t seed;
    uint64_t sync_mix, sync_rcp;  // gg_sync_interval_rcp's constants (gg_mix64(seed ^ GG_TAG_SYNC), gg_sync_rcp)
    uint32_t sync_base, sync_jitter;
    // an F buffer whose rows are zero where their flag byte is: only the flagged
    // rows and the flags are cleared (or nullptr)
    uint64_t* sparse_F;
    uint8_t* sparse_flg;  // [sparse_rows] flag bytes
    uint64_t sparse_rows;
    uint32_t nwp;         // even, <= 128
};

__global__ __launch_bounds__(kBlock) void reset_state(ResetArgs ra) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t t0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (int q = 0; q < ra.n_seg; ++q) {
        const ResetSeg s = ra.seg[q];
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        const u64x2 v = {s.val, s.val};
        // blocks own 16 KiB pieces (2048 words = 4 x kBlock 16-byte chunks): 4
        // coalesced 16-byte stores per thread, streamed past the caches
        constexpr uint64_t kPiece = 8 * kBlock;  // words
        const uint64_t pieces = s.n / kPiece;
        for (uint64_t b = blockIdx.x; b < pieces; b += gridDim.x) {
            u64x2* p = reinterpret_cast<u64x2*>(s.p + b * kPiece) + threadIdx.x;
#pragma unroll
            for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v, p + k * kBlock);  // chunk < 4 * kBlock
        }
        for (uint64_t w = pieces * kPiece + t0; w < s.n; w += stride) s.p[w] = s.val;
    }
    if (ra.sparse_F) {
        // one lane per 16-byte piece of a row, the rows of a wave whole (nwp / 2
        // divides 64, and so the stride): every lane of the wave has read the
        // row's flag byte before the piece-0 lane clears it
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        const uint32_t pieces = ra.nwp / 2;
        uint8_t* flg = reinterpret_cast<uint8_t*>(ra.sparse_flg);
        const uint64_t n = ra.sparse_rows * pieces;
        for (uint64_t t = t0; t < n; t += stride) {
            const uint64_t row = t / pieces;
            const uint32_t pc = (uint32_t)(t % pieces);
            if (!flg[row]) continue;
            __builtin_nontemporal_store((u64x2){0ull, 0ull}, reinterpret_cast<u64x2*>(ra.sparse_F + row * ra.nwp) + pc);
            if (pc == 0) flg[row] = 0;
        }
    }
    for (uint64_t t = t0; t < ra.n_own + ra.n_ghost; t += stride) {
        const uint64_t i = t < ra.n_own ? t : ra.ghost0 + (t - ra.n_own);
        ra.sync_k[i] = 0;
        ra.sync_next[i] = (int32_t)gg_sync_interval_rcp(ra.sync_mix, ra.sync_rcp, ra.gid ? (uint64_t)ra.gid[i] : i, 0,
                                                        ra.sync_base, ra.sync_jitter);
    }
}

// Seeded bisection groups of the local rows (padding rows: group 0, unused).
__global__ void fill_seeded_groups(uint8_t* grp, uint64_t rows, uint64_t n_valid, const uint32_t* gid,
                                   uint64_t seed, uint64_t epoch_seed) {
    const uint64_t rr = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rr >= rows) return;
    const uint32_t g = gid ? gid[rr] : (uint32_t)rr;
    grp[rr] = (rr < n_valid && g != ~0u) ? (uint8_t)gg_part_group(seed, epoch_seed, g) : 0;
}

// In-edge bitmap of a partition window: bit e = the sender and the receiver of
// in-edge e are in different groups (messages between them are dropped while
// the window is active). One thread per 64-edge word.
__global__ void build_edge_mask(const int64_t* in_ptr, const uint32_t* in_col, uint64_t n_own, uint64_t n_edges,
                                const uint8_t* grp, uint64_t* out) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t e0 = w * 64;
    if (e0 >= n_edges) return;
    uint64_t lo = 0, hi = n_own;  // the node whose in-list holds e0: in_ptr[v] <= e0 < in_ptr[v+1]
    while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if ((uint64_t)in_ptr[mid] <= e0) lo = mid;
        else hi = mid - 1;
    }
    uint64_t v = lo, bits = 0;
    for (uint64_t e = e0; e < e0 + 64 && e < n_edges; ++e) {
        while ((uint64_t)in_ptr[v + 1] <= e) ++v;
        if (grp[in_col[e] & kColMask] != grp[v]) bits |= 1ull << (e - e0);
    }
    out[w] = bits;
}

// ---------------------------------------------------------------------------
// Sharded exchange: only what a peer reads next round crosses.
// After its round-r kernels, engine p sends peer q, for the owned nodes q holds
// as ghosts (q's send list, `send_idx`):
//   kind F  the node's F row, if it is ACT in round r (non-zero: it forwards
//           these bits in r+1, broadcast.go:55; only first receipts cross, :64-76)
//   kind S  the node's whole set (base | F when LAG, folded here), if q reads it
//           in r+1: the node pushes in r+1 (it fired in r-2, :104-108) or a
//           neighbour on q runs its sync callback in r+1 (fired in r-1; marked by
//           mark_set_needs from p's own copy of that ghost's timer, :97-101)
// Sync timers are not exchanged: every engine runs its ghosts' timers itself.
// Segment for one peer (at a fixed capacity offset): a 16-byte header
// {entries, payload bytes}, then entries of `stride` bytes: a 16-byte head
// {position in the send list | XK_SET, 0, row word when nwp == 1} and the row
// (nwp >= 2). A quiet round sends headers only.
// The device-driven exchange (below) packs tile segments instead, with no head
// per entry (round 5: at W = 64 the heads were half of every entry):
//   header   {records | rows << 32, payload bytes}
//   records  [ceil(n / 256)] slots of 80 B, one per send tile (256 consecutive
//            send-list entries) that ships anything, in arrival order:
//            {tile's first entry - the peer's first | first row << 32, 0,
//             F bitmap (4 words), S bitmap (4 words)}
//   rows     [2 n] rows of W/8 bytes (8 at W = 64): a tile's rows in entry
//            order, F before S for one entry; entry j's F row sits at
//            first row + (F and S bits below j), its S row one after its F row
// so a dense round ships 8 bytes a sender row at W = 64 (plus 80 B a tile)
// instead of 16.
constexpr uint32_t XK_SET = 0x80000000u;
constexpr uint32_t kTileRec = 80;  // tile record bytes
__host__ __device__ inline uint64_t tile_rows_off(uint64_t n_entries) {  // rows area of a tile segment
    return 16 + kTileRec * ((n_entries + kBlock - 1) / kBlock);
}

// Device-driven exchange (gg_dist_ipc_*): every engine exports one window of
// uncached HBM — flags, then two receive buffers by the parity of the exchange
// sequence number seq (one per round, never reset) — and maps its peers'
// windows. The sender packs each peer's segment straight into the peer's
// receive buffer over xGMI, fences (system scope) and sets the peer's ready
// slot to seq + 1; the receiver's unpack waits for those slots, reads, and its
// last block sets each sender's consumed slot to seq + 1 and advances seq; a
// sender waits for consumed >= seq - 1 before packing into a buffer (seq - 2
// used it last). seq lives in device memory, so the round is a fixed launch
// sequence with no host wait and no collective call, and a captured batch of
// rounds replays for any seq.
// Waits are bounded (IpcArgs::spin_limit sleeps, default kSpinLimit ≈ 15 s): a
// peer that never arrives sets the engine's error word instead of hanging the
// GPU. Once the word is set every later wait, pack and unpack of the engine
// returns at once (the exchange is dead until a new topology is exported and
// imported again), so a missing peer costs one bound, not one per wait of every
// queued round: the word counts the waits that ran out (at most one per
// engine, plus any running concurrently with the first).
constexpr uint64_t kWinHdr = 4096;         // flags area at the start of a window
constexpr uint32_t kWinReady = 0;          // u64 ready[64]: by source part
constexpr uint32_t kWinConsumed = 512;     // u64 consumed[64]: by receiving part
constexpr uint32_t kSpinLimit = 1u << 25;

__device__ __forceinline__ bool ipc_failed(const uint32_t* err) {
    return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// Wait until flags[q] >= want for every q in mask (system-scope acquire loads).
// One thread calls it; false after the bound (err counts it) or as soon as
// another wait of this engine has run out (err already set).
__device__ __forceinline__ bool wait_flags(const uint64_t* flags, uint64_t mask, uint64_t want, uint32_t* err,
                                           uint32_t limit) {
    for (; mask; mask &= mask - 1) {
        const int q = __ffsll((long long)mask) - 1;
        uint32_t it = 0;
        while (__hip_atomic_load(flags + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            if ((it & 255u) == 0u && ipc_failed(err)) return false;
            if (++it > limit) {
                atomicAdd(err, 1u);
                return false;
            }
            __builtin_amdgcn_s_sleep(16);
        }
    }
    return true;
}

struct IpcArgs {
    uint8_t* const* peer_win;  // [parts] mapped peer windows (nullptr: no IPC exchange)
    const uint64_t* peer_off;  // [parts] where this engine's segment lands in peer q's receive buffer
    const uint64_t* peer_rbuf; // [parts] peer q's receive buffer bytes (the parity stride)
    uint64_t* my_win;          // this engine's window
    uint64_t rbuf;             // this engine's receive buffer bytes
    uint64_t send_mask;        // parts this engine sends to
    uint64_t recv_mask;        // parts this engine receives from
    uint64_t* seq;             // exchange sequence number of this round (advanced by unpack)
    uint32_t* ticket;          // unpack's last-block counter
    uint32_t* err;             // waits that ran out (non-zero: the exchange is dead)
    uint32_t spin_limit;       // sleeps before a wait gives up (kSpinLimit; GG_IPC_SPIN_LIMIT for tests)
};

// One 64-thread block before pack_ghosts (which = 0: the peers consumed round
// seq - 2, whose buffers this round reuses) or before unpack_ghosts (which = 1:
// every source's segment of round seq has landed): lane q waits for part q. A
// single small block spins, so the kernels it guards hold no CU while a peer on
// the same GPU still needs one.
__global__ void ipc_wait(IpcArgs ip, int which) {
    const uint32_t q = threadIdx.x;
    const uint64_t seq = *ip.seq;
    const uint64_t mask = which ? ip.recv_mask : ip.send_mask;
    if (q >= 64 || !((mask >> q) & 1ull)) return;
    if (which == 0 && seq < 2) return;
    if (ipc_failed(ip.err)) return;
    const uint64_t* flags =
        reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(ip.my_win) + (which ? kWinReady : kWinConsumed));
    wait_flags(flags, 1ull << q, which ? seq + 1 : seq - 1, ip.err, ip.spin_limit);
}

// Peer q's segment for this engine in round seq's receive buffer.
__device__ __forceinline__ uint8_t* ipc_segment(const IpcArgs& ip, uint32_t q, uint64_t seq) {
    return ip.peer_win[q] + kWinHdr + (seq & 1) * ip.peer_rbuf[q] + ip.peer_off[q];
}

// Need bits (device-driven exchange, round 6): after its round r, part p writes
// into each peer q's window one bit per ghost it holds from q — "some owned
// receiver of this ghost is not saturated" (the lean digest, lsat == 0) — and q
// packs round r+1 without the F rows whose bit is clear. Exact when no client
// broadcasts anything in rounds r and r+1 (the host's condition; every part
// sees every broadcast): a saturated receiver holds every lane that can reach
// it among those broadcast through r — the digest is judged against targets
// that already count them (can't schedule into the past), and a clear by a
// later target change only forgets bits — and an F row of round r+1 carries
// only such lanes then; a row that is not sent is a ghost that sent nothing
// (its stale row is cleared as for any quiet ghost).
// Three slots rotate by seq % 3: q reads slot (seq - 1) % 3 in its pack of round
// seq while p may already write slot seq % 3; p writes a slot again three rounds
// later, after ipc_wait(0) saw q's unpack of round seq + 1, i.e. after q's pack
// of round seq + 1 read it. The slots sit in the sender's region of the parity-0
// receive buffer, after its rows area.
struct NeedWord {
    uint32_t peer;  // source part of the ghosts (the part we write to)
    uint32_t j0;    // first ghost of the word, relative to that source's first (a multiple of 64)
    uint32_t n;     // ghosts in the word (<= 64)
};
__host__ __device__ inline uint64_t need_slot_bytes(uint64_t n) { return (n + 127) / 128 * 16; }

struct XchgTile {
    uint32_t peer;   // part index of the destination
    uint32_t k0;     // first send entry of the tile (global send-list index)
    uint32_t n;      // entries (<= kBlock), all for `peer`
    uint32_t first;  // first send entry of `peer`
};

struct PackArgs {
    const uint64_t* F_cur;
    const uint64_t* base;
    const uint64_t* set_prev;   // double-buffered round: no F rows, F = base & ~set_prev
    const uint8_t* flg_cur;
    const uint64_t* fired_m2;   // round r-2: owned pushers of round r+1 (SYNC only)
    uint8_t* needmark;          // [n_send] set read by a callback on the peer in r+1 (cleared here)
    const uint32_t* send_idx;   // [n_send] owned local row of each send entry
    const XchgTile* tiles;
    uint32_t n_tiles;
    uint32_t* cnt;              // [parts] entries written per peer this round
    uint8_t* out;
    const uint64_t* seg_off;    // [parts] byte offset of each peer's segment in `out`
    uint32_t nwp, stride;
    int32_t sync;               // sets may be read next round
    IpcArgs ipc;                // device-driven exchange: segments go straight to the peers
    // finish_pack's work, done by the last block to finish (ticket): no launch of its own
    uint32_t* ticket;           // last-block counter (reset by that block)
    uint32_t parts, self;
    unsigned long long* seg_bytes;
    unsigned long long* payload;
    const uint32_t* sfirst;     // [parts + 1] first send entry of each peer (tile segments)
    // need bits of the round before (nullptr: every F row ships): window offset of
    // each source's slot 0 and slot bytes, and the sources that write them
    const uint64_t* need_in;
    const uint64_t* need_bytes_in;
    uint64_t need_peers;
};

__device__ __forceinline__ void finish_pack_body(uint32_t* cnt, uint8_t* out, const uint64_t* seg_off, uint32_t parts,
                                                 uint32_t self, uint32_t stride, unsigned long long* seg_bytes,
                                                 unsigned long long* payload, const IpcArgs& ip, uint32_t nwp);

__global__ __launch_bounds__(kBlock) void pack_ghosts(PackArgs x) {
    __shared__ uint32_t s_row[2 * kBlock], s_head[2 * kBlock];
    __shared__ uint32_t s_cnt[kBlock / 64];
    __shared__ uint32_t s_base, s_tot, s_rec;
    __shared__ unsigned long long s_bm[2][kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool tf = x.ipc.peer_win != nullptr;  // tile segments (device-driven exchange)
    // 16-byte chunks per entry (tile segments: per row; W = 64: one 8-byte word)
    const uint32_t cpe = tf ? (x.nwp >= 2 ? x.nwp / 2 : 1) : (x.nwp >= 2 ? 1 + x.nwp / 2 : 1);
    const uint64_t rowb = 8ull * x.nwp;
    // a dead exchange (a wait ran out; ipc_wait, the only writer, ran before this
    // launch, so every block reads the same word): store nothing into the peers
    if (x.ipc.peer_win && ipc_failed(x.ipc.err)) return;
    const uint64_t seq = x.ipc.peer_win ? *x.ipc.seq : 0;  // (ipc_wait ran before: the buffers are free)
    for (uint32_t ti = blockIdx.x; ti < x.n_tiles; ti += gridDim.x) {
        const XchgTile t = x.tiles[ti];
        const uint32_t k = t.k0 + threadIdx.x;
        const bool valid = threadIdx.x < t.n;
        const uint32_t u = valid ? x.send_idx[k] : 0u;
        const uint8_t fl = valid ? x.flg_cur[u] : (uint8_t)0;
        bool fa = (fl & FL_ACT) != 0;
        if (fa && x.need_in && ((x.need_peers >> t.peer) & 1ull)) {  // the peer's need bit of this entry
            const uint32_t j = k - t.first;
            const uint8_t* nb = reinterpret_cast<const uint8_t*>(x.ipc.my_win) + x.need_in[t.peer] +
                                ((seq + 2) % 3) * x.need_bytes_in[t.peer];
            fa = ((*reinterpret_cast<const unsigned long long*>(nb + (j >> 6) * 8) >> (j & 63)) & 1ull) != 0;
        }
        bool sn = false;
        if (valid && x.sync) {
            const bool nm = x.needmark[k] != 0;
            if (nm) x.needmark[k] = 0;
            sn = nm || bit_at(x.fired_m2, u);
        }
        const uint32_t c = (fa ? 1u : 0u) + (sn ? 1u : 0u);
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_cnt[wave] = incl;
        if (tf) {
            const unsigned long long bf = __ballot(fa), bs = __ballot(sn);
            if (lane == 0) {
                s_bm[0][wave] = bf;
                s_bm[1][wave] = bs;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int w = 0; w < kBlock / 64; ++w) {
                const uint32_t v = s_cnt[w];
                s_cnt[w] = tot;
                tot += v;
            }
            s_tot = tot;
            s_base = tot ? atomicAdd(&x.cnt[t.peer], tot) : 0u;
            s_rec = (tf && tot) ? atomicAdd(&x.cnt[x.parts + t.peer], 1u) : 0u;
        }
        __syncthreads();
        uint32_t pos = s_cnt[wave] + incl - c;
        const uint32_t idx = k - t.first;
        if (fa) {
            s_row[pos] = u;
            s_head[pos] = idx;
            ++pos;
        }
        if (sn) {
            s_row[pos] = u | ((fl & FL_LAG) ? XK_SET : 0u);  // bit 31: fold F into the set
            s_head[pos] = idx | XK_SET;
        }
        __syncthreads();
        if (tf) {
            // the tile's record and its rows (no head per entry)
            uint8_t* tseg = ipc_segment(x.ipc, t.peer, seq);
            if (threadIdx.x < 5 && s_tot) {
                ulonglong2 v;
                if (threadIdx.x == 0) {
                    v.x = (unsigned long long)(t.k0 - t.first) | ((unsigned long long)s_base << 32);
                    v.y = 0;
                } else {
                    const int q = threadIdx.x - 1;  // bitmap words F0 F1 | F2 F3 | S0 S1 | S2 S3
                    v.x = s_bm[q >> 1][(q & 1) * 2];
                    v.y = s_bm[q >> 1][(q & 1) * 2 + 1];
                }
                *reinterpret_cast<ulonglong2*>(tseg + 16 + (uint64_t)s_rec * kTileRec + 16 * threadIdx.x) = v;
            }
            uint8_t* rows = tseg + tile_rows_off(x.sfirst[t.peer + 1] - x.sfirst[t.peer]);
            for (uint32_t e = threadIdx.x; e < s_tot * cpe; e += kBlock) {
                const uint32_t j = e / cpe, ch = e % cpe;
                const uint32_t hd = s_head[j], rr = s_row[j];
                const bool set = (hd & XK_SET) != 0, lag = (rr & XK_SET) != 0;
                const uint64_t u2 = rr & ~XK_SET;
                uint8_t* dst = rows + (uint64_t)(s_base + j) * rowb;
                if (x.nwp == 1) {
                    *reinterpret_cast<uint64_t*>(dst) = set ? (x.base[u2] | (lag ? x.F_cur[u2] : 0ull))
                                                            : (x.set_prev ? x.base[u2] & ~x.set_prev[u2] : x.F_cur[u2]);
                    continue;
                }
                const uint64_t o = u2 * x.nwp + 2 * ch;
                ulonglong2 v;
                if (set) {
                    v = *reinterpret_cast<const ulonglong2*>(x.base + o);
                    if (lag) {
                        const ulonglong2 f = *reinterpret_cast<const ulonglong2*>(x.F_cur + o);
                        v.x |= f.x;
                        v.y |= f.y;
                    }
                } else if (x.set_prev) {
                    v = *reinterpret_cast<const ulonglong2*>(x.base + o);
                    const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(x.set_prev + o);
                    v.x &= ~q.x;
                    v.y &= ~q.y;
                } else {
                    v = *reinterpret_cast<const ulonglong2*>(x.F_cur + o);
                }
                *reinterpret_cast<ulonglong2*>(dst + 16 * ch) = v;
            }
            __syncthreads();  // LDS reuse
            continue;
        }
        uint8_t* seg = (x.ipc.peer_win ? ipc_segment(x.ipc, t.peer, seq) : x.out + x.seg_off[t.peer]) + 16 +
                       (uint64_t)s_base * x.stride;
        for (uint32_t e = threadIdx.x; e < s_tot * cpe; e += kBlock) {
            const uint32_t j = e / cpe, ch = e % cpe;
            const uint32_t hd = s_head[j], rr = s_row[j];
            const bool set = (hd & XK_SET) != 0, lag = (rr & XK_SET) != 0;
            const uint64_t u2 = rr & ~XK_SET;
            uint8_t* dst = seg + (uint64_t)j * x.stride + ch * 16;
            ulonglong2 v;
            if (ch == 0) {  // head (+ the row word when nwp == 1)
                v.x = hd;
                v.y = 0;
                if (x.nwp == 1)
                    v.y = set ? (x.base[u2] | (lag ? x.F_cur[u2] : 0ull))
                              : (x.set_prev ? x.base[u2] & ~x.set_prev[u2] : x.F_cur[u2]);
            } else {
                const uint64_t o = u2 * x.nwp + 2 * (ch - 1);
                if (set) {
                    v = *reinterpret_cast<const ulonglong2*>(x.base + o);
                    if (lag) {
                        const ulonglong2 f = *reinterpret_cast<const ulonglong2*>(x.F_cur + o);
                        v.x |= f.x;
                        v.y |= f.y;
                    }
                } else if (x.set_prev) {
                    v = *reinterpret_cast<const ulonglong2*>(x.base + o);
                    const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(x.set_prev + o);
                    v.x &= ~q.x;
                    v.y &= ~q.y;
                } else {
                    v = *reinterpret_cast<const ulonglong2*>(x.F_cur + o);
                }
            }
            *reinterpret_cast<ulonglong2*>(dst) = v;
        }
        __syncthreads();  // LDS reuse
    }
    if (x.ipc.peer_win) __threadfence_system();  // this thread's segment stores performed before the ready flags
    // the last block to finish runs finish_pack (every block's counts and stores are in)
    __shared__ uint32_t s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t t = atomicAdd(x.ticket, 1u);
        s_last = t == gridDim.x - 1 ? 1u : 0u;
        if (s_last) {
            *x.ticket = 0;
            __threadfence();
        }
    }
    __syncthreads();
    if (s_last && threadIdx.x < 64) finish_pack_body(x.cnt, x.out, x.seg_off, x.parts, x.self, x.stride, x.seg_bytes,
                                                     x.payload, x.ipc, x.nwp);
}

struct NeedArgs {
    const NeedWord* words;
    uint32_t n_words;
    const uint32_t* gfirst;     // [parts + 1] first ghost (exchange order) from each source
    const uint32_t* grow;       // ghost row of the g-th ghost, or nullptr (the same)
    const int64_t* gout_ptr;    // ghost -> owned receivers
    const uint32_t* gout_col;
    const uint8_t* lsat;        // the lean digest of the owned rows (after this round)
    const uint64_t* need_out;   // [parts] our slot 0 in part q's region (after its rows area)
    const uint64_t* need_bytes; // [parts] slot bytes
    IpcArgs ipc;
};

// One wave per word of 64 ghosts: the ghost's bit = some owned receiver of it is
// not saturated; the word goes into the source part's window (slot seq % 3).
__global__ __launch_bounds__(kBlock) void need_bits(NeedArgs a) {
    if (ipc_failed(a.ipc.err)) return;
    const uint64_t seq = *a.ipc.seq;
    const int lane = threadIdx.x & 63;
    for (uint32_t w = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < a.n_words; w += gridDim.x * (kBlock / 64)) {
        const NeedWord nw = a.words[w];
        bool need = false;
        if ((uint32_t)lane < nw.n) {
            const uint64_t g0 = (uint64_t)a.gfirst[nw.peer] + nw.j0 + lane;
            const uint64_t g = a.grow ? a.grow[g0] : g0;
            for (int64_t e = a.gout_ptr[g]; e < a.gout_ptr[g + 1] && !need; ++e) need = a.lsat[a.gout_col[e]] == 0;
        }
        const unsigned long long bits = __ballot(need);
        if (lane == 0) {
            uint8_t* dst = a.ipc.peer_win[nw.peer] + kWinHdr + a.ipc.peer_off[nw.peer] + a.need_out[nw.peer] +
                           (seq % 3) * a.need_bytes[nw.peer] + (nw.j0 >> 6) * 8;
            *reinterpret_cast<unsigned long long*>(dst) = bits;
        }
    }
    __threadfence_system();  // before pack_ghosts' ready flags (a later kernel of this stream)
}

// After pack_ghosts: each peer's header, its byte count for an exact-size
// exchange, the round's payload bytes; counters reset for the next round.
// (threads 0..63 of one block; pack_ghosts' last block, or a launch of its own
// when no tile has entries to pack)
__device__ __forceinline__ void finish_pack_body(uint32_t* cnt, uint8_t* out, const uint64_t* seg_off, uint32_t parts,
                                                 uint32_t self, uint32_t stride, unsigned long long* seg_bytes,
                                                 unsigned long long* payload, const IpcArgs& ip, uint32_t nwp) {
    const uint32_t q = threadIdx.x;
    unsigned long long pay = 0;
    const uint64_t seq = ip.peer_win ? *ip.seq : 0;
    if (q < parts) {
        const uint32_t n = cnt[q];
        const bool peer = q != self && seg_off[q + 1] > seg_off[q];  // segments with capacity only
        if (peer) {
            ulonglong2 h;
            if (ip.peer_win) {  // tile segment: records and rows
                const uint32_t nr = cnt[parts + q];
                h.x = (unsigned long long)nr | ((unsigned long long)n << 32);
                h.y = (unsigned long long)nr * kTileRec + (unsigned long long)n * 8ull * nwp;
                cnt[parts + q] = 0;
            } else {
                h.x = n;
                h.y = (unsigned long long)n * stride;
            }
            *reinterpret_cast<ulonglong2*>(ip.peer_win ? ipc_segment(ip, q, seq) : out + seg_off[q]) = h;
            pay = h.y;
            if (ip.peer_win) {  // the segment is complete at system scope: peer q may read it
                __threadfence_system();
                __hip_atomic_store(reinterpret_cast<uint64_t*>(ip.peer_win[q] + kWinReady) + self, seq + 1,
                                   __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        seg_bytes[q] = peer ? 16 + pay : 0ull;
        cnt[q] = 0;
    }
    pay = wave_sum(pay);
    if (threadIdx.x == 0) *payload = pay;
}

__global__ void finish_pack(uint32_t* cnt, uint8_t* out, const uint64_t* seg_off, uint32_t parts, uint32_t self,
                            uint32_t stride, unsigned long long* seg_bytes, unsigned long long* payload, IpcArgs ip,
                            uint32_t nwp) {
    if (ip.peer_win && ipc_failed(ip.err)) return;
    finish_pack_body(cnt, out, seg_off, parts, self, stride, seg_bytes, payload, ip, nwp);
}

// Sync rounds: ghosts that fired in r-1 run their callback in r+1 and read the
// sets of their out-peers; mark those owned nodes' send entries for the
// ghost's owner (gout_sidx: the send entry of each ghost -> owned edge).
__global__ void mark_set_needs(const uint64_t* fired_m1, const int64_t* gout_ptr, const uint32_t* gout_sidx,
                               uint64_t ghost0, uint64_t n_ghost, uint8_t* needmark) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_ghost || !bit_at(fired_m1, ghost0 + g)) return;
    for (int64_t e = gout_ptr[g]; e < gout_ptr[g + 1]; ++e) needmark[gout_sidx[e]] = 1;
}

struct UnpackArgs {
    uint64_t* F_cur;
    uint64_t* base;              // where kind S (a whole set) goes: the ghost's base row, or in batched
                                 // gossip with sync the set buffer of this round (read as bset_prev next round)
    uint8_t* flg_cur;
    uint32_t* stamp;             // [n_ghost] last round a ghost's F row arrived (by ghost row)
    const uint32_t* grow;        // [n_ghost] ghost row of the g-th ghost in exchange order, or nullptr (same)
    uint32_t* act_cur;           // spread act slots of round r ([kSlots])
    const uint8_t* in;
    const uint64_t* seg_off;     // [parts + 1] capacity offset of each source's segment
    const uint32_t* gfirst;      // [parts + 1] first ghost index from each source part
    uint32_t parts, self;
    uint64_t ghost0, n_ghost;
    uint32_t nwp, stride;
    uint32_t round;
    IpcArgs ipc;                 // device-driven exchange: `in` is this round's receive buffer
    uint32_t* stale_ticket;      // non-null: the last block clears the stale ghost rows (clear_stale_ghosts'
                                 // work; few ghosts, so no launch of its own)
    uint8_t* cand_mark;          // non-null (marking rounds): round r+1's candidate bytes; a ghost that sent
    const int64_t* gout_ptr;     // an F row marks its owned receivers (ghost -> owned CSR), round_prep's
    const uint32_t* gout_col;    // ghost pass moved here
};

// Every received entry into its ghost row (kind F: F row, flag ACT, stamp;
// kind S: the set into base).
__global__ __launch_bounds__(kBlock) void unpack_ghosts(UnpackArgs x) {
    __shared__ uint32_t s_src[64], s_pref[65];
    const uint32_t cpe = x.nwp >= 2 ? 1 + x.nwp / 2 : 1;
    if (x.ipc.peer_win && ipc_failed(x.ipc.err)) return;  // a dead exchange: nothing landed
    const uint64_t seq = x.ipc.peer_win ? *x.ipc.seq : 0;
    if (x.ipc.peer_win)  // this round's receive buffer
        x.in = reinterpret_cast<const uint8_t*>(x.ipc.my_win) + kWinHdr + (seq & 1) * x.ipc.rbuf;
    // (IPC: ipc_wait ran before — every source's segment of this round has landed)
    const bool tf = x.ipc.peer_win != nullptr;  // tile segments: s_pref counts records
    if (threadIdx.x == 0) {
        uint32_t tot = 0, m = 0;
        for (uint32_t p = 0; p < x.parts; ++p) {
            if (p == x.self || x.seg_off[p + 1] == x.seg_off[p]) continue;
            const uint32_t n = (uint32_t)*reinterpret_cast<const unsigned long long*>(x.in + x.seg_off[p]);
            s_src[m] = p;
            s_pref[m] = tot;
            tot += n;
            ++m;
        }
        s_pref[m] = tot;
        s_src[63] = m;
    }
    __syncthreads();
    const uint32_t m = s_src[63];
    uint32_t nact = 0;
    if (tf) {
        // one record (a send tile of 256 entries) per block iteration: item q of the
        // tile is entry j = q / cpr, chunk q % cpr of its rows (W = 64: the row word)
        const uint32_t cpr = x.nwp >= 2 ? x.nwp / 2 : 1, lcpr = __ffs(cpr) - 1;
        const uint64_t rowb = 8ull * x.nwp;
        __shared__ unsigned long long s_rb[9];  // k0 | first row << 32, F[4], S[4]
        for (uint32_t rr = blockIdx.x; rr < s_pref[m]; rr += gridDim.x) {
            uint32_t lo = 0, hi = m - 1;  // the source segment holding record rr
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (s_pref[mid] <= rr) lo = mid;
                else hi = mid - 1;
            }
            const uint32_t p = s_src[lo];
            const uint8_t* seg = x.in + x.seg_off[p];
            __syncthreads();  // s_rb reuse
            if (threadIdx.x < 9)
                s_rb[threadIdx.x] = *reinterpret_cast<const unsigned long long*>(
                    seg + 16 + (uint64_t)(rr - s_pref[lo]) * kTileRec + (threadIdx.x ? 8 + 8 * threadIdx.x : 0));
            __syncthreads();
            const uint32_t k0 = (uint32_t)s_rb[0], r0 = (uint32_t)(s_rb[0] >> 32);
            const uint8_t* rows = seg + tile_rows_off(x.gfirst[p + 1] - x.gfirst[p]);
            for (uint32_t q = threadIdx.x; q < ((uint32_t)kBlock << lcpr); q += kBlock) {
                const uint32_t j = q >> lcpr, ch = q & (cpr - 1), w = j >> 6;
                const unsigned long long bit = 1ull << (j & 63), below = bit - 1ull;
                const bool fb = (s_rb[1 + w] & bit) != 0, sb = (s_rb[5 + w] & bit) != 0;
                if (!fb && !sb) continue;
                uint32_t pos = r0 + __popcll(s_rb[1 + w] & below) + __popcll(s_rb[5 + w] & below);
                for (int ww = 0; ww < 4; ++ww)
                    if (ww < (int)w) pos += __popcll(s_rb[1 + ww]) + __popcll(s_rb[5 + ww]);
                const uint64_t g0 = x.gfirst[p] + k0 + j;
                const uint64_t g = x.grow ? x.grow[g0] : g0;  // locality-ordered shards: the ghost's row
                const uint64_t row = x.ghost0 + g;
                if (fb) {
                    const uint8_t* src = rows + (uint64_t)pos * rowb;
                    if (x.nwp == 1) x.F_cur[row] = *reinterpret_cast<const uint64_t*>(src);
                    else *reinterpret_cast<ulonglong2*>(x.F_cur + row * x.nwp + 2 * ch) =
                             *reinterpret_cast<const ulonglong2*>(src + 16 * ch);
                    if (ch == 0) {
                        x.flg_cur[row] = FL_ACT;
                        x.stamp[g] = x.round;
                        ++nact;
                        if (x.cand_mark)
                            for (int64_t qq = x.gout_ptr[g]; qq < x.gout_ptr[g + 1]; ++qq) x.cand_mark[x.gout_col[qq]] = CA_NODE;
                    }
                }
                if (sb) {
                    const uint8_t* src = rows + (uint64_t)(pos + (fb ? 1 : 0)) * rowb;
                    if (x.nwp == 1) x.base[row] = *reinterpret_cast<const uint64_t*>(src);
                    else *reinterpret_cast<ulonglong2*>(x.base + row * x.nwp + 2 * ch) =
                             *reinterpret_cast<const ulonglong2*>(src + 16 * ch);
                }
            }
        }
    }
    const uint64_t total = tf ? 0ull : (uint64_t)s_pref[m] * cpe;
    for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += (uint64_t)gridDim.x * kBlock) {
        const uint32_t j = (uint32_t)(e / cpe), ch = (uint32_t)(e % cpe);
        uint32_t lo = 0, hi = m - 1;  // the source segment holding entry j
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_pref[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t p = s_src[lo];
        const uint8_t* ent = x.in + x.seg_off[p] + 16 + (uint64_t)(j - s_pref[lo]) * x.stride;
        const uint32_t hd = *reinterpret_cast<const uint32_t*>(ent);
        const bool set = (hd & XK_SET) != 0;
        const uint64_t g0 = x.gfirst[p] + (hd & ~XK_SET);
        const uint64_t g = x.grow ? x.grow[g0] : g0;  // locality-ordered shards: the ghost's row
        const uint64_t row = x.ghost0 + g;
        if (ch == 0) {
            if (x.nwp == 1) {
                const uint64_t w = *reinterpret_cast<const uint64_t*>(ent + 8);
                if (set) x.base[row] = w;
                else x.F_cur[row] = w;
            }
            if (!set) {
                x.flg_cur[row] = FL_ACT;
                x.stamp[g] = x.round;
                ++nact;
                if (x.cand_mark)
                    for (int64_t q = x.gout_ptr[g]; q < x.gout_ptr[g + 1]; ++q) x.cand_mark[x.gout_col[q]] = CA_NODE;
            }
        } else {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(ent + 16 * ch);
            *reinterpret_cast<ulonglong2*>((set ? x.base : x.F_cur) + row * x.nwp + 2 * (ch - 1)) = v;
        }
    }
    const unsigned long long s = wave_sum(nact);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(x.act_cur + (blockIdx.x % kSlots), (uint32_t)s);
    if (x.stale_ticket) {  // the last block: ghosts whose F row of r-2 sits here and that sent none this round
        __shared__ uint32_t s_last;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            s_last = atomicAdd(x.stale_ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
            if (s_last) {
                *x.stale_ticket = 0;
                __threadfence();
            }
        }
        __syncthreads();
        if (s_last)
            for (uint64_t g = threadIdx.x; g < x.n_ghost; g += kBlock) {
                const uint64_t row = x.ghost0 + g;
                if (!(x.flg_cur[row] & FL_ACT) || x.stamp[g] == x.round) continue;
                for (uint32_t w = 0; w < x.nwp; ++w) x.F_cur[row * x.nwp + w] = 0;
                x.flg_cur[row] = 0;
            }
    }
    if (x.ipc.peer_win) {  // the last block to finish tells every source its buffer is free
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(x.ipc.ticket, 1u) == gridDim.x - 1) {
                *x.ipc.ticket = 0;
                for (uint64_t m = x.ipc.recv_mask; m; m &= m - 1) {
                    const int p = __ffsll((long long)m) - 1;
                    __hip_atomic_store(reinterpret_cast<uint64_t*>(x.ipc.peer_win[p] + kWinConsumed) + x.self,
                                       seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                *x.ipc.seq = seq + 1;  // every block of this launch has read seq
            }
        }
    }
}

// Ghosts whose F row of round r-2 sits in this round's buffer and that sent no
// F row this round: zero it (F rows are zero unless ACT) and clear the flag.
__global__ void clear_stale_ghosts(uint64_t* F_cur, uint8_t* flg_cur, const uint32_t* stamp, uint64_t ghost0,
                                   uint64_t n_ghost, uint32_t nwp, uint32_t round) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_ghost) return;
    const uint64_t row = ghost0 + g;
    if (!(flg_cur[row] & FL_ACT) || stamp[g] == round) return;
    for (uint32_t w = 0; w < nwp; ++w) F_cur[row * nwp + w] = 0;
    flg_cur[row] = 0;
}

}  // namespace gg
