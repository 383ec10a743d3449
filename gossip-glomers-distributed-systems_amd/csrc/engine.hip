// engine.hip — libgossip_hip.so: the C ABI of include/gossip.h on MI355X.
//
// Host side of the engine: input validation and CSR transposition
// (HandleTopology, `broadcast/broadcast.go:36-48`, for every node at once),
// message-value <-> lane bookkeeping (`BroadcastMsgBody.Message`, `:22-25`),
// the client broadcast queue, partition windows, device memory, and the
// per-round launch sequence of csrc/expand_kernels.hpp on one HIP stream.
//
// Device layout: node sets are rows of nwp u64 words (nwp =
// W/64 rounded up to a power of two), node-major: `base` (sets, updated in
// place), F[2] (new bits of a round = what the node forwards next round) and
// flags[2] (ACT: F row valid; LAG: set = base | F); fired[4] is a ring of
// per-round sync-timer bitmaps; CSR in-lists carry the sender's local row with
// bit 31 set when the sender is also in the receiver's out-list (forward
// exclusion, `:52`). Local rows: the owned nodes first, then (sharded mode,
// from ghost0 on) read-only ghost copies of the remote nodes adjacent to them,
// refreshed every round by the exchange (pack_ghosts / unpack_ghosts).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <iterator>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "expand_kernels.hpp"
#include "generate.h"
#include "gossip.h"
#include "gossip_gen.h"

namespace {

constexpr uint32_t kMaxBatch = 256;  // rounds per counter readback
constexpr int kMaxBlocks = 2048;

// Test hooks: environment variables the test suite sets to force a code path
// that the engine would otherwise choose by size (every forced path is
// bit-exact; only the kernels that run change): GG_HUB_DEG, GG_HUB_CHUNK,
// GG_SYNC_TILES, GG_SYNC_DIGEST, GG_ORDER, GG_XCHG_MODE, GG_PREP_BLOCKS,
// GG_SHARD_NATIVE (device-built shards keep native row order), GG_NO_DB (no
// double-buffered lean rounds: the F-row kernels take them), GG_DB (double-buffered
// lean rounds whatever the free memory), GG_SYNC_EAGER / GG_SYNC_ALLOC_ROUND (the
// streamed-sync buffers with the topology / from a given round), GG_COMPACT_ATOMIC /
// GG_COMPACT_SPLIT (one-launch or split compaction whatever the size),
// GG_IPC_SPIN_LIMIT (sleeps before a device-driven exchange wait gives up), GG_LSAT=0 / 1
// (lean saturation digest off / on whatever the graph), GG_NEED_BITS=0 (the device-driven
// exchange ships every active F row), GG_LSAT_LABELS_FAIL=1 (vertex parts: the component
// labels' build fails; the digest falls back to "every lane"), GG_IPC_OPEN_TIMEOUT_S (default 30 s),
// GG_IPC_WINDOW_ALIGN_MB (granularity of new IPC windows; win_round).
const char* test_knob(const char* name) { return getenv(name); }
// A/B switches of past measurements (GG_ALL_FULL, GG_NO_GRAPH, GG_SYNC_ALLPUSH,
// GG_FLAGS_FIRST, GG_FF_FRAC16, GG_PREP_WIDE, GG_XCHG_EXACT_BYTES): read only in a -DGG_AB_KNOBS build.
#ifdef GG_AB_KNOBS
const char* ab_knob(const char* name) { return getenv(name); }
#else
const char* ab_knob(const char*) { return nullptr; }
#endif

struct Window {
    int64_t from, to;
    bool seeded;
    uint64_t epoch_seed;
    std::vector<uint8_t> group;  // explicit: global node -> group
    bool edges = false;          // gg_set_partition: per-edge drops (overrides group windows)
    std::vector<uint64_t> ebits; // ... as a bitmap over this engine's local in-edges
    uint8_t* d_grp = nullptr;    // local-row groups on device (per-edge window: all zero)
    uint64_t* d_ebits = nullptr; // in-edge bitmap: ends in different groups (build_edge_mask),
                                 // or the per-edge window's bits
};

struct Injection {
    uint32_t node;
    uint32_t lane;
};

// Host loops over nodes on up to 16 threads (topology ingest of 10^8-node graphs).
template <class F>
void host_parallel(uint64_t n, F f) {
    unsigned hc = std::thread::hardware_concurrency();
    uint64_t T = std::min<uint64_t>(std::max(1u, std::min(hc, 16u)), std::max<uint64_t>(1, n / 65536));
    if (T <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < T; ++t) th.emplace_back(f, n * t / T, n * (t + 1) / T);
    for (auto& x : th) x.join();
}

uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Lanes per node group of the expand kernel for a row of nwp words
// (two 8-byte words per lane; see launch_expand).
uint32_t lanes_per_node(uint32_t nwp) { return nwp <= 2 ? 1u : nwp / 2; }

struct BatchKey {
    int64_t r0 = -1;
    uint32_t m = 0;
    uint64_t inj_hash = 0;
    uint64_t u_hash = 0;  // lanes_through of rounds r0-1 .. r0+m-1 (sync digest)
    size_t windows = 0;
    const void* inj_buf = nullptr;
    int db_state = 0;  // double-buffered rounds active at r0, and the current set buffer
    uint64_t solo_hash = 0;  // the solo schedule of the batch's marking rounds (and the round before r0)
    uint32_t zr = 0;         // rounds of counter slots zeroed before the batch (0: fold_slots left them zero)
    bool operator==(const BatchKey& o) const {
        return r0 == o.r0 && m == o.m && inj_hash == o.inj_hash && u_hash == o.u_hash && windows == o.windows &&
               inj_buf == o.inj_buf && db_state == o.db_state && solo_hash == o.solo_hash && zr == o.zr;
    }
};



}  // namespace

// message value -> lane: open addressing over 2x the lane count; clear() is
// O(1) (an epoch bump), so reset + re-inject of a benchmark episode costs no
// allocation.
struct LaneTable {
    std::vector<int64_t> key;
    std::vector<uint32_t> val, epoch_of;
    uint32_t epoch = 1;
    uint64_t mask = 0;
    void init(uint64_t lanes) {
        uint64_t cap = 16;
        while (cap < 2 * lanes) cap <<= 1;
        key.assign(cap, 0);
        val.assign(cap, 0);
        epoch_of.assign(cap, 0);
        mask = cap - 1;
        epoch = 1;
    }
    uint64_t slot(int64_t k) const {
        uint64_t h = gg_mix64((uint64_t)k) & mask;
        while (epoch_of[h] == epoch && key[h] != k) h = (h + 1) & mask;
        return h;
    }
    uint32_t find(int64_t k) const {  // ~0u: absent
        if (!mask) return ~0u;
        const uint64_t h = slot(k);
        return epoch_of[h] == epoch ? val[h] : ~0u;
    }
    void insert(int64_t k, uint32_t v) {  // k absent; at most `lanes` keys live
        const uint64_t h = slot(k);
        key[h] = k;
        val[h] = v;
        epoch_of[h] = epoch;
    }
    void clear() {
        if (++epoch == 0) {
            std::fill(epoch_of.begin(), epoch_of.end(), 0u);
            epoch = 1;
        }
    }
};

struct gg_engine {
    gg_config cfg{};
    std::string err;
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t V = 0, nw = 0, nwp = 0;
    uint32_t rank = 0, world = 1;
    // 2-D sharding: world = L lane groups x P vertex parts; this engine holds lane
    // words [w0, w0 + nw) of nw_g (its lane group lgrp) for the nodes of part `part`
    uint32_t L = 1, P = 1, lgrp = 0, part = 0;
    uint64_t nw_g = 0, w0 = 0;
    uint32_t peer_rank(uint32_t q) const { return lgrp * P + q; }
    uint64_t n_own = 0, ghost0 = 0, n_ghost = 0, rows = 0;  // local rows: own, then ghosts
    std::vector<uint32_t> gid;     // [rows] original id of each local row (~0u: padding)
    std::vector<uint32_t> loc_of;  // [V] local row of an owned node, ~0u otherwise (sharded)
    bool range_mode = false;       // device-partitioned shard: owned nodes [range_lo, range_hi)
    uint64_t range_lo = 0, range_hi = 0;  // are rows 0.. (no loc_of), or own_row[node - range_lo]
    std::vector<uint32_t> own_row; // [n_own] range shard in locality order: row of node range_lo + i
    uint32_t* d_grow = nullptr;    // [n_ghost] range shard in locality order: ghost row of the g-th ghost
                                   // in exchange order (ascending id)
    bool have_topo = false, symmetric = true;
    bool part_rows = false;        // built from a caller's own rows (gg_topology_part*): per-edge window
                                   // bits are over those rows
    std::vector<int64_t> host_rp;  // vertex-sharded: the caller's row offsets (gg_set_partition)
    uint32_t* d_gid = nullptr;     // sharded only (single engine: row == id)
    // exchange: owned rows each rank needs (concatenated per destination) and
    // ghost counts per source rank; outgoing ghost edges (ghost -> owned receivers)
    std::vector<uint64_t> send_off, recv_off;  // [world+1] node counts
    uint32_t* d_send_idx = nullptr;
    int64_t* d_gout_ptr = nullptr;
    uint32_t* d_gout_col = nullptr;
    uint8_t* d_xsend = nullptr;
    uint8_t* d_xrecv = nullptr;
    // filtered exchange (expand_kernels.hpp pack_ghosts): per-part segment
    // capacity offsets (bytes, [P+1]), pack tiles, per-gout-edge send entry,
    // set-need marks, per-ghost F arrival stamps, per-peer counters and sizes
    std::vector<uint64_t> xsoff, xroff;
    uint64_t* d_xsoff = nullptr;
    uint64_t* d_xroff = nullptr;
    uint32_t* d_gfirst = nullptr;
    gg::XchgTile* d_xtiles = nullptr;
    uint32_t n_xtiles = 0;
    uint32_t* d_gout_sidx = nullptr;
    uint8_t* d_needmark = nullptr;
    uint32_t* d_stamp = nullptr;
    uint32_t* d_xcnt = nullptr;
    uint32_t* d_sfirst = nullptr;        // [P+1] first send entry of each peer (tile segments)
    uint32_t* d_xtk = nullptr;           // [4] last-block tickets: pack_ghosts (finish), unpack_ghosts (stale clear)
    unsigned long long* d_segbytes = nullptr;  // [2P]: bytes to each part, bytes from each part
    unsigned long long* h_segbytes = nullptr;  // pinned copy
    unsigned long long* d_payload = nullptr;   // [kMaxBatch] payload bytes of each pending round
    uint32_t xstride = 16;
    // need bits (device-driven exchange): per source part, where its
    // need slots sit in this engine's receive region and their size, and for each
    // destination where ours sit in its window; which peers produce them
    uint64_t* d_need_in = nullptr;             // [P] window offset of source q's need slot 0 (receiver side)
    uint64_t* d_need_out = nullptr;            // [P] offset of our need slot 0 in part q's receive region
    uint64_t* d_need_bytes = nullptr;          // [2P] need slot bytes: [q] we write to q, [P + q] q writes to us
    gg::NeedWord* d_need_words = nullptr;      // the words our need_bits kernel writes (per source, 64 ghosts)
    uint32_t n_need_words = 0;
    uint64_t need_peers = 0;                   // parts whose need bits we may use (they hold the digest)
    std::set<int64_t> inj_rounds;              // rounds with a client broadcast (the need bits' condition)
    bool need_produce = false;                 // we write need bits (we hold the digest)
    // exact-size directions (their sizes travel first, one host wait per round),
    // decided per direction from its capacity, which both ends compute alike
    std::vector<uint8_t> xexact_s, xexact_r;   // [P] to / from each part
    bool xexact = false;                       // any exact direction
    std::vector<uint64_t> xsend_bytes, xrecv_bytes, xsend_off, xrecv_off;  // [world]
    uint32_t dist_k = 0;                       // pending rounds (counter slots in use)
    uint32_t ctr_dirty = kMaxBatch;            // counter slots [0, ctr_dirty) may be non-zero
    uint32_t batch_zr = 0;                     // enqueue_step_batch: rounds of slots it zeroes first (BatchKey::zr)
    std::vector<int64_t> dist_round_of;        // round of each pending slot
    std::vector<uint64_t> dist_path;           // its kernel path (GG_PATH_*)
    uint64_t last_path = 0;                    // path of the round enqueue_round enqueued last
    // solo marking rounds (RoundArgs::solo): per round, the busy flag the stream
    // kernels reported the last time it ran (-1: not seen), with a strike count
    // (a hint flips after two runs in a row that disagree with it), and the solo
    // kind of the last enqueued round
    std::vector<int8_t> busy_hint, busy_strike;
    uint32_t last_solo = 0;
    bool last_mark = false;                    // ... and whether it marks round r+1's candidates (mark_cand):
                                               // then the unpack of its exchange marks the owned receivers of
                                               // the ghosts that sent an F row (round r+1 runs no round_prep)
    std::vector<uint64_t> dist_sent;           // payload bytes sent in each pending slot
    std::vector<gg_round_stats> dist_done;     // folded, not yet flushed
    size_t inj_off = 0;                        // pinned injection ring offset (async rounds)
    uint32_t quiet = 0;                        // trailing rounds without new bits (gg_step)
    int dirty_parity = 0;                      // gg_reset: parity of the round before the last one

    int64_t* d_in_ptr = nullptr;
    uint32_t* d_in_col = nullptr;
    int64_t* d_out_ptr = nullptr;
    uint32_t* d_out_col = nullptr;
    uint64_t* d_base = nullptr;      // the buffer holding the current sets (d_sets[set_cur])
    // double-buffered lean rounds (db_ok engines): round r reads the
    // sets of r-1 from d_sets[(r+1)&1] and writes d_sets[r&1]; F rows are not written
    // until the first round that needs them (materialize_F), and from then on the
    // episode updates d_sets[set_cur] in place
    uint64_t* d_sets[2] = {nullptr, nullptr};  // d_sets[0] is d_base's allocation
    bool db_ok = false;       // single engine, no hubs, W >= 128, not batched, both buffers fit
    bool db_active = false;   // every round of this episode so far was double-buffered
    int set_cur = 0;
    bool f_dirty = true;      // some F row may be non-zero (reset must clear them)
    bool db_decided = false;  // ensure_db ran since the topology was installed
    bool sync_alloc = false;  // alloc_sync ran since the topology was installed
    bool no_mark = false;     // GG_NO_MARK=1 at the install: no marking rounds (round_prep every round)
    uint64_t* d_F[2] = {nullptr, nullptr};
    uint8_t* d_flg[2] = {nullptr, nullptr};
    uint8_t* d_cand = nullptr;       // [2][rows] candidate bytes by round parity
    uint8_t* d_zmark = nullptr;      // [rows] stale-F-row marks
    uint8_t* d_tile_cand = nullptr;  // [tile_bytes]
    gg::TileWork* d_work = nullptr;  // [tiles] live-tile worklist (sparse sync/mask rounds)
    uint32_t* d_n_work = nullptr;    // [2][2] live tiles, candidate nodes, by round parity
    uint32_t* d_bcount = nullptr;    // [compact blocks + 1] split compaction (large graphs)
    uint64_t prep_cap = 1024;        // round_prep's grid cap in rounds without timers (GG_PREP_BLOCKS)
    uint32_t* d_nodes = nullptr;     // [n_own] candidate-node list (sparse lean rounds)
    uint32_t* d_act = nullptr;       // [4] ring: nodes that became active per round
    unsigned long long* d_act_deg = nullptr;  // [4] ring: their out-degree sums
    unsigned long long* d_tot = nullptr;      // [4] ring: new bits of the owned nodes in rounds <= r
    uint32_t* d_act_s = nullptr;              // [4][64] the three rings' per-round increments, spread
    unsigned long long* d_act_deg_s = nullptr;
    unsigned long long* d_tot_s = nullptr;
    uint64_t* d_abits = nullptr;     // [rows/64] ACT bits of the previous round (flags-first rounds)
    bool ff_ok = false;              // flags-first gathers allowed
    uint32_t ff_frac16 = 8;          // ... in rounds where < ff_frac16/16 of the in-edges carry data
    // hubs (see expand_kernels.hpp): in-edge chunks of high in-degree nodes,
    // out-edge chunks of high out-degree senders, per-chunk partial rows
    uint32_t hub_deg = 0;
    uint64_t n_hubs = 0, n_hchunks = 0, n_mchunks = 0;
    uint32_t* d_hubs = nullptr;
    uint32_t* d_hub_c0 = nullptr;
    gg::HubChunk* d_hchunks = nullptr;
    gg::HubChunk* d_mchunks = nullptr;
    uint4* d_srec = nullptr;         // [2 n_own] sync records (streamed sync rounds), or none
    uint8_t* d_pushb = nullptr;      // [out-edges] non-empty sync pushes of the last callbacks
    uint32_t* d_rev = nullptr;       // [in-edges] sender's out-edge index (streamed sync rounds)
    uint64_t n_out_edges = 0;
    uint8_t* d_sstate = nullptr;     // [rows] sender states (streamed sync rounds)
    uint64_t* d_ibits = nullptr;     // [rows/64] non-zero sender states
    uint64_t* d_sat = nullptr;       // [rows/64] saturation digest (streamed sync rounds)
    uint64_t* d_pend = nullptr;      // batched gossip: [rows][nwp] pending values
    uint32_t* d_pend_src = nullptr;  // batched gossip: [rows] who delivered them
    uint64_t* d_bset[2] = {nullptr, nullptr};  // batched gossip with sync: sets after odd / even rounds
    uint8_t* d_pushany = nullptr;    // [rows] a streamed callback pushed to some peer
    uint2* d_nmeta = nullptr;        // [n_own] node list with the nodes' bytes (streamed sync rounds)
    uint64_t* d_sat_new = nullptr;   // [rows/64] its bits found in the current round
    uint8_t* d_lsat = nullptr;       // [rows] lean-round saturation digest (RoundArgs::lsat)
    uint32_t* d_llab = nullptr;      // [n_own] component labels of the owned rows (several components)
    uint32_t* d_lreach = nullptr;    // [rows] per owned row: lanes broadcast into its component
    uint32_t* d_ltab = nullptr;      // [1 + 2 ltab_cap] (label, count) table behind d_lreach
    uint32_t ltab_cap = 0;
    uint64_t ltab_hash = 0;          // the table d_lreach was filled from (0: none yet)
    std::vector<uint32_t> h_ltab;    // its host copy (the source of the last upload)
    hipEvent_t ltab_ev = nullptr;    // recorded after that upload: h_ltab is reused only past it
    bool ltab_ev_live = false;
    std::vector<uint32_t> h_lab;     // labels on the host: by local row (single engine) or by node id
    bool lab_global = false;         // (vertex parts: labels of the whole graph)
    std::vector<uint64_t> lret;      // label << 32 | lane of the retired rounds' broadcasts (lane in range; sorted, unique)
    std::vector<uint32_t> u_hist;    // u_hist[r]: lanes of this engine injected in rounds <= r
    std::vector<uint64_t> u_bits;    // those lanes (nw words)
    bool sync_tiles = false;         // GG_SYNC_TILES=1: sync rounds on the tile path (A/B)
    uint64_t* d_hscratch = nullptr;
    uint32_t* d_hflag = nullptr;     // [hub chunks] streamed sync rounds with hubs
    uint8_t* d_hlive = nullptr;      // [hubs] streamed sync rounds with hubs
    uint64_t tile_nodes = 0, tile_bytes = 0;
    uint64_t n_in_edges = 0;
    uint64_t* d_fired[4] = {nullptr, nullptr, nullptr, nullptr};
    int32_t* d_sync_next = nullptr;
    uint32_t* d_sync_k = nullptr;
    int32_t* d_dr = nullptr;
    unsigned long long* d_counters = nullptr;
    unsigned long long* h_counters = nullptr;  // pinned
    unsigned long long* d_ep = nullptr;  // gg_run_episodes: each episode's folded counter rows
    unsigned long long* h_ep = nullptr;  // pinned
    size_t ep_cap = 0;                   // bytes of each
    uint32_t* d_inj = nullptr;
    uint32_t* h_inj = nullptr;  // pinned
    uint32_t* d_injtab = nullptr;  // [kMaxBatch + 1] first pair of each round of a batch (gg_step)
    uint32_t* h_injtab = nullptr;  // pinned
    uint64_t injtab_dev_hash = ~0ull;
    size_t inj_cap = 0;         // pairs
    std::vector<hipEvent_t> ev;  // 2 per batched round
    hipEvent_t inj_ev = nullptr;   // after the last copy out of h_inj (gg_step reuses h_inj)
    bool inj_ev_live = false;
    uint64_t inj_dev_hash = 0;   // run_batch: hash of the pairs d_inj holds from its last upload (0: unknown)

    std::vector<Window> windows;
    LaneTable lanes;                 // message value -> lane
    std::vector<int64_t> lane_value;
    std::map<int64_t, std::vector<Injection>> inj;
    int64_t round = 0;
    unsigned long long pend_acks = 0, pend_ackdrop = 0;
    unsigned long long hash_total = 0;
    bool dist_open = false;
    hipGraphExec_t graph_exec = nullptr;  // launch cache (run_batch)
    double step_event_ms = 0.0;           // HIP-event time of the last gg_step (device)
    BatchKey graph_key;
    bool graph_broken = false;
    hipGraphExec_t dist_exec = nullptr;   // gg_dist_step's captured batch of sharded rounds (IPC / no exchange)
    BatchKey dist_key;
    uint32_t dist_key_k0 = 0;             // ... and the counter slot it starts at

    // device-driven exchange over IPC-mapped peer windows (gg_dist_ipc_*)
    bool ipc = false;
    uint8_t* d_win = nullptr;            // this engine's window (uncached): flags, 2 receive buffers
    uint64_t win_rbuf = 0;               // receive buffer bytes (xroff[P] rounded up)
    std::vector<void*> peer_map;         // [P] opened peer windows
    uint8_t** d_peer_win = nullptr;      // [P] the same on the device
    uint64_t* d_peer_off = nullptr;      // [P] this engine's segment offset in peer q's receive buffer
    uint64_t* d_peer_rbuf = nullptr;     // [P] peer q's receive buffer bytes
    uint64_t send_mask = 0, recv_mask = 0;
    uint32_t* d_xticket = nullptr;       // [4] unpack's last-block counter, error word, exchange sequence
                                         // number (u64: one per sharded round, never reset; on the device)
    ncclComm_t comm = nullptr;  // engine-owned RCCL communicator over the lane group's parts
    gg_transport xport{};       // or the caller's transport (gg_dist_transport_init)
    bool have_xport = false;

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    void free_topology();
    ~gg_engine();
};

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t err_ = (x);                                                             \
        if (err_ != hipSuccess)                                                            \
            return e->fail(GG_EIO, std::string(#x) + ": " + hipGetErrorString(err_));      \
    } while (0)

template <class T>
static void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

namespace {
void win_release(uint8_t* p);  // the IPC window pool (below, gg_dist_ipc_export)
}

void gg_engine::free_topology() {
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    graph_exec = nullptr;
    if (dist_exec) (void)hipGraphExecDestroy(dist_exec);
    dist_exec = nullptr;
    if (d_out_col == d_in_col) d_out_col = nullptr;
    if (d_out_ptr == d_in_ptr) d_out_ptr = nullptr;
    dfree(d_out_col);
    dfree(d_out_ptr);
    dfree(d_in_ptr);
    dfree(d_in_col);
    // d_base points at one of the two set buffers (d_sets[set_cur]): free the
    // allocations, not the alias (a double free left a sticky hipErrorInvalidValue)
    if (!d_sets[0]) d_sets[0] = d_base;
    dfree(d_sets[1]);
    dfree(d_sets[0]);
    d_base = nullptr;
    set_cur = 0;
    db_ok = false;
    for (auto& p : d_F) dfree(p);
    for (auto& p : d_flg) dfree(p);
    dfree(d_cand);
    dfree(d_zmark);
    dfree(d_tile_cand);
    dfree(d_hubs);
    dfree(d_hub_c0);
    dfree(d_hchunks);
    dfree(d_mchunks);
    dfree(d_srec);
    dfree(d_pushb);
    dfree(d_rev);
    dfree(d_sstate);
    dfree(d_ibits);
    dfree(d_sat);
    dfree(d_sat_new);
    dfree(d_lsat);
    dfree(d_llab);
    dfree(d_lreach);
    dfree(d_ltab);
    dfree(d_pushany);
    dfree(d_nmeta);
    dfree(d_pend);
    dfree(d_pend_src);
    dfree(d_bset[0]);
    dfree(d_bset[1]);
    dfree(d_hscratch);
    dfree(d_hflag);
    dfree(d_hlive);
    n_hubs = n_hchunks = n_mchunks = 0;
    dfree(d_work);
    dfree(d_n_work);
    dfree(d_bcount);
    dfree(d_nodes);
    dfree(d_act);
    dfree(d_act_deg);
    dfree(d_tot);
    dfree(d_act_s);
    dfree(d_act_deg_s);
    dfree(d_tot_s);
    dfree(d_abits);
    for (auto& p : d_fired) dfree(p);
    dfree(d_sync_next);
    dfree(d_sync_k);
    dfree(d_dr);
    dfree(d_gid);
    dfree(d_grow);
    own_row.clear();
    dfree(d_send_idx);
    dfree(d_gout_ptr);
    dfree(d_gout_col);
    dfree(d_xsend);
    dfree(d_xrecv);
    dfree(d_xsoff);
    dfree(d_xroff);
    dfree(d_gfirst);
    dfree(d_xtiles);
    dfree(d_gout_sidx);
    dfree(d_needmark);
    dfree(d_stamp);
    dfree(d_xcnt);
    dfree(d_sfirst);
    dfree(d_xtk);
    dfree(d_need_in);
    dfree(d_need_out);
    dfree(d_need_bytes);
    dfree(d_need_words);
    n_need_words = 0;
    need_peers = 0;
    need_produce = false;
    dfree(d_segbytes);
    dfree(d_payload);
    peer_map.clear();  // mappings: the process's cache keeps them (see win_acquire)
    dfree(d_peer_win);
    dfree(d_peer_off);
    dfree(d_peer_rbuf);
    dfree(d_xticket);
    if (d_win) win_release(d_win);  // back to the pool, not freed (see win_acquire)
    d_win = nullptr;
    ipc = false;
    if (h_segbytes) (void)hipHostFree(h_segbytes);
    h_segbytes = nullptr;
    n_xtiles = 0;
    for (auto& w : windows) {
        dfree(w.d_grp);
        dfree(w.d_ebits);
    }
    have_topo = false;
    part_rows = false;
    busy_hint.clear();
    busy_strike.clear();
}

static void rccl_destroy(ncclComm_t c);

gg_engine::~gg_engine() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (comm) rccl_destroy(comm);
    comm = nullptr;
    free_topology();
    dfree(d_counters);
    dfree(d_inj);
    if (h_counters) (void)hipHostFree(h_counters);
    dfree(d_ep);
    if (h_ep) (void)hipHostFree(h_ep);
    if (h_inj) (void)hipHostFree(h_inj);
    if (h_injtab) (void)hipHostFree(h_injtab);
    dfree(d_injtab);
    for (auto& x : ev) (void)hipEventDestroy(x);
    if (inj_ev) (void)hipEventDestroy(inj_ev);
    if (ltab_ev) (void)hipEventDestroy(ltab_ev);
    if (stream) (void)hipStreamDestroy(stream);
}

// ---------------------------------------------------------------------------

namespace {

int zero_async(gg_engine* e, void* p, size_t bytes);

// Back to round 0, asynchronously: every call that reads results waits on the stream.
int reset_device_state(gg_engine* e) {
    const size_t rowbytes = e->rows * e->nwp * 8;
    // one launch clears every per-episode array (sizes are multiples of 8
    // bytes: rows is a multiple of 64) and starts the sync timers
    gg::ResetArgs ra{};
    auto seg = [&](void* p, uint64_t bytes, uint64_t val) {
        if (ra.n_seg < gg::kResetSegs) ra.seg[ra.n_seg++] = {reinterpret_cast<uint64_t*>(p), bytes / 8, val};
        else e->err = "internal: reset segment table full";  // caught below
    };
    e->set_cur = 0;
    e->d_base = e->d_sets[0];
    e->db_active = e->db_ok;
    seg(e->d_sets[0], rowbytes, 0);
    if (e->db_ok) seg(e->d_sets[1], rowbytes, 0);
    // F rows and flags are already all zero after two rounds without new bits
    // (a stale row is cleared in the round it expires), e.g. after an episode
    // run to quiescence. Single engine only: ghost rows follow remote rounds.
    // After exactly one quiet round r only the buffers of round r-1 (parity
    // dirty_parity = (r+1) & 1, recorded by gg_reset) can hold non-zero rows,
    // and only where their flag byte is set: those rows and the flags are
    // cleared (a sparse last delivery round: 1 MB read instead of C2's 134 MB
    // F buffer written; batched engines keep whole-buffer clears).
    if (e->db_ok && !e->f_dirty) {  // only double-buffered rounds ran: F rows are all zero
        for (int b = 0; b < 2; ++b) seg(e->d_flg[b], e->rows, 0);
    } else if (e->P == 1 && e->quiet == 1 && !e->d_pend && e->nwp >= 2 && e->nwp <= 128 && !(e->nwp & (e->nwp - 1))) {
        ra.sparse_F = e->d_F[e->dirty_parity];
        ra.sparse_flg = e->d_flg[e->dirty_parity];
        ra.sparse_rows = e->rows;
        ra.nwp = (uint32_t)e->nwp;
    } else if (!(e->P == 1 && e->quiet >= 2)) {
        for (int b = 0; b < 2; ++b) {
            if (e->P == 1 && e->quiet == 1 && b != e->dirty_parity) continue;
            seg(e->d_F[b], rowbytes, 0);  // F rows are zero unless ACT
            seg(e->d_flg[b], e->rows, 0);
        }
    }
    e->quiet = 2;
    e->f_dirty = !e->db_ok || e->P > 1;  // (sharded: the exchange writes the ghosts' F rows)
    for (int b = 0; b < 4; ++b) seg(e->d_fired[b], e->rows / 8, 0);
    seg(e->d_cand, 2 * e->rows, 0);
    seg(e->d_n_work, 16, 0);
    seg(e->d_zmark, e->rows, 0);
    seg(e->d_tile_cand, e->tile_bytes, 0);
    seg(e->d_act, 16, 0);
    seg(e->d_act_deg, 32, 0);
    seg(e->d_tot, 32, 0);
    seg(e->d_act_s, 4 * gg::kSlots * 4, 0);
    seg(e->d_act_deg_s, 4 * gg::kSlots * 8, 0);
    seg(e->d_tot_s, 4 * gg::kSlots * 8, 0);
    if (e->d_sat) {
        seg(e->d_sat, e->rows / 8, 0);
        seg(e->d_sat_new, e->rows / 8, 0);
    }
    if (e->d_lsat) seg(e->d_lsat, e->rows, 0);
    if (e->d_hlive) seg(e->d_hlive, (e->n_hubs + 7) / 8 * 8, 0);
    if (e->d_pend) {
        seg(e->d_pend, e->rows * e->nwp * 8, 0);
        seg(e->d_pend_src, e->rows * 4, ~0ull);
    }
    const uint64_t n_own = e->n_own;
    if (e->d_dr) seg(e->d_dr, n_own * e->nw * 64 * 4, ~0ull);
    if (e->d_stamp) seg(e->d_stamp, (e->n_ghost + 1) / 2 * 8, ~0ull);
    if (e->d_needmark) seg(e->d_needmark, (e->send_off[e->P] + 7) / 8 * 8, 0);
    if (e->d_xcnt) seg(e->d_xcnt, (2 * e->P * 4 + 7) / 8 * 8, 0);
    ra.sync_next = e->d_sync_next;
    ra.sync_k = e->d_sync_k;
    ra.n_own = n_own;
    ra.ghost0 = e->ghost0;
    ra.n_ghost = e->n_ghost;
    ra.gid = e->d_gid;
    ra.seed = e->cfg.seed;
    ra.sync_base = e->cfg.sync_base_ticks;
    ra.sync_jitter = e->cfg.sync_jitter_ticks;
    ra.sync_mix = gg_mix64(e->cfg.seed ^ GG_TAG_SYNC);
    ra.sync_rcp = gg_sync_rcp(e->cfg.sync_jitter_ticks);
    if (e->err == "internal: reset segment table full") return GG_EIO;
    const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>(1, rowbytes / 16384), 4096);
    hipLaunchKernelGGL(gg::reset_state, dim3((unsigned)blocks), dim3(gg::kBlock), 0, e->stream, ra);
    HIPCHK(hipGetLastError());
    return GG_OK;
}

int materialize_windows(gg_engine* e) {
    bool any = false;
    for (auto& w : e->windows) {
        if (w.d_grp) continue;
        any = true;
        HIPCHK(hipMalloc(&w.d_grp, e->rows));
        if (w.edges) {  // the kernels take the bits; the groups only mark the window active
            HIPCHK(hipMemset(w.d_grp, 0, e->rows));
            HIPCHK(hipMalloc(&w.d_ebits, std::max<size_t>(1, w.ebits.size()) * 8));
            if (!w.ebits.empty())
                HIPCHK(hipMemcpy(w.d_ebits, w.ebits.data(), w.ebits.size() * 8, hipMemcpyHostToDevice));
            continue;
        }
        if (w.seeded) {
            const uint64_t valid = e->d_gid ? e->rows : e->n_own;
            hipLaunchKernelGGL(gg::fill_seeded_groups, dim3((unsigned)((e->rows + 255) / 256)), dim3(256), 0,
                               e->stream, w.d_grp, e->rows, valid, e->d_gid, e->cfg.seed, w.epoch_seed);
            HIPCHK(hipGetLastError());
        } else {
            std::vector<uint8_t> h(e->rows, 0);
            for (uint64_t r = 0; r < e->rows; ++r) {
                const uint64_t g = e->gid.empty() ? r : e->gid[r];
                if (g < e->V) h[r] = w.group[g];
            }
            HIPCHK(hipMemcpy(w.d_grp, h.data(), e->rows, hipMemcpyHostToDevice));
        }
        const uint64_t words = std::max<uint64_t>(1, (e->n_in_edges + 63) / 64);
        HIPCHK(hipMalloc(&w.d_ebits, words * 8));
        if (e->n_in_edges) {
            hipLaunchKernelGGL(gg::build_edge_mask, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, e->stream,
                               e->d_in_ptr, e->d_in_col, e->n_own, e->n_in_edges, w.d_grp, w.d_ebits);
            HIPCHK(hipGetLastError());
        }
    }
    if (any) HIPCHK(hipStreamSynchronize(e->stream));
    return GG_OK;
}

const Window* window_at(const gg_engine* e, int64_t r) {
    for (const auto& w : e->windows)  // a per-edge window overrides a group window
        if (w.edges && w.from <= r && r < w.to) return &w;
    for (const auto& w : e->windows)
        if (w.from <= r && r < w.to) return &w;
    return nullptr;
}

template <int G, int WPL>
void launch_t(const gg::RoundArgs& a, bool syncw, bool maskw, hipStream_t s) {
    const uint64_t groups = gg::kBlock / G;
    uint64_t blocks = (a.n_own + groups - 1) / groups;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, kMaxBlocks));
    dim3 grid((unsigned)blocks), block(gg::kBlock);
    if (syncw) {
        if (maskw) hipLaunchKernelGGL((gg::expand_round<G, WPL, true, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((gg::expand_round<G, WPL, true, false>), grid, block, 0, s, a);
    } else {
        if (maskw) hipLaunchKernelGGL((gg::expand_round<G, WPL, false, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((gg::expand_round_lean<G, WPL>), grid, block, 0, s, a);
    }
}

void launch_expand(const gg::RoundArgs& a, bool syncw, bool maskw, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_t<1, 1>(a, syncw, maskw, s); break;
        case 2: launch_t<1, 2>(a, syncw, maskw, s); break;
        case 4: launch_t<2, 2>(a, syncw, maskw, s); break;
        case 8: launch_t<4, 2>(a, syncw, maskw, s); break;
        case 16: launch_t<8, 2>(a, syncw, maskw, s); break;
        case 32: launch_t<16, 2>(a, syncw, maskw, s); break;
        case 64: launch_t<32, 2>(a, syncw, maskw, s); break;
        case 128: launch_t<64, 2>(a, syncw, maskw, s); break;
        default: break;
    }
}

// expand_stream grid: one resident wave of blocks (node groups walk their
// items grid-stride), so no partial second wave of blocks trails the round.
template <int G, bool MASKW, int DB = 0>
void launch_stream_t(const gg::RoundArgs& a, hipStream_t s) {
    static int resident = 0;
    auto kern = MASKW ? gg::expand_stream_masked<G, 2>
                      : (DB == 3 ? gg::expand_stream_db<G, 2, 3>
                                 : (DB == 2 ? gg::expand_stream_db_mark<G, 2>
                                            : (DB ? gg::expand_stream_db<G, 2> : gg::expand_stream<G, 2>)));
    if (!resident) {
        int dev = 0, cus = 0, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, gg::kBlock, 0);
        resident = std::max(1, cus) * std::max(1, per_cu);
    }
    const uint64_t ngb = gg::kBlock / G;
    uint64_t blocks = (a.n_own + ngb - 1) / ngb;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)resident));
    // block lists: a block's 256 granules of 16 nodes cover its share of the nodes
    if (DB && a.block_lists) blocks = std::max<uint64_t>(blocks, (a.n_own + gg::kBllMax - 1) / gg::kBllMax);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(gg::kBlock), 0, s, a);
}

template <int G>
void launch_stream_m(const gg::RoundArgs& a, bool maskw, hipStream_t s) {
    if (maskw) {
        launch_stream_t<G, true>(a, s);
    } else if (a.db) {
        // the marking kernel first: in rounds with block lists it sums round r-1's
        // rings and publishes them for the other one
        // (solo marking rounds: only the kernel the last run of this round needed)
        if (a.mark_cand && a.solo != gg::SOLO_DB) launch_stream_t<G, false, 2>(a, s);  // the rounds that are not busy
        if (a.solo == gg::SOLO_MARK) return;
        if (a.n_edges < 4ull * a.n_own) launch_stream_t<G, false, 3>(a, s);  // mean in-degree < 4: 3 rows a batch
        else launch_stream_t<G, false, 1>(a, s);
    } else {
        launch_stream_t<G, false>(a, s);
    }
}

template <int G, int WPL = 2>
void launch_hubs_t(const gg::RoundArgs& a, hipStream_t s) {
    const unsigned bc = (unsigned)std::min<uint64_t>(a.n_hchunks, 8192);
    const unsigned bh = (unsigned)std::min<uint64_t>(a.n_hubs, 8192);
    hipLaunchKernelGGL((gg::hub_chunks<G, WPL>), dim3(bc), dim3(gg::kBlock), 0, s, a);
    hipLaunchKernelGGL((gg::hub_finish<G, WPL>), dim3(bh), dim3(gg::kBlock), 0, s, a);
}

// Streamed sync rounds with hubs (symmetric topologies): hub_sync_chunks,
// hub_sync_finish, hub_sync_push (expand_kernels.hpp), after expand_stream_sync.
template <int G, int WPL = 2>
void launch_hub_sync_t(const gg::RoundArgs& a, hipStream_t s) {
    const unsigned bc = (unsigned)std::min<uint64_t>(a.n_hchunks, 8192);
    const unsigned bh = (unsigned)std::min<uint64_t>(a.n_hubs, 8192);
    hipLaunchKernelGGL((gg::hub_sync_chunks<G, WPL>), dim3(bc), dim3(gg::kBlock), 0, s, a);
    hipLaunchKernelGGL((gg::hub_sync_finish<G, WPL>), dim3(bh), dim3(gg::kBlock), 0, s, a);
    hipLaunchKernelGGL((gg::hub_sync_push<G, WPL>), dim3(bc), dim3(gg::kBlock), 0, s, a);
}

void launch_hub_sync(const gg::RoundArgs& a, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_hub_sync_t<1, 1>(a, s); break;
        case 2: launch_hub_sync_t<1>(a, s); break;
        case 4: launch_hub_sync_t<2>(a, s); break;
        case 8: launch_hub_sync_t<4>(a, s); break;
        case 16: launch_hub_sync_t<8>(a, s); break;
        case 32: launch_hub_sync_t<16>(a, s); break;
        case 64: launch_hub_sync_t<32>(a, s); break;
        case 128: launch_hub_sync_t<64>(a, s); break;
        default: break;
    }
}

void launch_hubs(const gg::RoundArgs& a, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_hubs_t<1, 1>(a, s); break;
        case 2: launch_hubs_t<1>(a, s); break;
        case 4: launch_hubs_t<2>(a, s); break;
        case 8: launch_hubs_t<4>(a, s); break;
        case 16: launch_hubs_t<8>(a, s); break;
        case 32: launch_hubs_t<16>(a, s); break;
        case 64: launch_hubs_t<32>(a, s); break;
        case 128: launch_hubs_t<64>(a, s); break;
        default: break;
    }
}

void launch_stream1(const gg::RoundArgs& a, hipStream_t s) {
    static int resident = 0;
    if (!resident) {
        int dev = 0, cus = 0, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gg::expand_stream1, gg::kBlock, 0);
        resident = std::max(1, cus) * std::max(1, per_cu);
    }
    uint64_t blocks = (a.n_own + gg::kBlock - 1) / gg::kBlock;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)resident));
    hipLaunchKernelGGL(gg::expand_stream1, dim3((unsigned)blocks), dim3(gg::kBlock), 0, s, a);
}

void launch_stream(const gg::RoundArgs& a, bool maskw, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_stream1(a, s); break;  // never with masks (stream_ok)
        case 2: launch_stream_m<1>(a, maskw, s); break;
        case 4: launch_stream_m<2>(a, maskw, s); break;
        case 8: launch_stream_m<4>(a, maskw, s); break;
        case 16: launch_stream_m<8>(a, maskw, s); break;
        case 32: launch_stream_m<16>(a, maskw, s); break;
        case 64: launch_stream_m<32>(a, maskw, s); break;
        case 128: launch_stream_m<64>(a, maskw, s); break;
        default: break;
    }
}

template <int G, int WPL = 2>
void launch_stream_sync_t(const gg::RoundArgs& a, hipStream_t s) {
    static int resident = 0;
    if (!resident) {
        int dev = 0, cus = 0, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gg::expand_stream_sync<G, WPL>, gg::kBlock, 0);
        resident = std::max(1, cus) * std::max(1, per_cu);
    }
    const uint64_t rb = std::min<uint64_t>((a.n_own + gg::kBlock - 1) / gg::kBlock, 4096);
    hipLaunchKernelGGL(gg::sync_records, dim3((unsigned)std::max<uint64_t>(1, rb)), dim3(gg::kBlock), 0, s, a);
    const uint64_t ngb = gg::kBlock / G;
    uint64_t blocks = (a.n_own + ngb - 1) / ngb;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)resident));
    hipLaunchKernelGGL((gg::expand_stream_sync<G, WPL>), dim3((unsigned)blocks), dim3(gg::kBlock), 0, s, a);
}

void launch_stream_sync(const gg::RoundArgs& a, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_stream_sync_t<1, 1>(a, s); break;  // W = 64: one word per node, one lane
        case 2: launch_stream_sync_t<1>(a, s); break;
        case 4: launch_stream_sync_t<2>(a, s); break;
        case 8: launch_stream_sync_t<4>(a, s); break;
        case 16: launch_stream_sync_t<8>(a, s); break;
        case 32: launch_stream_sync_t<16>(a, s); break;
        case 64: launch_stream_sync_t<32>(a, s); break;
        case 128: launch_stream_sync_t<64>(a, s); break;
        default: break;
    }
}

// Number of distinct lanes of this engine's word range broadcast in rounds
// <= r (every engine sees every broadcast: gg_broadcast does not filter by
// owner), extended round by round from the rounds' lists. A round's list is
// dropped once the round has run (retire_round), which first extends the
// history through that round: a history extended past a dropped list would
// miss its lanes (the saturation digest, the all-full test and expand_stream1's
// saturation skip all compare set sizes with these counts).
uint32_t lanes_through(gg_engine* e, int64_t r) {
    if (r < 0) return 0;
    if (e->u_bits.size() != e->nw) e->u_bits.assign(e->nw, 0);
    while ((int64_t)e->u_hist.size() <= r) {
        const int64_t q = (int64_t)e->u_hist.size();
        uint32_t u = q ? e->u_hist.back() : 0;
        auto it = e->inj.find(q);
        if (it != e->inj.end())
            for (const auto& x : it->second) {
                const uint64_t wd = x.lane >> 6;
                if (wd < e->w0 || wd >= e->w0 + e->nw) continue;
                uint64_t& word = e->u_bits[wd - e->w0];
                const uint64_t bit = 1ull << (x.lane & 63);
                if (!(word & bit)) ++u;
                word |= bit;
            }
        e->u_hist.push_back(u);
    }
    return e->u_hist[r];
}

// Round r has run: its client broadcasts are no longer needed, once the lane
// history covers it.
uint32_t lab_of(const gg_engine* e, uint64_t node);

void retire_round(gg_engine* e, int64_t r) {
    (void)lanes_through(e, r);
    if (e->d_ltab) {  // the digest's component counts keep the round's broadcasts
        auto it = e->inj.find(r);
        if (it != e->inj.end()) {
            std::vector<uint64_t> add;
            for (const auto& x : it->second) {
                const uint64_t wd = x.lane >> 6;
                if (wd < e->w0 || wd >= e->w0 + e->nw) continue;
                const uint32_t l = lab_of(e, x.node);
                if (l != ~0u) add.push_back((uint64_t)l << 32 | x.lane);
            }
            // lret stays sorted and unique: it grows with distinct (label, lane) pairs only
            std::sort(add.begin(), add.end());
            const size_t mid = e->lret.size();
            e->lret.insert(e->lret.end(), add.begin(), add.end());
            std::inplace_merge(e->lret.begin(), e->lret.begin() + mid, e->lret.end());
            e->lret.erase(std::unique(e->lret.begin(), e->lret.end()), e->lret.end());
        }
    }
    e->inj.erase(r);
}

template <int G, int WPL>
void launch_batched_t(const gg::RoundArgs& a, hipStream_t s) {
    const uint64_t groups = a.n_own, per = gg::kBlock / G;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((groups + per - 1) / per, 8192));
    hipLaunchKernelGGL((gg::expand_batched<G, WPL>), dim3(blocks), dim3(gg::kBlock), 0, s, a);
}

void launch_batched(const gg::RoundArgs& a, hipStream_t s) {
    switch (a.nwp) {
        case 1: launch_batched_t<1, 1>(a, s); break;
        case 2: launch_batched_t<1, 2>(a, s); break;
        case 4: launch_batched_t<2, 2>(a, s); break;
        case 8: launch_batched_t<4, 2>(a, s); break;
        case 16: launch_batched_t<8, 2>(a, s); break;
        case 32: launch_batched_t<16, 2>(a, s); break;
        case 64: launch_batched_t<32, 2>(a, s); break;
        case 128: launch_batched_t<64, 2>(a, s); break;
        default: break;
    }
}

// Round r runs the streamed sync kernels (sync_records + expand_stream_sync):
// callbacks and pushes reach the expand, no partition window touches rounds
// r-3..r+1, and the engine has the sync records.
bool sync_stream_at(gg_engine* e, int64_t r) {
    if (!e->cfg.enable_sync || !e->d_srec || r < (int64_t)e->cfg.sync_base_ticks + 2) return false;
    for (int k = 0; k < 5; ++k)
        if (window_at(e, r - 3 + k)) return false;
    return true;
}

// The streamed-sync buffers (records, sender states and their bitmap, the node
// list with its bytes, the saturation digest, the reverse edge index, push
// bytes): no round before the first timer round reads or writes any of them
// (round_prep, sync_records and the sync expand kernels are the only users, and
// those run from round sync_base on), so an episode that ends before the timers
// never needs them — C5 at 2^30 nodes: 66 GiB of the 145. Allocated zeroed at
// the first call that enqueues a round >= sync_base, which is before the first
// round whose kernels touch them; from then on they stay for the topology's
// life (gg_reset keeps them). Every reader of them reads what a kernel of the
// same or the previous round wrote (pushb/pushany: the callback of r-1; sstate,
// ibits: round_prep of r; srec, nmeta: the round's own launches; sat: zero or
// bits of earlier rounds of this episode), so where in the episode the
// allocation happens cannot change a result.
int alloc_sync(gg_engine* e) {
    if (e->sync_alloc) return GG_OK;
    e->sync_alloc = true;
    const uint64_t n_own = e->n_own;
    auto zalloc = [&](auto*& p, size_t bytes) -> int {
        HIPCHK(hipMalloc(&p, std::max<size_t>(bytes, 8)));
        HIPCHK(hipMemsetAsync(p, 0, std::max<size_t>(bytes, 8), e->stream));
        return GG_OK;
    };
    int rc = GG_OK;
    if (e->cfg.enable_sync && !e->cfg.batch_ticks && (e->n_hubs == 0 || e->symmetric) && !e->sync_tiles && n_own) {
        if ((rc = zalloc(e->d_srec, 2 * n_own * sizeof(uint4)))) return rc;
        if ((rc = zalloc(e->d_sstate, e->rows))) return rc;
        if ((rc = zalloc(e->d_ibits, e->rows / 8))) return rc;
        if ((rc = zalloc(e->d_nmeta, n_own * sizeof(uint2)))) return rc;
        // saturation digest (GG_SYNC_DIGEST=0 turns it off, for A/B)
        if (!(test_knob("GG_SYNC_DIGEST") && atoi(test_knob("GG_SYNC_DIGEST")) == 0)) {
            if ((rc = zalloc(e->d_sat, e->rows / 8))) return rc;
            if ((rc = zalloc(e->d_sat_new, e->rows / 8))) return rc;
        }
        if (e->n_in_edges) {  // receivers look up whether an owned pusher sent them anything
            HIPCHK(hipMalloc(&e->d_rev, e->n_in_edges * 4));
            const unsigned blocks = (unsigned)std::min<uint64_t>((e->n_in_edges / 8 + 255) / 256 + 1, 16384);
            hipLaunchKernelGGL(gg::build_rev, dim3(blocks), dim3(256), 0, e->stream, e->d_in_ptr, e->d_in_col,
                               e->d_out_ptr, e->d_out_col, e->d_gid, n_own, e->n_in_edges, e->d_rev);
            HIPCHK(hipGetLastError());
        }
    }
    // non-empty pushes per out-edge, written by each sync callback (SyncBroadcast
    // sends nothing for an empty difference): receivers of empty pushes are not
    // candidates (GG_SYNC_ALLPUSH=1 keeps every push edge, for A/B)
    if (e->cfg.enable_sync && e->n_out_edges && !(ab_knob("GG_SYNC_ALLPUSH") && atoi(ab_knob("GG_SYNC_ALLPUSH"))))
        if ((rc = zalloc(e->d_pushb, e->n_out_edges))) return rc;
    if (!e->d_pushb) dfree(e->d_rev);
    if (e->d_pushb && e->d_srec)
        if ((rc = zalloc(e->d_pushany, e->rows))) return rc;
    return GG_OK;
}

// Before enqueueing rounds up to last_round: the streamed-sync buffers once a
// timer round is among them (alloc_sync).
int ensure_sync(gg_engine* e, int64_t last_round) {
    static const char* at = test_knob("GG_SYNC_ALLOC_ROUND");  // A/B: allocate from this round on
    const int64_t r0 = at ? (int64_t)atoi(at) : (int64_t)e->cfg.sync_base_ticks;
    if (e->sync_alloc || !e->cfg.enable_sync || last_round < r0) return GG_OK;
    return alloc_sync(e);
}

// Double-buffered lean rounds need a second set buffer: W >= 128 (the streaming
// kernels), not batched, and 16 GiB of HBM left free after it and the F rows.
// Decided at the first step after an install (round 0, so the episode starts in
// double-buffered rounds), not at the install itself: the device generator's
// scratch (C4 at 10^8 nodes: tens of GiB) is only freed afterwards.
int ensure_db(gg_engine* e) {
    if (e->db_decided) return GG_OK;
    e->db_decided = true;
    const size_t rowbytes = e->rows * e->nwp * 8;
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    // (graphs with hubs are bound by their gathers: C4 at 10^8 nodes ran 1.154 s per
    // episode either way, profiles/r3/bench_c4_db.json, and with the lean digest
    // 823 vs 826 ms for 48 GiB more HBM, profiles/r5/INDEX.md, so they keep their HBM;
    // GG_DB=1 forces the double-buffered rounds on them too)
    // GG_NO_DB=1 / GG_DB=1 (test hooks): never / whenever the graph allows it,
    // whatever the free memory (the tests pin both paths; gg_round_stats.path says
    // which one a round took)
    const bool force = test_knob("GG_DB") && atoi(test_knob("GG_DB"));
    const bool ok = e->round == 0 && e->nwp >= 2 && e->nwp <= 128 && !e->cfg.batch_ticks && (e->n_hubs == 0 || force) &&
                    (force || free_b > rowbytes + (16ull << 30)) && !test_knob("GG_NO_DB");
    if (!ok) return GG_OK;
    HIPCHK(hipMalloc(&e->d_sets[1], rowbytes));
    HIPCHK(hipMemsetAsync(e->d_sets[1], 0, rowbytes, e->stream));
    e->db_ok = true;
    e->db_active = true;
    e->f_dirty = e->P > 1;  // (sharded: the exchange writes the ghosts' F rows)
    return GG_OK;
}

// Round r is double-buffered: every round of the episode so far
// was, and r is a lean streaming round — no sync event reaches the expand and no
// partition window touches r-3..r+1 (so no message has been dropped yet either:
// the earlier rounds were lean too).
bool db_round(const gg_engine* e, int64_t r) {
    if (!e->db_active) return false;
    if (e->cfg.enable_sync && r >= (int64_t)e->cfg.sync_base_ticks + 2) return false;
    for (int k = 0; k < 5; ++k)
        if (window_at(e, r - 3 + k)) return false;
    return true;
}

// Host state after round r: which buffer holds the sets, and whether the
// episode has left the double-buffered rounds (for good). enqueue_round calls it
// while it enqueues; gg_step replays it for a batch replayed from its graph.
void db_advance(gg_engine* e, int64_t r, bool db) {
    if (db) {
        e->set_cur = (int)(r & 1);
    } else {
        e->db_active = false;
        e->f_dirty = true;
    }
    e->d_base = e->d_sets[e->set_cur];
}

// Marking rounds are for double-buffered engines on symmetric graphs without
// hubs (no hub_mark; a node's receivers are its in-list); on vertex parts the
// exchange's unpack marks the owned receivers of the ghosts that sent an F row
// (round_prep's ghost pass); GG_NO_MARK=1 keeps round_prep.
bool mark_ok(const gg_engine* e) {
    return !e->no_mark && e->symmetric && e->n_hubs == 0 && e->n_mchunks == 0 && !e->cfg.batch_ticks;
}

// Which kernel path round r takes (gg_round_stats.path, diagnostics): the host
// decides it from the round number, the windows and the buffers, so a replayed
// batch reports the same bits as the enqueued one. db: db_round(e, r) before
// db_advance.
uint64_t path_of(const gg_engine* e, int64_t r, bool db) {
    if (e->cfg.batch_ticks) return GG_PATH_BATCHED;
    bool maskw = false;
    for (int k = 0; k < 5; ++k) maskw |= window_at(e, r - 3 + k) != nullptr;
    const bool syncw = e->cfg.enable_sync && r >= (int64_t)e->cfg.sync_base_ticks + 2;
    uint64_t p = maskw ? GG_PATH_MASKED : 0;
    if (e->d_lsat) p |= GG_PATH_LSAT | (e->d_lreach ? GG_PATH_LSAT_COMP : 0u);
    if (db && mark_ok(e) && !(e->cfg.enable_sync && r >= (int64_t)e->cfg.sync_base_ticks)) p |= GG_PATH_NO_PREP;
    if (db) return p | GG_PATH_DB;
    if (syncw && !maskw && e->d_srec) return p | GG_PATH_SYNC_STREAM;
    const bool lean = !syncw && (!maskw || (e->symmetric && e->n_hubs == 0 && e->nwp >= 2));
    return p | (lean ? GG_PATH_STREAM : GG_PATH_TILES);
}

int zero_async(gg_engine* e, void* p, size_t bytes);

// Round r is a marking round with block lists (RoundArgs::block_lists: the
// marking kernel and expand_stream_db are both launched, each exits when the
// round is the other's) — enqueue_round's rule, from the host state before
// db_advance(r). db: db_round(e, r).
bool bll_round(const gg_engine* e, int64_t r, bool db) {
    static const bool no_bll = ab_knob("GG_BLOCK_LISTS") && atoi(ab_knob("GG_BLOCK_LISTS")) == 0;  // A/B
    const int64_t base = (int64_t)e->cfg.sync_base_ticks;
    const bool sync = e->cfg.enable_sync != 0;
    return db && mark_ok(e) && !(sync && r >= base) && db_round(e, r + 1) && !(sync && r + 1 >= base) &&
           e->n_hubs == 0 && !no_bll;
}

// The solo kind of marking round r (RoundArgs::solo): the kernel the device chose
// the last time this round ran (busy_hint), or 0 (launch both) when unknown.
// Test hook GG_SOLO: 0 = never solo; mark / db / alt = that kind in every marking
// round whatever the hints (every schedule is exact; only the speed differs).
uint32_t solo_of(const gg_engine* e, int64_t r, bool db) {
    if (!bll_round(e, r, db)) return 0;
    const char* force = test_knob("GG_SOLO");
    if (r == 0 && !force) return gg::SOLO_MARK;  // nothing became active before round 0: never busy
    if (force) {
        if (!strcmp(force, "0")) return 0;
        if (!strcmp(force, "mark")) return gg::SOLO_MARK;
        if (!strcmp(force, "db")) return gg::SOLO_DB;
        if (!strcmp(force, "alt")) return (r & 1) ? gg::SOLO_DB : gg::SOLO_MARK;
    }
    const int8_t h = r >= 0 && (size_t)r < e->busy_hint.size() ? e->busy_hint[r] : (int8_t)-1;
    return h < 0 ? 0u : (h ? gg::SOLO_DB : gg::SOLO_MARK);
}

// A round's busy flag (busy_count of the nodes that became active the round before): the hint
// for the next run of that round flips only after two runs in a row disagree.
void learn_busy(gg_engine* e, int64_t r, bool busy) {
    if (r < 0 || r > (1 << 20)) return;
    if (e->busy_hint.size() <= (size_t)r) {
        e->busy_hint.resize(r + 1, -1);
        e->busy_strike.resize(r + 1, 0);
    }
    const int8_t b = busy ? 1 : 0;
    if (e->busy_hint[r] < 0 || e->busy_hint[r] == b) {
        e->busy_hint[r] = b;
        e->busy_strike[r] = 0;
    } else if (++e->busy_strike[r] >= 2) {
        e->busy_hint[r] = b;
        e->busy_strike[r] = 0;
    }
}

// The solo schedule of rounds r0..r0+m-1 as enqueue_round will set it (with the
// solo kind of the round before r0), for the batch key; the host state is
// simulated and restored.
// Lean streaming rounds whose last run was busy skip compact_round and run
// dense (RoundArgs::no_list; exact either way: a dense round visits every
// node). GG_NO_LIST = 0: never; 1: in every such round whatever the hints.
bool list_skip_hint(const gg_engine* e, int64_t r) {
    const char* k = test_knob("GG_NO_LIST");
    if (k) return atoi(k) != 0;
    return r >= 0 && (size_t)r < e->busy_hint.size() && e->busy_hint[r] == 1;
}

uint64_t solo_sched_hash(gg_engine* e, int64_t r0, uint32_t m) {
    const bool sdb = e->db_active, sfd = e->f_dirty;
    const int sset = e->set_cur;
    uint64_t h = gg_mix64(0x501Dull ^ e->last_solo);
    for (uint32_t k = 0; k < m; ++k) {
        const bool dbk = db_round(e, r0 + k);
        h = gg_mix64(h ^ ((uint64_t)solo_of(e, r0 + k, dbk) << 8) ^ ((uint64_t)list_skip_hint(e, r0 + k) << 16) ^ k);
        db_advance(e, r0 + k, dbk);
    }
    e->db_active = sdb;
    e->f_dirty = sfd;
    e->set_cur = sset;
    e->d_base = e->d_sets[sset];
    return h;
}

// Enqueue round e->round (kernels only). inj: device pairs for this round.
int enqueue_round(gg_engine* e, const uint32_t* d_inj, uint32_t n_inj, unsigned long long* d_ctr,
                  const uint32_t* d_tab = nullptr) {
    const int64_t r = e->round;
    const bool db = db_round(e, r);
    e->last_path = path_of(e, r, db);
    if (e->db_active && !db && r > 0) {
        // the first round that needs F rows: those of round r-1, from its two set buffers
        const uint64_t n = e->n_own * e->nwp;
        const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
        hipLaunchKernelGGL(gg::materialize_F, dim3(blocks), dim3(256), 0, e->stream, e->d_sets[(r - 1) & 1],
                           e->d_sets[r & 1], e->d_flg[(r - 1) & 1], e->d_F[(r - 1) & 1], e->n_own, (uint32_t)e->nwp);
        HIPCHK(hipGetLastError());
    }
    db_advance(e, r, db);
    gg::RoundArgs a{};
    a.db = db ? 1 : 0;
    a.base_prev = db ? e->d_sets[(r + 1) & 1] : nullptr;
    a.in_ptr = e->d_in_ptr;
    a.in_col = e->d_in_col;
    a.out_ptr = e->d_out_ptr;
    a.out_col = e->d_out_col;
    a.base = e->d_base;
    a.F_prev = e->d_F[(r + 1) & 1];
    a.F_cur = e->d_F[r & 1];
    a.flg_prev = e->d_flg[(r + 1) & 1];
    a.flg_cur = e->d_flg[r & 1];
    a.cand = e->d_cand + (size_t)(r & 1) * e->rows;
    a.cand_next = e->d_cand + (size_t)((r + 1) & 1) * e->rows;
    a.flg_prev_w = e->d_flg[(r + 1) & 1];
    a.zmark = e->d_zmark;
    a.tile_cand = e->d_tile_cand;
    a.work = e->d_work;
    a.n_work = e->d_n_work + 2 * (r & 1);
    a.n_work_next = e->d_n_work + 2 * ((r + 1) & 1);
    a.bcount = e->d_bcount;
    a.nodes = e->d_nodes;
    a.act = e->d_act;
    a.act_deg = e->d_act_deg;
    a.act_s = e->d_act_s;
    a.act_deg_s = e->d_act_deg_s;
    a.tot_s = e->d_tot_s;
    a.abits = e->d_abits;
    a.ff_ok = e->ff_ok ? (int32_t)e->ff_frac16 : 0;
    // W = 64: a sender's F word is one 8-byte request, so below ~V/256 edges with
    // data the saved gathers cost less than the bitmap pass over V flag bytes
    a.ff_min = e->nwp == 1 ? e->n_own / 256 : 0;
    a.prep_wide = ab_knob("GG_PREP_WIDE") && atoi(ab_knob("GG_PREP_WIDE")) ? 1 : 0;
    a.tile_nodes = (uint32_t)e->tile_nodes;
    a.symmetric = e->symmetric ? 1 : 0;
    a.n_edges = e->n_in_edges;
    a.rows = e->rows;
    a.gid = e->d_gid;
    a.ghost0 = e->ghost0;
    a.n_ghost = e->n_ghost;
    a.gout_ptr = e->d_gout_ptr;
    a.gout_col = e->d_gout_col;
    a.hub_deg = e->hub_deg;
    a.hchunks = e->d_hchunks;
    a.n_hchunks = e->n_hchunks;
    a.hubs = e->d_hubs;
    a.hub_c0 = e->d_hub_c0;
    a.n_hubs = e->n_hubs;
    a.hscratch = e->d_hscratch;
    a.hflag = e->d_hflag;
    a.hlive = e->d_hlive;
    a.mchunks = e->d_mchunks;
    a.srec = e->d_srec;
    a.pushb = e->d_pushb;
    a.rev = e->d_rev;
    a.sstate = e->d_sstate;
    a.ibits = e->d_ibits;
    if (e->d_sat) {
        a.sat = e->d_sat;
        a.sat_new = e->d_sat_new;
        a.usat = lanes_through(e, r);
        a.sat_reset = (r == 0 || a.usat != lanes_through(e, r - 1)) ? 1u : 0u;
    }
    a.lsat = nullptr;
    a.lusat = 0;
    a.lreach = e->d_lreach;
    if (e->d_lsat) {
        // lean saturation digest: a bit is set when the node's set holds every
        // lane injected through the round that set it; lanes injected in r-1 >= 1
        // void the older bits (those of r-1 too: it only costs their skips)
        a.lsat = e->d_lsat;
        a.lusat = lanes_through(e, r);
        static const bool nomark = ab_knob("GG_LSAT_NOMARK") != nullptr;  // A/B: read only
        a.lmark = nomark ? 0u : 1u;
        // (component targets cover the whole known schedule: ltab_sync clears the
        // digest when they change)
        if (!e->d_lreach && r >= 2 && lanes_through(e, r - 1) != lanes_through(e, r - 2))
            if (int rz = zero_async(e, e->d_lsat, e->rows)) return rz;
    }
    a.n_mchunks = e->n_mchunks;
    a.fired_m1 = e->d_fired[(r - 1) & 3];
    a.fired_m2 = e->d_fired[(r - 2) & 3];
    a.fired_m3 = e->d_fired[(r - 3) & 3];
    a.fired_cur = e->d_fired[r & 3];
    a.sync_next = e->d_sync_next;
    a.sync_k = e->d_sync_k;
    bool maskw = false;
    a.ewin = 0;
    for (int k = 0; k < 5; ++k) {
        const Window* w = window_at(e, r - 3 + k);
        a.grp[k] = w ? w->d_grp : nullptr;
        a.ebits[k] = w ? w->d_ebits : nullptr;
        if (w && w->edges) a.ewin |= 1u << k;
        maskw |= a.grp[k] != nullptr;
    }
    a.inj = d_inj;
    a.n_inj = n_inj;
    a.inj_tab = d_tab;
    static const bool no_full = ab_knob("GG_ALL_FULL") && atoi(ab_knob("GG_ALL_FULL")) == 0;  // A/B
    a.tot = no_full ? nullptr : e->d_tot;
    a.full_new = (unsigned long long)e->n_own * lanes_through(e, r - 1);
    a.lanes_prev = lanes_through(e, r - 1);
    a.counters = d_ctr;
    a.n_own = e->n_own;
    a.own0 = 0;
    a.lo = 0;
    a.nwp = (uint32_t)e->nwp;
    a.nw = (uint32_t)e->nw_g;
    a.word0 = (uint32_t)e->w0;
    a.count_nodes = e->lgrp == 0 ? 1u : 0u;
    a.round = r;
    a.seed = e->cfg.seed;
    a.sync_base = e->cfg.sync_base_ticks;
    a.sync_jitter = e->cfg.sync_jitter_ticks;
    a.sync_mix = gg_mix64(e->cfg.seed ^ GG_TAG_SYNC);
    a.sync_rcp = gg_sync_rcp(e->cfg.sync_jitter_ticks);
    a.enable_sync = e->cfg.enable_sync;
    // timers fire from round sync_base on (round_prep: timers, read_ok counts);
    // the first callbacks and pushes reach the expand kernels two rounds later
    const int64_t base = (int64_t)e->cfg.sync_base_ticks;
    const bool syncw_prep = e->cfg.enable_sync && r >= base;
    const bool syncw = e->cfg.enable_sync && r >= base + 2;
    // marking rounds (RoundArgs::mark_cand): this double-buffered round's expand
    // marks round r+1's candidates when r+1 is one too (before the timers), and
    // such a round r+1 launches no round_prep (round 0: nothing to mark yet)
    if (db && mark_ok(e) && !syncw_prep) {
        a.prep_in_compact = 1;
        a.mark_cand = (db_round(e, r + 1) && !(e->cfg.enable_sync && r + 1 >= base)) ? 1u : 0u;
    }
    e->last_mark = a.mark_cand != 0;
    // streaming rounds: no sync event reaches the expand; partition windows only
    // on symmetric graphs without hubs at W >= 128 (expand_stream<.., MASKW>)
    // streamed sync rounds (sync_records + expand_stream_sync [+ hub_sync_*]): no masks
    const bool sync_stream = syncw && !maskw && e->d_srec != nullptr;
    a.nmeta = sync_stream ? e->d_nmeta : nullptr;
    if (e->cfg.batch_ticks) {  // batched gossip: one kernel over every node
        a.pend = e->d_pend;
        a.pend_src = e->d_pend_src;
        a.batch_tick = (r + 1) % (int64_t)e->cfg.batch_ticks == 0 ? 1u : 0u;
        if (e->d_bset[0]) {  // sync timers: this round's fired bits are set by the kernel
            a.bset_prev = e->d_bset[(r + 1) & 1];
            a.bset_cur = e->d_bset[r & 1];
            if (int rz = zero_async(e, a.fired_cur, e->rows / 8)) return rz;
        }
        if (n_inj) {
            hipLaunchKernelGGL(gg::mark_injections, dim3(gg::kMarkInjBlocks), dim3(256), 0, e->stream, a);
            HIPCHK(hipGetLastError());
        }
        a.tot = nullptr;  // no round_prep here to start each round's slot
        a.dr = e->d_dr;  // first-seen rounds are written by the kernel (F rows hold batches here)
        a.dr_w = (uint32_t)(e->nw * 64);
        if (a.n_own) launch_batched(a, e->stream);
        HIPCHK(hipGetLastError());
        return GG_OK;
    }
    if (e->d_pushany) {  // streamed callbacks mark the receivers of their pushes for the next round
        a.pushany = e->d_pushany;
        a.mark_next = (sync_stream && sync_stream_at(e, r + 1)) ? 1u : 0u;
        a.push_marked = (sync_stream && sync_stream_at(e, r - 1)) ? 1u : 0u;
    }
    a.stream_ok = ((!syncw && (!maskw || (e->symmetric && e->n_hubs == 0 && e->nwp >= 2))) || sync_stream) ? 1 : 0;

    if (a.n_own) {
        {
            // grid-stride over the nodes; a capped grid keeps the launch cheap in
            // dense lean rounds, where it is a no-op (C2 A/B: 1024 blocks 1.99 ms/episode,
            // 4096 2.02, 256 2.10; GG_PREP_BLOCKS overrides)
            const uint64_t prep_cap = e->prep_cap;
            if (e->d_sat && r == base + 2) {  // the digest's first bits (sat_scan)
                const uint64_t thr = a.n_own * std::max<uint64_t>(1, e->nwp / 2);
                hipLaunchKernelGGL(gg::sat_scan, dim3((unsigned)((thr + gg::kBlock - 1) / gg::kBlock)), dim3(gg::kBlock),
                                   0, e->stream, e->d_base, a.n_own, (uint32_t)e->nwp, lanes_through(e, r - 1), e->d_sat);
                HIPCHK(hipGetLastError());
            }
            // sync rounds do real work per node: a larger capped grid (each block's
            // counter flush is a few same-address atomics, so not one block per 256 nodes)
            // (timer rounds: 8+ nodes per thread; C2 at 2^20 nodes, A/B on one box
            // (profiles/r3/ab_sync_prep.log): 1024 blocks 20 / 19 us per timer round, 4096 26 / 25 us)
            const uint64_t sync_cap = ab_knob("GG_SYNC_PREP_BLOCKS") ? (uint64_t)atoi(ab_knob("GG_SYNC_PREP_BLOCKS"))
                                      : std::min<uint64_t>(4096, std::max<uint64_t>(1024, a.n_own / 2048));
            const uint64_t blocks = std::max<uint64_t>(
                1, std::min<uint64_t>((a.n_own + gg::kBlock - 1) / gg::kBlock, syncw_prep ? sync_cap : prep_cap));
            dim3 grid((unsigned)blocks), block(gg::kBlock);
            if (a.prep_in_compact) {
                // the expand of r-1 marked this round's candidates; compact_round sums the rings
            } else if (syncw_prep) {
                if (maskw) hipLaunchKernelGGL((gg::round_prep<true, true>), grid, block, 0, e->stream, a);
                else hipLaunchKernelGGL((gg::round_prep<true, false>), grid, block, 0, e->stream, a);
            } else {
                if (maskw) hipLaunchKernelGGL((gg::round_prep<false, true>), grid, block, 0, e->stream, a);
                else hipLaunchKernelGGL((gg::round_prep<false, false>), grid, block, 0, e->stream, a);
            }
            HIPCHK(hipGetLastError());
        }
        if (e->n_mchunks) {  // high out-degree senders mark their receivers (sparse rounds);
        // before mark_injections, whose CA_INJ bit these plain stores would clear
            const unsigned blocks = (unsigned)std::min<uint64_t>(e->n_mchunks, 4096);
            hipLaunchKernelGGL(gg::hub_mark, dim3(blocks), dim3(gg::kBlock), 0, e->stream, a);
            HIPCHK(hipGetLastError());
        }
        if (n_inj) {
            hipLaunchKernelGGL(gg::mark_injections, dim3(gg::kMarkInjBlocks), dim3(256), 0, e->stream, a);
            HIPCHK(hipGetLastError());
        }
        // block lists (RoundArgs::block_lists): a marking round needs
        // no compact_round — its two double-buffered expand kernels list their
        // blocks' candidates themselves (C2: one launch and a list pass less a round)
        static const bool no_bll = ab_knob("GG_BLOCK_LISTS") && atoi(ab_knob("GG_BLOCK_LISTS")) == 0;  // A/B
        a.block_lists = (a.prep_in_compact && a.mark_cand && a.db && a.stream_ok && !sync_stream && !maskw &&
                         e->n_hubs == 0 && !no_bll) ? 1u : 0u;
        // one expand kernel in a marking round when the last run of it says which
        a.solo = a.block_lists ? solo_of(e, r, db) : 0u;
        a.prev_mark = e->last_solo == gg::SOLO_MARK ? 1u : e->last_solo == gg::SOLO_DB ? 2u : 0u;
        e->last_solo = a.solo;
        if (a.solo) e->last_path |= GG_PATH_SOLO;
        // a lean streaming round the last run found busy: no list, dense (exact either
        // way). Not when compact_round sums the rings (prep_in_compact)
        a.no_list = (!a.block_lists && a.stream_ok && !sync_stream && !a.prep_in_compact && !e->cfg.batch_ticks &&
                     list_skip_hint(e, r)) ? 1u : 0u;
        if (!a.block_lists && !a.no_list) {
            const uint64_t groups = (a.n_own + 7) / 8;  // >= tile groups
            const uint64_t per_block = (uint64_t)gg::kBlock * gg::kCompactQ;
            const uint64_t nb = (groups + per_block - 1) / per_block;
            if (e->d_bcount) {  // split compaction (large graphs): counts, offsets, list
                hipLaunchKernelGGL(gg::compact_round<1>, dim3((unsigned)nb), dim3(gg::kBlock), 0, e->stream, a);
                hipLaunchKernelGGL(gg::compact_scan, dim3(1), dim3(1024), 0, e->stream, a, (uint32_t)nb);
                hipLaunchKernelGGL(gg::compact_round<2>, dim3((unsigned)nb), dim3(gg::kBlock), 0, e->stream, a);
            } else {
                hipLaunchKernelGGL(gg::compact_round<0>, dim3((unsigned)nb), dim3(gg::kBlock), 0, e->stream, a);
            }
            HIPCHK(hipGetLastError());
        }
        if (sync_stream) {
            launch_stream_sync(a, e->stream);
            if (e->n_hubs) {
                HIPCHK(hipGetLastError());
                launch_hub_sync(a, e->stream);
            }
        } else if (a.stream_ok) {  // lean rounds: all nodes (dense) or the candidate list (sparse)
            if (e->ff_ok && !maskw) {  // the sender bitmap of a flags-first round (the kernel decides)
                const uint64_t blocks = std::min<uint64_t>((e->rows / 16 + gg::kBlock - 1) / gg::kBlock, 4096);
                hipLaunchKernelGGL(gg::pack_act_bits, dim3((unsigned)blocks), dim3(gg::kBlock), 0, e->stream, a);
                HIPCHK(hipGetLastError());
            }
            launch_stream(a, maskw, e->stream);
            if (e->n_hubs) {
                HIPCHK(hipGetLastError());
                launch_hubs(a, e->stream);
            }
        } else {
            launch_expand(a, syncw, maskw, e->stream);
        }
        HIPCHK(hipGetLastError());
        if (e->d_dr) {
            const uint64_t n = a.n_own * e->nw;
            hipLaunchKernelGGL(gg::track_delivery, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream,
                               db ? a.base : a.F_cur, a.flg_cur, e->d_dr, a.n_own, a.own0, (uint32_t)e->nwp,
                               (uint32_t)e->nw, (uint32_t)(e->nw * 64), (int32_t)r, a.base_prev);
            HIPCHK(hipGetLastError());
        }
    }
    return GG_OK;
}

// Host-side stats of one round from its 64 counter slots; per-kind times from
// the device clock stamps (first block start .. last block end, 100 MHz).
// slots: nslots x kCounters (kSlots raw slots, or 1 slot folded by gg::fold_slots)
void fold_stats(gg_engine* e, const unsigned long long* slots, int64_t round, gg_round_stats* s, int nslots = gg::kSlots,
                bool learn = true) {
    unsigned long long c[gg::kCounters] = {0};
    unsigned long long t0[gg::K_NKIND], t1[gg::K_NKIND];
    for (int q = 0; q < gg::K_NKIND; ++q) t0[q] = ~0ull, t1[q] = 0;
    for (int k = 0; k < nslots; ++k) {
        for (int j = 0; j < gg::kCounters; ++j) c[j] += slots[k * gg::kCounters + j];
        for (int q = 0; q < gg::K_NKIND; ++q) {
            const unsigned long long si = slots[k * gg::kCounters + gg::kStamp0 + 2 * q];
            if (si) t0[q] = std::min(t0[q], ~si);
            t1[q] = std::max(t1[q], slots[k * gg::kCounters + gg::kStamp0 + 2 * q + 1]);
        }
    }
    auto span = [](unsigned long long a, unsigned long long b) {
        return (b > a && a != ~0ull) ? (double)(b - a) / 1.0e5 : 0.0;
    };
    const unsigned long long ta = std::min(t0[gg::K_PREP], std::min(t0[gg::K_EXPAND], t0[gg::K_STREAM]));
    const unsigned long long tb = std::max(t1[gg::K_PREP], std::max(t1[gg::K_EXPAND], t1[gg::K_STREAM]));
    const double ms = span(ta, tb);
    s->prep_ms = span(t0[gg::K_PREP], t1[gg::K_PREP]);
    s->expand_ms = span(t0[gg::K_EXPAND], t1[gg::K_EXPAND]);
    s->stream_ms = span(t0[gg::K_STREAM], t1[gg::K_STREAM]);
    s->prep_bytes = c[gg::kBytes0 + gg::K_PREP];
    s->expand_bytes = c[gg::kBytes0 + gg::K_EXPAND];
    s->stream_bytes = c[gg::kBytes0 + gg::K_STREAM];
    s->sent_bytes = 0;
    s->path = 0;
    s->round = round;
    s->new_bits = c[gg::C_NEW];
    s->fwd_sent = c[gg::C_FWD_SENT];
    s->fwd_delivered = c[gg::C_FWD_DELIV];
    s->pushes = c[gg::C_PUSH];
    s->push_delivered = c[gg::C_PUSH_DELIV];
    s->acks = e->pend_acks;
    s->reads = c[gg::C_READS];
    s->read_oks = c[gg::C_READ_OKS];
    s->dropped = c[gg::C_DROPPED] + e->pend_ackdrop;
    s->syncs_fired = c[gg::C_FIRED];
    e->hash_total += c[gg::C_HASH];
    s->seen_hash = e->hash_total;
    s->kernel_ms = ms;
    s->work_rows = c[gg::C_ACTIVE];
    s->work_gathers = c[gg::C_GATHERS];
    e->pend_acks = c[gg::C_NEXT_ACKS];
    e->pend_ackdrop = c[gg::C_NEXT_ACKDROP];
    // round + 1 is busy (the stream kernels' busy_count, from the nodes that became
    // active in this round): the hint for which expand kernel its next run needs
    if (learn)
        learn_busy(e, round + 1, 2.0 * (double)c[gg::C_NACT] * (double)e->n_in_edges >=
                                     (double)e->n_own * (double)e->n_own);
}

// Zero `bytes` (a multiple of 8, 16-byte aligned) on the engine stream with a
// kernel of ours: every clear that can sit inside a captured batch (gg::zero_words).
int zero_async(gg_engine* e, void* p, size_t bytes) {
    const uint64_t n = bytes / 8;
    if (!n) return GG_OK;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n / 2 + 255) / 256, 1024));
    hipLaunchKernelGGL(gg::zero_words, dim3(blocks), dim3(256), 0, e->stream, reinterpret_cast<uint64_t*>(p), n);
    HIPCHK(hipGetLastError());
    return GG_OK;
}

int ensure_events(gg_engine* e, size_t n) {
    while (e->ev.size() < n) {
        hipEvent_t x;
        HIPCHK(hipEventCreate(&x));
        e->ev.push_back(x);
    }
    return GG_OK;
}

int ensure_inj(gg_engine* e, size_t pairs) {
    if (pairs <= e->inj_cap) return GG_OK;
    size_t cap = std::max<size_t>(pairs, 2 * e->inj_cap + 1024);
    HIPCHK(hipStreamSynchronize(e->stream));
    dfree(e->d_inj);
    if (e->h_inj) (void)hipHostFree(e->h_inj);
    e->h_inj = nullptr;
    HIPCHK(hipMalloc(&e->d_inj, cap * 8));
    HIPCHK(hipHostMalloc(&e->h_inj, cap * 8));
    e->inj_cap = cap;
    e->inj_dev_hash = 0;
    return GG_OK;
}

// Local row of an owned node, ~0u if another engine owns it.
uint32_t local_row(const gg_engine* e, uint64_t node) {
    if (node >= e->V) return ~0u;
    if (e->range_mode) {
        if (node < e->range_lo || node >= e->range_hi) return ~0u;
        return e->own_row.empty() ? (uint32_t)(node - e->range_lo) : e->own_row[node - e->range_lo];
    }
    if (e->loc_of.empty()) return (uint32_t)node;
    return e->loc_of[node];
}

// A node's component label (lean digest targets), ~0u if unknown.
uint32_t lab_of(const gg_engine* e, uint64_t node) {
    if (e->h_lab.empty() || node >= e->V) return ~0u;
    if (e->lab_global) return e->h_lab[node];
    const uint32_t l = local_row(e, node);
    return l < e->h_lab.size() ? e->h_lab[l] : ~0u;
}

// The lean digest's component targets: per label, the distinct lanes (of this
// engine's range) broadcast into the component over the whole known schedule —
// retired rounds and every round still listed — so a target is never below
// what the component will receive, and equals it once every listed round has
// run (a value sent twice into one component counts once). When the table changes (new
// broadcasts, another episode's set) it is uploaded, every owned row's target
// refilled and the digest cleared (its bits were judged against the old
// targets). Called before a batch is enqueued (never while capturing).
int ltab_sync(gg_engine* e) {
    if (!e->d_ltab) return GG_OK;
    std::vector<uint64_t> pend;  // the listed rounds' pairs, merged with the retired ones (sorted, unique)
    for (const auto& kv : e->inj)
        for (const auto& x : kv.second) {
            const uint64_t wd = x.lane >> 6;
            if (wd < e->w0 || wd >= e->w0 + e->nw) continue;
            const uint32_t l = lab_of(e, x.node);
            if (l != ~0u) pend.push_back((uint64_t)l << 32 | x.lane);
        }
    std::sort(pend.begin(), pend.end());
    std::vector<uint64_t> keys;
    keys.reserve(e->lret.size() + pend.size());
    std::set_union(e->lret.begin(), e->lret.end(), pend.begin(), pend.end(), std::back_inserter(keys));
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    std::vector<std::pair<uint32_t, uint32_t>> t;
    for (const uint64_t k : keys) {
        const uint32_t l = (uint32_t)(k >> 32);
        if (t.empty() || t.back().first != l) t.push_back({l, 0u});
        ++t.back().second;
    }
    uint64_t h = gg_mix64(0x6c7361747461626cull ^ t.size());
    for (const auto& p : t) h = gg_mix64(h ^ ((uint64_t)p.first << 32 | p.second));
    h |= 1;  // (0: none yet)
    if (h == e->ltab_hash) return GG_OK;
    if (e->ltab_ev_live) {  // the previous upload has read h_ltab
        HIPCHK(hipEventSynchronize(e->ltab_ev));
        e->ltab_ev_live = false;
    }
    std::vector<uint32_t>& buf = e->h_ltab;
    buf.assign(1, t.size() > e->ltab_cap ? gg::kTabOverflow : (uint32_t)t.size());
    if (buf[0] != gg::kTabOverflow)
        for (const auto& p : t) {
            buf.push_back(p.first);
            buf.push_back(p.second);
        }
    HIPCHK(hipMemcpyAsync(e->d_ltab, buf.data(), buf.size() * 4, hipMemcpyHostToDevice, e->stream));
    if (!e->ltab_ev) HIPCHK(hipEventCreateWithFlags(&e->ltab_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e->ltab_ev, e->stream));
    e->ltab_ev_live = true;
    hipLaunchKernelGGL(gg::lreach_fill_tab, dim3((unsigned)std::min<uint64_t>((e->n_own + 255) / 256, 8192)), dim3(256),
                       0, e->stream, e->d_llab, e->d_ltab, e->d_lreach, e->n_own);
    HIPCHK(hipGetLastError());
    if (int rc = zero_async(e, e->d_lsat, e->rows)) return rc;
    e->ltab_hash = h;
    return GG_OK;
}

// Pack the owned injections of rounds [r0, r0+n) into h_inj; off[k] = first pair of round r0+k.
size_t pack_injections(gg_engine* e, int64_t r0, uint32_t n, std::vector<size_t>& off, size_t base = 0) {
    if (ltab_sync(e) != GG_OK) return (size_t)-1;
    off.assign(n + 1, 0);
    std::vector<std::pair<uint32_t, uint32_t>> tmp;
    for (uint32_t k = 0; k < n; ++k) {
        off[k] = tmp.size();
        auto it = e->inj.find(r0 + k);
        if (it == e->inj.end()) continue;
        const size_t b = tmp.size();
        for (const auto& x : it->second) {
            const uint32_t l = local_row(e, x.node);
            const uint64_t wd = x.lane >> 6;  // another lane group's value: not this engine's
            if (l != ~0u && wd >= e->w0 && wd < e->w0 + e->nw) tmp.emplace_back(l, x.lane - 64 * (uint32_t)e->w0);
        }
        std::stable_sort(tmp.begin() + b, tmp.end(),
                         [](const auto& p, const auto& q) { return p.first < q.first; });
    }
    off[n] = tmp.size();
    if (ensure_inj(e, base + tmp.size()) != GG_OK) return (size_t)-1;
    for (size_t t = 0; t < tmp.size(); ++t) {
        e->h_inj[2 * (base + t)] = tmp[t].first;
        e->h_inj[2 * (base + t) + 1] = tmp[t].second;
    }
    return tmp.size();
}


// ---- launch cache: a multi-round batch is captured once into a hipGraph and
// replayed while (first round, length, the rounds that inject, lanes injected
// so far, partition windows, buffers) are unchanged — e.g. every episode after
// gg_reset in a benchmark loop, with the same or fresh injections (the kernels
// read the pairs and each round's share of them from device memory). The
// replayed kernels are exactly the captured launches; only host launch cost is
// saved. GG_NO_GRAPH=1 disables it.
template <class F>
int run_batch(gg_engine* e, int64_t r0, uint32_t m, const std::vector<size_t>& off, size_t total, F&& enqueue,
              bool wait = true) {
    static const bool no_graph = ab_knob("GG_NO_GRAPH") != nullptr;
    uint64_t h = gg_mix64(total);
    for (size_t t = 0; t < 2 * total; ++t) h = gg_mix64(h ^ e->h_inj[t]);
    // the same pairs as the last upload (every episode of a benchmark loop): d_inj
    // already holds them, so the copy (and its wait before h_inj is reused) is skipped
    if (total && h != e->inj_dev_hash) {
        HIPCHK(hipMemcpyAsync(e->d_inj, e->h_inj, total * 8, hipMemcpyHostToDevice, e->stream));
        if (!e->inj_ev) HIPCHK(hipEventCreateWithFlags(&e->inj_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(e->inj_ev, e->stream));
        e->inj_ev_live = true;
        e->inj_dev_hash = h;
    }
    // the rounds' first pairs, read by the kernels (inj_tab): the captured launch
    // sequence does not name the pairs, so new injections in the same rounds
    // replay it after these two copies (a fresh episode of a benchmark loop)
    if (!e->d_injtab) {
        HIPCHK(hipMalloc(&e->d_injtab, (kMaxBatch + 1) * sizeof(uint32_t)));
        HIPCHK(hipHostMalloc(&e->h_injtab, (kMaxBatch + 1) * sizeof(uint32_t)));
    }
    uint64_t th = gg_mix64(m);
    for (size_t k = 0; k <= m; ++k) th = gg_mix64(th ^ off[k]);
    if (th != e->injtab_dev_hash) {
        for (size_t k = 0; k <= m; ++k) e->h_injtab[k] = (uint32_t)off[k];
        HIPCHK(hipMemcpyAsync(e->d_injtab, e->h_injtab, (m + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
        if (!e->inj_ev) HIPCHK(hipEventCreateWithFlags(&e->inj_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(e->inj_ev, e->stream));
        e->inj_ev_live = true;
        e->injtab_dev_hash = th;
    }
    if (no_graph || m < 4 || e->graph_broken) {
        if (!wait) return enqueue();  // (gg_run_episodes: timed and synchronised by the caller)
        HIPCHK(hipEventRecord(e->ev[0], e->stream));
        int rc = enqueue();
        if (rc) return rc;
        HIPCHK(hipEventRecord(e->ev[1], e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
        e->step_event_ms += ms;
        return GG_OK;
    }
    BatchKey key;
    key.r0 = r0;
    key.m = m;
    key.windows = e->windows.size();
    key.inj_buf = e->d_inj;
    key.db_state = (e->db_active ? 2 : 0) | e->set_cur;
    key.solo_hash = solo_sched_hash(e, r0, m);
    key.zr = e->batch_zr;
    {  // which rounds inject (mark_injections is launched only there), not what
        uint64_t p = gg_mix64(m);
        for (size_t k = 0; k < m; ++k) p = gg_mix64(p ^ (off[k + 1] > off[k] ? 2 * k + 1 : 2 * k));
        key.inj_hash = p;
    }
    {  // the digest's usat and the all-full test's full_new follow the lanes injected so far
        uint64_t u = gg_mix64(~0ull);
        for (int64_t q = r0 - 1; q < r0 + (int64_t)m; ++q) u = gg_mix64(u ^ lanes_through(e, q));
        key.u_hash = u;
    }
    if (!(e->graph_exec && key == e->graph_key)) {
        if (e->graph_exec) (void)hipGraphExecDestroy(e->graph_exec);
        e->graph_exec = nullptr;
        hipGraph_t g = nullptr;
        if (hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            e->graph_broken = true;
            return run_batch(e, r0, m, off, 0, enqueue, wait);
        }
        const int rc = enqueue();
        const hipError_t ec = hipStreamEndCapture(e->stream, &g);
        hipGraphExec_t ge = nullptr;
        if (rc || ec != hipSuccess || !g || hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            e->graph_broken = true;  // fall back to direct launches for good
            return run_batch(e, r0, m, off, 0, enqueue, wait);
        }
        (void)hipGraphDestroy(g);
        e->graph_exec = ge;
        e->graph_key = key;
    }
    if (!wait) {
        HIPCHK(hipGraphLaunch(e->graph_exec, e->stream));
        return GG_OK;
    }
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    HIPCHK(hipGraphLaunch(e->graph_exec, e->stream));
    HIPCHK(hipEventRecord(e->ev[1], e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
    e->step_event_ms += ms;
    return GG_OK;
}


// Edge-balanced cut of a node order into `parts` contiguous ranges (weight of a
// node: in-degree + 1, the pull work of its row).
void balanced_ranges(uint64_t V, const int64_t* tin, const std::vector<uint32_t>& order, uint32_t parts,
                     std::vector<uint64_t>& plo) {
    plo.assign(parts + 1, V);
    plo[0] = 0;
    const uint64_t total = (uint64_t)tin[V] + V;
    uint64_t cum = 0;
    uint32_t p = 1;
    for (uint64_t pos = 0; pos < V && p < parts; ++pos) {
        const uint64_t v = order.empty() ? pos : order[pos];
        cum += (uint64_t)(tin[v + 1] - tin[v]) + 1;
        while (p < parts && cum >= total * p / parts) plo[p++] = pos + 1;
    }
    while (p < parts) plo[p++] = V;
}

void owners_of(uint64_t V, const std::vector<uint32_t>& order, const std::vector<uint64_t>& plo,
               std::vector<uint32_t>& owner) {
    owner.assign(V, 0);
    for (uint32_t p = 0; p + 1 < plo.size(); ++p)
        for (uint64_t pos = plo[p]; pos < plo[p + 1]; ++pos) owner[order.empty() ? pos : order[pos]] = p;
}

uint64_t cut_edges(uint64_t V, const int64_t* row_ptr, const int32_t* col, const std::vector<uint32_t>& owner) {
    uint64_t cut = 0;
    for (uint64_t v = 0; v < V; ++v)
        for (int64_t k = row_ptr[v]; k < row_ptr[v + 1]; ++k) cut += owner[v] != owner[(uint32_t)col[k]];
    return cut;
}

// The sharded engine's node order: the native id order or a DFS preorder over
// the out-lists (roots in ascending id, neighbours ascending), whichever cuts
// fewer edges when split into edge-balanced ranges (trees: subtrees stay whole;
// grids: native rows). Deterministic, so every rank computes the same one.
void choose_partition(uint64_t V, const int64_t* row_ptr, const int32_t* col, const int64_t* tin, uint32_t parts,
                      std::vector<uint32_t>& order, std::vector<uint64_t>& plo, std::vector<uint32_t>& owner) {
    std::vector<uint64_t> plo_n;
    std::vector<uint32_t> own_n;
    balanced_ranges(V, tin, {}, parts, plo_n);
    owners_of(V, {}, plo_n, own_n);
    const uint64_t cut_n = cut_edges(V, row_ptr, col, own_n);
    std::vector<uint32_t> dfs;
    dfs.reserve(V);
    {
        std::vector<uint8_t> seen(V, 0);
        std::vector<uint32_t> stack;
        std::vector<int64_t> next(V);
        for (uint64_t root = 0; root < V; ++root) {
            if (seen[root]) continue;
            seen[root] = 1;
            dfs.push_back((uint32_t)root);
            next[root] = row_ptr[root];
            stack.push_back((uint32_t)root);
            while (!stack.empty()) {
                const uint32_t v = stack.back();
                if (next[v] == row_ptr[v + 1]) {
                    stack.pop_back();
                    continue;
                }
                const uint32_t u = (uint32_t)col[next[v]++];
                if (seen[u]) continue;
                seen[u] = 1;
                dfs.push_back(u);
                next[u] = row_ptr[u];
                stack.push_back(u);
            }
        }
    }
    std::vector<uint64_t> plo_d;
    std::vector<uint32_t> own_d;
    balanced_ranges(V, tin, dfs, parts, plo_d);
    owners_of(V, dfs, plo_d, own_d);
    const uint64_t cut_d = cut_edges(V, row_ptr, col, own_d);
    if (cut_d < cut_n) {
        // the DFS ranges decide who owns what; inside a part the rows keep the
        // native id order (a tree's native order is breadth-first: a node's
        // children are neighbouring rows and siblings share their parent's row,
        // which the DFS order scatters — C2's part of 2^20 nodes at world 2: dense
        // rounds 0.125 -> 0.097 ms, episode kernels 1.93 -> 1.58 ms vs 1.54 for the
        // single engine, tools/dist_rounds.py)
        for (uint32_t p = 0; p < parts; ++p) std::sort(dfs.begin() + plo_d[p], dfs.begin() + plo_d[p + 1]);
        order.swap(dfs);
        plo.swap(plo_d);
        owner.swap(own_d);
    } else {
        order.clear();
        plo.swap(plo_n);
        owner.swap(own_n);
    }
}

// Local row order of an unsharded engine: on a power-law graph (max in-degree
// > 16 x the mean, or GG_ORDER=degree) the nodes by descending in-degree, ties
// by id: the hubs, which most in-lists name (R-MAT at 2^22 nodes: the top 1% of
// nodes hold 56% of all edge ends), share cache lines, DRAM pages and TLB
// entries instead of being scattered over the whole F array by the generator's
// random relabelling. Claim order is unaffected (in-lists stay ascending by
// original id). Empty: keep the native order.
std::vector<uint32_t> degree_order(uint64_t V, const int64_t* tin) {
    const char* o = test_knob("GG_ORDER");
    if (o && !strcmp(o, "native")) return {};
    uint64_t maxd = 0;
    for (uint64_t v = 0; v < V; ++v) maxd = std::max<uint64_t>(maxd, (uint64_t)(tin[v + 1] - tin[v]));
    const double mean = (double)tin[V] / (double)std::max<uint64_t>(1, V);
    if (!(o && !strcmp(o, "degree")) && !((double)maxd > 16.0 * std::max(1.0, mean))) return {};
    std::vector<uint64_t> pos(maxd + 2, 0);  // counting sort, descending degree, stable in id
    for (uint64_t v = 0; v < V; ++v) pos[maxd - (uint64_t)(tin[v + 1] - tin[v]) + 1]++;
    for (uint64_t d = 0; d <= maxd; ++d) pos[d + 1] += pos[d];
    std::vector<uint32_t> order(V);
    for (uint64_t v = 0; v < V; ++v) order[pos[maxd - (uint64_t)(tin[v + 1] - tin[v])]++] = (uint32_t)v;
    return order;
}

}  // namespace

// ---------------------------------------------------------------------------

extern "C" {

int gg_abi_version(void) { return GG_ABI_VERSION; }

int gg_create(const gg_config* cfg, gg_engine** out) {
    if (!cfg || !out) return GG_EINVAL;
    *out = nullptr;
    if (cfg->n_nodes == 0 || cfg->n_nodes > 0x7fffffffull) return GG_EINVAL;
    if (cfg->n_lanes == 0 || cfg->n_lanes % 64 || cfg->n_lanes > 8192) return GG_EINVAL;
    if (cfg->enable_sync && cfg->sync_base_ticks == 0) return GG_EINVAL;
    if (cfg->world == 0 || cfg->rank >= cfg->world) return GG_EINVAL;
    const uint32_t L = cfg->lane_groups ? cfg->lane_groups : 1u;
    if (cfg->world % L || L > cfg->n_lanes / 64) return GG_EINVAL;
    // the exchange kernels keep one LDS slot per source part (unpack_ghosts) and
    // one lane per destination part (finish_pack, a 64-thread block)
    if (cfg->world / L > 63) return GG_EINVAL;
    if (cfg->batch_ticks && L != 1) return GG_EINVAL;  // batched gossip: vertex parts, no lane groups
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GG_EIO;
    auto* e = new gg_engine();
    e->cfg = *cfg;
    e->lanes.init(cfg->n_lanes);
    e->V = cfg->n_nodes;
    e->rank = cfg->rank;
    e->world = cfg->world;
    e->L = L;
    e->P = cfg->world / L;
    e->lgrp = cfg->rank / e->P;
    e->part = cfg->rank % e->P;
    e->nw_g = cfg->n_lanes / 64;
    e->w0 = e->nw_g * e->lgrp / L;
    e->nw = e->nw_g * (e->lgrp + 1) / L - e->w0;
    e->nwp = next_pow2((uint32_t)e->nw);
    if (cfg->device >= 0) {
        e->device = cfg->device;
        if (hipSetDevice(e->device) != hipSuccess) { delete e; return GG_EIO; }
    } else if (hipGetDevice(&e->device) != hipSuccess) {
        delete e;
        return GG_EIO;
    }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_counters, (size_t)kMaxBatch * (gg::kSlots + 1) * gg::kCounters * 8) != hipSuccess ||
        hipHostMalloc(&e->h_counters, (size_t)kMaxBatch * gg::kSlots * gg::kCounters * 8) != hipSuccess) {
        delete e;
        return GG_EIO;
    }
    *out = e;
    return GG_OK;
}

void gg_destroy(gg_engine* e) { delete e; }

const char* gg_last_error(const gg_engine* e) { return e ? e->err.c_str() : "null engine"; }

// In-/out-degree above which a node takes the hub path (GG_HUB_DEG overrides).
static uint32_t hub_threshold() {
    if (const char* h = test_knob("GG_HUB_DEG")) return (uint32_t)std::max(1, atoi(h));
    return 512;
}

// Component labels (gg::cc_*) of a symmetric CSR of n rows into d_lab: passes
// of pull-min (nodes of in-degree <= 256 one thread each; above, a hub chunk
// list when there is one, else a wave per node) and pointer jumping, until one
// changes nothing; *roots = the number of components.
static int cc_labels(gg_engine* e, const int64_t* d_ptr, const uint32_t* d_col, uint64_t n, uint32_t* d_lab,
                     unsigned long long* roots, const gg::HubChunk* chunks, uint64_t n_ch, uint32_t hub_deg) {
    uint32_t* d_ch = nullptr;
    HIPCHK(hipMalloc(&d_ch, 16));
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 16384);
    const uint32_t split = chunks ? hub_deg : 256u;
    hipLaunchKernelGGL(gg::cc_init, dim3(blocks), dim3(256), 0, e->stream, d_lab, n);
    int rc = GG_OK;
    for (int pass = 0;; ++pass) {
        uint32_t h = 0;
        if (hipMemsetAsync(d_ch, 0, 4, e->stream) != hipSuccess) { rc = GG_EIO; break; }
        hipLaunchKernelGGL(gg::cc_pass, dim3(blocks), dim3(256), 0, e->stream, d_ptr, d_col, d_lab, n, split, d_ch);
        if (chunks)
            hipLaunchKernelGGL(gg::cc_hubs, dim3((unsigned)std::min<uint64_t>(n_ch, 16384)), dim3(gg::kBlock), 0,
                               e->stream, chunks, n_ch, d_col, d_lab, d_ch);
        else
            hipLaunchKernelGGL(gg::cc_pass_wide, dim3(blocks), dim3(256), 0, e->stream, d_ptr, d_col, d_lab, n, split,
                               d_ch);
        for (int j = 0; j < 2; ++j)
            hipLaunchKernelGGL(gg::cc_jump, dim3(blocks), dim3(256), 0, e->stream, d_lab, n, d_ch);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&h, d_ch, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess) {
            rc = GG_EIO;
            break;
        }
        if (!h) break;
        if (pass > 100000) {
            rc = GG_EIO;
            break;
        }
    }
    if (rc == GG_OK) {
        unsigned long long* d_r = reinterpret_cast<unsigned long long*>(d_ch + 2);
        if (hipMemsetAsync(d_r, 0, 8, e->stream) != hipSuccess) rc = GG_EIO;
        hipLaunchKernelGGL(gg::cc_roots, dim3(blocks), dim3(256), 0, e->stream, d_lab, n, d_r);
        if (rc || hipMemcpyAsync(roots, d_r, 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            rc = GG_EIO;
    }
    (void)hipFree(d_ch);
    if (rc) e->err = "lean digest: component labels failed";
    return rc;
}

// The digest's per-component targets once labels are known (h_lab, d_llab set):
// the per-row targets and their table; ltab_sync fills them.
static int lsat_targets_alloc(gg_engine* e) {
    e->ltab_cap = std::max<uint32_t>(64, (uint32_t)std::min<uint64_t>(4ull * e->cfg.n_lanes, 1u << 20));
    HIPCHK(hipMalloc(&e->d_lreach, e->rows * 4));
    HIPCHK(hipMemsetAsync(e->d_lreach, 0, e->rows * 4, e->stream));
    HIPCHK(hipMalloc(&e->d_ltab, (1 + 2 * (size_t)e->ltab_cap) * 4));
    HIPCHK(hipMemsetAsync(e->d_ltab, 0, 4, e->stream));
    e->ltab_hash = 0;
    e->lret.clear();
    return GG_OK;
}

// Symmetric single engine: labels of its rows (its hub chunk list for the hubs).
// One component: no targets (lusat is every node's).
static int lsat_components(gg_engine* e) {
    const uint64_t n = e->n_own;
    HIPCHK(hipMalloc(&e->d_llab, n * 4));
    unsigned long long roots = 0;
    if (int rc = cc_labels(e, e->d_in_ptr, e->d_in_col, n, e->d_llab, &roots, e->n_hubs ? e->d_hchunks : nullptr,
                           e->n_hchunks, e->hub_deg))
        return rc;
    if (roots <= 1) {
        dfree(e->d_llab);
        return GG_OK;
    }
    e->h_lab.resize(n);
    HIPCHK(hipMemcpy(e->h_lab.data(), e->d_llab, n * 4, hipMemcpyDeviceToHost));
    e->lab_global = false;
    return lsat_targets_alloc(e);
}

// Hubs, per-node state and the episode reset after the in-lists are on the
// device. iptr/optr: host copies of the in-/out-list pointers (optr null:
// symmetric, out-lists = in-lists); iptr null: the caller has checked that no
// node's degree exceeds the hub threshold.
static int finish_topology(gg_engine* e, const int64_t* iptr, const int64_t* optr) {
    const uint64_t n_own = e->n_own;
    // hubs: in-degree > hub_deg (hub_chunks/hub_finish in lean rounds), senders
    // with out-degree > hub_deg (hub_mark)
    e->hub_deg = 0;
    {
        e->hub_deg = hub_threshold();
        uint64_t per = 128ull * (gg::kBlock / lanes_per_node((uint32_t)e->nwp));  // senders per chunk
        if (const char* h = test_knob("GG_HUB_CHUNK")) per = (uint64_t)std::max(1, atoi(h));
        std::vector<uint32_t> hubs, hub_c0;
        std::vector<gg::HubChunk> hch, mch;
        for (uint64_t i = 0; iptr && i < n_own; ++i) {
            const int64_t din = iptr[i + 1] - iptr[i];
            if (din > (int64_t)e->hub_deg) {
                hubs.push_back((uint32_t)i);
                hub_c0.push_back((uint32_t)hch.size());
                for (int64_t x = iptr[i]; x < iptr[i + 1]; x += (int64_t)per)
                    hch.push_back({(uint32_t)i, (uint32_t)std::min<int64_t>((int64_t)per, iptr[i + 1] - x), x});
            }
            const int64_t o0 = optr ? optr[i] : iptr[i], o1 = optr ? optr[i + 1] : iptr[i + 1];
            if (o1 - o0 > (int64_t)e->hub_deg)
                for (int64_t x = o0; x < o1; x += 1024)
                    mch.push_back({(uint32_t)i, (uint32_t)std::min<int64_t>(1024, o1 - x), x});
        }
        hub_c0.push_back((uint32_t)hch.size());
        e->n_hubs = hubs.size();
        e->n_hchunks = hch.size();
        e->n_mchunks = mch.size();
        if (e->n_hubs) {
            HIPCHK(hipMalloc(&e->d_hubs, hubs.size() * 4));
            HIPCHK(hipMemcpy(e->d_hubs, hubs.data(), hubs.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMalloc(&e->d_hub_c0, hub_c0.size() * 4));
            HIPCHK(hipMemcpy(e->d_hub_c0, hub_c0.data(), hub_c0.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMalloc(&e->d_hchunks, hch.size() * sizeof(gg::HubChunk)));
            HIPCHK(hipMemcpy(e->d_hchunks, hch.data(), hch.size() * sizeof(gg::HubChunk), hipMemcpyHostToDevice));
            // streamed sync rounds (symmetric, sync on): a third row per chunk (hub_sync_*)
            const bool hsync = e->cfg.enable_sync && e->symmetric;
            HIPCHK(hipMalloc(&e->d_hscratch, hch.size() * (hsync ? 3 : 2) * e->nwp * 8));
            if (hsync) {
                HIPCHK(hipMalloc(&e->d_hflag, hch.size() * 4));
                HIPCHK(hipMalloc(&e->d_hlive, (hubs.size() + 7) / 8 * 8));
            }
        }
        if (e->n_mchunks) {
            HIPCHK(hipMalloc(&e->d_mchunks, mch.size() * sizeof(gg::HubChunk)));
            HIPCHK(hipMemcpy(e->d_mchunks, mch.data(), mch.size() * sizeof(gg::HubChunk), hipMemcpyHostToDevice));
        }
    }
    // streamed sync rounds: any row width (W = 64: one word per node, one lane);
    // hubs on symmetric topologies only (hub_sync_*: a hub's in-list is its out-list)
    e->sync_tiles = test_knob("GG_SYNC_TILES") && atoi(test_knob("GG_SYNC_TILES")) != 0;
    dfree(e->d_srec);
    dfree(e->d_pushb);
    dfree(e->d_rev);
    dfree(e->d_sstate);
    dfree(e->d_ibits);
    dfree(e->d_sat);
    dfree(e->d_sat_new);
    dfree(e->d_lsat);
    dfree(e->d_llab);
    dfree(e->d_lreach);
    dfree(e->d_ltab);
    e->h_lab.clear();
    e->h_lab.shrink_to_fit();
    e->lret.clear();
    e->ltab_hash = 0;
    dfree(e->d_pushany);
    dfree(e->d_nmeta);
    dfree(e->d_pend);
    dfree(e->d_pend_src);
    for (int b = 0; b < 2; ++b) dfree(e->d_bset[b]);
    if (e->cfg.batch_ticks) {
        HIPCHK(hipMalloc(&e->d_pend, e->rows * e->nwp * 8));
        HIPCHK(hipMalloc(&e->d_pend_src, e->rows * 4));
        if (e->cfg.enable_sync)  // every node writes its set of round r into d_bset[r & 1]
            for (int b = 0; b < 2; ++b) {
                HIPCHK(hipMalloc(&e->d_bset[b], e->rows * e->nwp * 8));
                HIPCHK(hipMemset(e->d_bset[b], 0, e->rows * e->nwp * 8));
            }
    }
    // the streamed-sync buffers: before the first round that reaches a timer
    // (ensure_sync), not here; GG_SYNC_EAGER=1 allocates them with the topology
    e->sync_alloc = false;
    e->no_mark = test_knob("GG_NO_MARK") && atoi(test_knob("GG_NO_MARK"));
    const size_t rowbytes = e->rows * e->nwp * 8;
    e->tile_nodes = gg::kBlock / lanes_per_node((uint32_t)e->nwp);
    const uint64_t ntiles = (n_own + e->tile_nodes - 1) / e->tile_nodes;
    e->tile_bytes = (ntiles + 8) / 8 * 8;
    HIPCHK(hipMalloc(&e->d_cand, 2 * e->rows));
    HIPCHK(hipMalloc(&e->d_zmark, e->rows));
    HIPCHK(hipMalloc(&e->d_tile_cand, e->tile_bytes));
    HIPCHK(hipMalloc(&e->d_work, std::max<uint64_t>(1, ntiles) * sizeof(gg::TileWork)));
    HIPCHK(hipMalloc(&e->d_n_work, 4 * sizeof(uint32_t)));
    e->prep_cap = test_knob("GG_PREP_BLOCKS") ? (uint64_t)std::max(1, atoi(test_knob("GG_PREP_BLOCKS"))) : 1024;
    {  // split compaction when one atomic per block would serialise (compact_round)
        const uint64_t per_block = (uint64_t)gg::kBlock * gg::kCompactQ;
        const uint64_t nb = ((n_own + 7) / 8 + per_block - 1) / per_block;
        if ((nb > gg::kCompactSplit || test_knob("GG_COMPACT_SPLIT")) && !test_knob("GG_COMPACT_ATOMIC"))
            HIPCHK(hipMalloc(&e->d_bcount, (nb + 1) * sizeof(uint32_t)));
    }
    HIPCHK(hipMalloc(&e->d_nodes, std::max<uint64_t>(1, n_own) * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&e->d_act, 4 * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&e->d_act_deg, 4 * 8));
    HIPCHK(hipMalloc(&e->d_tot, 4 * 8));
    HIPCHK(hipMalloc(&e->d_act_s, 4 * gg::kSlots * 4));
    HIPCHK(hipMalloc(&e->d_act_deg_s, 4 * gg::kSlots * 8));
    HIPCHK(hipMalloc(&e->d_tot_s, 4 * gg::kSlots * 8));
    // flags-first gathers (ff_round): rows of >= 64 B (the request-rate-bound
    // regime) or of 8 B (expand_stream1: every gather a random 8-byte request,
    // the bitmap 1/64 of the F words) and a mean in-degree >= 4;
    // GG_FLAGS_FIRST=0/1 overrides, GG_FF_FRAC16 sets the threshold (A/B)
    {
        const char* f = ab_knob("GG_FLAGS_FIRST");
        e->ff_ok = f ? atoi(f) != 0
                     : ((e->nwp >= 8 || e->nwp == 1) && e->n_in_edges >= 4 * std::max<uint64_t>(1, n_own));
        const char* q = ab_knob("GG_FF_FRAC16");
        e->ff_frac16 = q ? (uint32_t)std::max(1, atoi(q)) : 8u;
        if (e->ff_ok) HIPCHK(hipMalloc(&e->d_abits, e->rows / 8));
    }
    // lean-round saturation digest (RoundArgs::lsat; W >= 128) on graphs with hubs:
    // there the hubs — most of the in-edges — saturate rounds before the last
    // delivery round (C4 1190 -> 840 ms/step); on a tree nodes saturate only in
    // the last delivery rounds and the marking costs more than the skips save
    // (C2 +1 %, profiles/r5/INDEX.md). Vertex parts hold no whole component, so
    // their targets would be every lane, which a disconnected graph never reaches:
    // off there too. GG_LSAT=1 / 0 forces it on / off.
    const char* lk = test_knob("GG_LSAT");
    const bool whole = e->symmetric && e->P <= 1 && e->n_ghost == 0;
    if (e->nwp >= 2 && (lk ? atoi(lk) != 0 : (e->n_hubs > 0 && whole))) {
        HIPCHK(hipMalloc(&e->d_lsat, e->rows));
        HIPCHK(hipMemsetAsync(e->d_lsat, 0, e->rows, e->stream));
        // targets per component when there are several (a node never holds a lane
        // injected outside its component: R-MAT's isolated nodes and small
        // components keep every node of the giant one below "every lane")
        if (whole && n_own > 1)
            if (int rc = lsat_components(e)) return rc;
    }
    HIPCHK(hipMalloc(&e->d_base, rowbytes));
    e->d_sets[0] = e->d_base;
    e->set_cur = 0;
    // double-buffered lean rounds: decided at the first step (ensure_db), when
    // the generator's scratch is gone
    e->db_ok = false;
    e->db_decided = false;
    e->f_dirty = true;
    for (int b = 0; b < 2; ++b) {
        HIPCHK(hipMalloc(&e->d_F[b], rowbytes));
        HIPCHK(hipMalloc(&e->d_flg[b], e->rows));
    }
    for (int b = 0; b < 4; ++b) HIPCHK(hipMalloc(&e->d_fired[b], e->rows / 8));
    HIPCHK(hipMalloc(&e->d_sync_next, e->rows * 4));  // owned nodes' and ghosts' timers
    HIPCHK(hipMalloc(&e->d_sync_k, e->rows * 4));
    if (e->cfg.flags & GG_TRACK_DELIVERY) HIPCHK(hipMalloc(&e->d_dr, std::max<uint64_t>(1, n_own) * e->nw * 64 * 4));
    e->have_topo = true;
    e->quiet = 0;  // fresh buffers: clear everything
    e->dist_k = 0;
    e->dist_done.clear();
    e->inj_off = 0;
    e->lanes.clear();
    e->lane_value.clear();
    e->inj.clear();
    e->inj_rounds.clear();
    e->round = 0;
    e->pend_acks = e->pend_ackdrop = 0;
    e->hash_total = 0;
    e->dist_open = false;
    e->u_hist.clear();
    e->u_bits.clear();
    e->lret.clear();
    if (test_knob("GG_SYNC_EAGER") && atoi(test_knob("GG_SYNC_EAGER"))) {
        const int rc = alloc_sync(e);
        if (rc) return rc;
    }
    return reset_device_state(e);
}

// Exchange buffers of a vertex-sharded engine from its send/receive lists
// (send_off, recv_off, n_ghost; d_send_idx, d_gout_* already on the device):
// segment capacities (header + an F and an S entry per send-list node), pack
// tiles, the size mode of every direction.
static int setup_exchange(gg_engine* e) {
    const uint32_t Wd = e->P;
    e->xstride = (uint32_t)(e->nwp >= 2 ? 16 + 8 * e->nwp : 16);
    e->xsoff.assign(Wd + 1, 0);
    e->xroff.assign(Wd + 1, 0);
    std::vector<gg::XchgTile> tiles;
    // a segment holds either layout (expand_kernels.hpp: entries with heads, or the
    // device-driven exchange's tile records + rows)
    auto cap = [&](uint64_t n) -> uint64_t {
        return n ? std::max<uint64_t>(16 + 2 * n * e->xstride, gg::tile_rows_off(n) + 2 * n * 8 * e->nwp) : 0;
    };
    // a region also holds three need slots (IPC exchange: one bit per entry of the
    // opposite direction, rotating by seq % 3) when both directions carry entries
    auto need = [&](uint64_t n_this, uint64_t n_back) -> uint64_t {
        return (n_this && n_back) ? 3 * gg::need_slot_bytes(n_back) : 0;
    };
    std::vector<uint64_t> need_in(Wd, 0), need_out(Wd, 0), need_bytes(2 * Wd, 0);
    std::vector<gg::NeedWord> words;
    for (uint32_t q = 0; q < Wd; ++q) {
        const uint64_t ns = e->send_off[q + 1] - e->send_off[q], nr = e->recv_off[q + 1] - e->recv_off[q];
        if (ns && nr) {
            // our region in q's window (we send ns entries, q sends us nr: our bits cover q's nr)
            need_out[q] = cap(ns);
            need_bytes[q] = gg::need_slot_bytes(nr);
            // q's region in ours (q sends nr, we send ns: q's bits cover our ns entries to q)
            need_in[q] = gg::kWinHdr + e->xroff[q] + cap(nr);
            need_bytes[Wd + q] = gg::need_slot_bytes(ns);
            for (uint64_t j = 0; j < nr; j += 64)
                words.push_back({q, (uint32_t)j, (uint32_t)std::min<uint64_t>(64, nr - j)});
        }
        e->xsoff[q + 1] = e->xsoff[q] + cap(ns) + need(ns, nr);
        e->xroff[q + 1] = e->xroff[q] + cap(nr) + need(nr, ns);
        for (uint64_t k0 = e->send_off[q]; k0 < e->send_off[q + 1]; k0 += gg::kBlock)
            tiles.push_back({q, (uint32_t)k0, (uint32_t)std::min<uint64_t>(gg::kBlock, e->send_off[q + 1] - k0),
                             (uint32_t)e->send_off[q]});
    }
    HIPCHK(hipMalloc(&e->d_need_in, Wd * 8));
    HIPCHK(hipMemcpy(e->d_need_in, need_in.data(), Wd * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_need_out, Wd * 8));
    HIPCHK(hipMemcpy(e->d_need_out, need_out.data(), Wd * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_need_bytes, 2 * Wd * 8));
    HIPCHK(hipMemcpy(e->d_need_bytes, need_bytes.data(), 2 * Wd * 8, hipMemcpyHostToDevice));
    e->n_need_words = (uint32_t)words.size();
    HIPCHK(hipMalloc(&e->d_need_words, std::max<size_t>(1, words.size()) * sizeof(gg::NeedWord)));
    if (!words.empty())
        HIPCHK(hipMemcpy(e->d_need_words, words.data(), words.size() * sizeof(gg::NeedWord), hipMemcpyHostToDevice));
    e->n_xtiles = (uint32_t)tiles.size();
    HIPCHK(hipMalloc(&e->d_xtiles, std::max<size_t>(1, tiles.size()) * sizeof(gg::XchgTile)));
    if (!tiles.empty())
        HIPCHK(hipMemcpy(e->d_xtiles, tiles.data(), tiles.size() * sizeof(gg::XchgTile), hipMemcpyHostToDevice));
    std::vector<uint32_t> gfirst(Wd + 1);
    for (uint32_t q = 0; q <= Wd; ++q) gfirst[q] = (uint32_t)e->recv_off[q];
    HIPCHK(hipMalloc(&e->d_gfirst, (Wd + 1) * 4));
    HIPCHK(hipMemcpy(e->d_gfirst, gfirst.data(), (Wd + 1) * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_xsoff, (Wd + 1) * 8));
    HIPCHK(hipMemcpy(e->d_xsoff, e->xsoff.data(), (Wd + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_xroff, (Wd + 1) * 8));
    HIPCHK(hipMemcpy(e->d_xroff, e->xroff.data(), (Wd + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_needmark, (e->send_off[Wd] + 7) / 8 * 8 + 8));
    HIPCHK(hipMalloc(&e->d_stamp, (e->n_ghost + 1) / 2 * 8 + 8));
    HIPCHK(hipMalloc(&e->d_xcnt, 2 * Wd * 4 + 8));  // rows (entries) per peer, then tile records per peer
    {
        std::vector<uint32_t> sf(Wd + 1);
        for (uint32_t q = 0; q <= Wd; ++q) sf[q] = (uint32_t)e->send_off[q];
        HIPCHK(hipMalloc(&e->d_sfirst, (Wd + 1) * 4));
        HIPCHK(hipMemcpy(e->d_sfirst, sf.data(), (Wd + 1) * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc(&e->d_xtk, 16));
    HIPCHK(hipMemset(e->d_xtk, 0, 16));
    HIPCHK(hipMalloc(&e->d_segbytes, 2 * Wd * 8));
    HIPCHK(hipHostMalloc(&e->h_segbytes, 2 * Wd * 8));
    HIPCHK(hipMalloc(&e->d_payload, kMaxBatch * 8));
    HIPCHK(hipMalloc(&e->d_xsend, std::max<uint64_t>(16, e->xsoff[Wd])));
    HIPCHK(hipMalloc(&e->d_xrecv, std::max<uint64_t>(16, e->xroff[Wd])));
    // a direction whose static capacity exceeds GG_XCHG_EXACT_BYTES (default
    // 4 MiB) sends its exact size first and then only the used bytes (one host
    // wait per round); GG_XCHG_MODE=exact|static forces every direction
    const char* mode = test_knob("GG_XCHG_MODE");
    uint64_t lim = 4ull << 20;
    if (const char* l = ab_knob("GG_XCHG_EXACT_BYTES")) lim = strtoull(l, nullptr, 10);
    e->xexact_s.assign(Wd, 0);
    e->xexact_r.assign(Wd, 0);
    e->xexact = false;
    for (uint32_t q = 0; q < Wd; ++q) {
        const uint64_t cs = e->xsoff[q + 1] - e->xsoff[q], cr = e->xroff[q + 1] - e->xroff[q];
        const bool force = mode && !strcmp(mode, "exact"), never = mode && !strcmp(mode, "static");
        e->xexact_s[q] = cs && !never && (force || cs > lim);
        e->xexact_r[q] = cr && !never && (force || cr > lim);
        e->xexact |= e->xexact_s[q] || e->xexact_r[q];
    }
    return GG_OK;
}

int gg_topology(gg_engine* e, const int64_t* row_ptr, const int32_t* col, uint64_t nnz) {
    if (!e || !row_ptr || (nnz && !col)) return GG_EINVAL;
    HIPCHK(hipSetDevice(e->device));
    const uint64_t V = e->V;
    if (row_ptr[0] != 0 || (uint64_t)row_ptr[V] != nnz) return e->fail(GG_EINVAL, "row_ptr[0]/row_ptr[V] mismatch");
    {
        std::atomic<int> bad{0};  // 1 monotone, 2 range, 3 order
        host_parallel(V, [&](uint64_t lo, uint64_t hi) {
            for (uint64_t v = lo; v < hi && !bad.load(std::memory_order_relaxed); ++v) {
                if (row_ptr[v + 1] < row_ptr[v]) { bad = 1; return; }
                for (int64_t k = row_ptr[v]; k < row_ptr[v + 1]; ++k) {
                    if (col[k] < 0 || (uint64_t)col[k] >= V) { bad = 2; return; }
                    if (k > row_ptr[v] && col[k] <= col[k - 1]) { bad = 3; return; }
                }
            }
        });
        if (bad == 1) return e->fail(GG_EINVAL, "row_ptr not monotone");
        if (bad == 2) return e->fail(GG_EINVAL, "neighbour id out of range");
        if (bad == 3) return e->fail(GG_EINVAL, "neighbour list not ascending/unique");
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    e->free_topology();
    if (e->P > 1) e->host_rp.assign(row_ptr, row_ptr + V + 1);
    else e->host_rp.clear();
    // per-edge windows are in the old topology's edge order
    e->windows.erase(std::remove_if(e->windows.begin(), e->windows.end(), [](const Window& w) { return w.edges; }),
                     e->windows.end());
    // symmetric (u lists v iff v lists u)? then the in-lists are the rows themselves
    bool sym = true;
    {
        std::atomic<bool> asym{false};
        host_parallel(V, [&](uint64_t lo, uint64_t hi) {
            for (uint64_t u = lo; u < hi && !asym.load(std::memory_order_relaxed); ++u)
                for (int64_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) {
                    const uint32_t v = (uint32_t)col[k];
                    if (!std::binary_search(col + row_ptr[v], col + row_ptr[v + 1], (int32_t)u)) {
                        asym = true;
                        return;
                    }
                }
        });
        sym = !asym.load();
    }
    e->symmetric = sym;
    // transpose (directed lists only): in-lists ascending by sender
    std::vector<int64_t> tin_v;
    std::vector<uint32_t> tcol_v;
    const int64_t* tin = row_ptr;
    const uint32_t* tcol = reinterpret_cast<const uint32_t*>(col);
    if (!sym) {
        tin_v.assign(V + 1, 0);
        for (uint64_t k = 0; k < nnz; ++k) tin_v[col[k] + 1]++;
        for (uint64_t v = 0; v < V; ++v) tin_v[v + 1] += tin_v[v];
        tcol_v.resize(nnz);
        std::vector<int64_t> pos(tin_v.begin(), tin_v.end() - 1);
        for (uint64_t u = 0; u < V; ++u)
            for (int64_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) tcol_v[pos[col[k]]++] = (uint32_t)u;
        tin = tin_v.data();
        tcol = tcol_v.data();
    }
    // ---- partition (sharded): a locality order of the nodes cut into
    // edge-balanced contiguous ranges; rank p owns order[plo[p] .. plo[p+1])
    const uint32_t Wd = e->P;  // vertex parts of this engine's lane group
    std::vector<uint32_t> order;    // position -> node (empty: identity)
    std::vector<uint64_t> plo;      // [Wd+1] position ranges
    std::vector<uint32_t> owner;    // node -> rank (sharded)
    if (Wd > 1) {
        choose_partition(V, row_ptr, col, tin, Wd, order, plo, owner);
    } else {
        plo = {0, V};
        order = degree_order(V, tin);
    }
    const bool perm = Wd > 1 || !order.empty();  // local rows != node ids
    auto node_at = [&](uint64_t pos) -> uint32_t { return order.empty() ? (uint32_t)pos : order[pos]; };
    const uint64_t n_own = plo[e->part + 1] - plo[e->part];
    e->n_own = n_own;
    e->loc_of.clear();
    e->gid.clear();
    e->range_mode = false;
    std::vector<uint32_t> ghosts;                     // ghost nodes in local ghost order
    std::vector<std::vector<uint32_t>> sendl(Wd);     // owned local rows per destination
    std::vector<std::vector<uint32_t>> send_ids(Wd);  // the same, original ids (ascending)
    e->send_off.assign(Wd + 1, 0);
    e->recv_off.assign(Wd + 1, 0);
    if (perm) {
        e->loc_of.assign(V, ~0u);
        for (uint64_t i = 0; i < n_own; ++i) e->loc_of[node_at(plo[e->part] + i)] = (uint32_t)i;
    }
    if (Wd > 1) {
        // ghosts: remote nodes adjacent (in or out) to owned ones; send lists:
        // owned nodes adjacent to each remote rank. Both sorted by node id, so
        // rank q's receive order from p equals p's send order to q.
        std::vector<std::vector<uint32_t>> gfrom(Wd);
        std::vector<uint32_t> peers;
        for (uint64_t i = 0; i < n_own; ++i) {
            const uint32_t v = node_at(plo[e->part] + i);
            peers.clear();
            auto visit = [&](uint32_t u) {
                const uint32_t q = owner[u];
                if (q == e->part) return;
                gfrom[q].push_back(u);
                peers.push_back(q);
            };
            for (int64_t k = row_ptr[v]; k < row_ptr[v + 1]; ++k) visit((uint32_t)col[k]);
            for (int64_t k = tin[v]; k < tin[v + 1]; ++k) visit(tcol[k]);
            std::sort(peers.begin(), peers.end());
            peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
            for (uint32_t q : peers) sendl[q].push_back(v);
        }
        for (uint32_t q = 0; q < Wd; ++q) {
            auto& g = gfrom[q];
            std::sort(g.begin(), g.end());
            g.erase(std::unique(g.begin(), g.end()), g.end());
            std::sort(sendl[q].begin(), sendl[q].end());
            send_ids[q] = sendl[q];
            for (auto& v : sendl[q]) v = e->loc_of[v];  // node -> owned local row
            ghosts.insert(ghosts.end(), g.begin(), g.end());
            e->recv_off[q + 1] = e->recv_off[q] + g.size();
            e->send_off[q + 1] = e->send_off[q] + sendl[q].size();
        }
    }
    e->n_ghost = ghosts.size();
    e->ghost0 = Wd > 1 ? (n_own + 63) / 64 * 64 : n_own;
    e->rows = std::max<uint64_t>(64, (e->ghost0 + e->n_ghost + 63) / 64 * 64);
    if (e->rows > 0x7fffffffull) return e->fail(GG_EINVAL, "local rows exceed 2^31");
    if (perm) {
        e->gid.assign(e->rows, ~0u);
        for (uint64_t i = 0; i < n_own; ++i) e->gid[i] = node_at(plo[e->part] + i);
        for (uint64_t k = 0; k < ghosts.size(); ++k) e->gid[e->ghost0 + k] = ghosts[k];
    }
    // local row of a node: owned, or a ghost (the ghosts from part q are ascending
    // ids at ghost0 + recv_off[q]); read-only lookups, so rows build in parallel
    auto row_of = [&](uint32_t u) -> uint32_t {
        if (!perm) return u;
        const uint32_t l = e->loc_of[u];
        if (l != ~0u) return l;
        const uint32_t q = owner[u];
        const uint32_t* g0 = ghosts.data() + e->recv_off[q];
        const uint32_t* g1 = ghosts.data() + e->recv_off[q + 1];
        return (uint32_t)(e->ghost0 + e->recv_off[q] + (std::lower_bound(g0, g1, u) - g0));
    };
    // ---- owned rows: in-lists (ascending sender id: claim order) and out-lists
    // (ascending receiver id: callback order) with local-row columns
    std::vector<int64_t> iptr(n_own + 1, 0), optr(n_own + 1, 0);
    for (uint64_t i = 0; i < n_own; ++i) {
        const uint32_t v = node_at(plo[e->part] + i);
        iptr[i + 1] = iptr[i] + (tin[v + 1] - tin[v]);
        optr[i + 1] = optr[i] + (row_ptr[v + 1] - row_ptr[v]);
    }
    std::vector<uint32_t> icol(iptr[n_own]), ocol(sym ? 0 : optr[n_own]);
    std::vector<int64_t> gcnt(e->n_ghost + 1, 0);
    auto build_rows = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) {
            const uint32_t v = node_at(plo[e->part] + i);
            const int32_t* ob = col + row_ptr[v];
            const int32_t* oe = col + row_ptr[v + 1];
            for (int64_t k = 0; k < tin[v + 1] - tin[v]; ++k) {
                const uint32_t u = tcol[tin[v] + k];
                const bool recip = sym || std::binary_search(ob, oe, (int32_t)u);
                icol[iptr[i] + k] = row_of(u) | (recip ? gg::kRecipBit : 0u);
            }
            if (!sym)
                for (int64_t k = 0; k < row_ptr[v + 1] - row_ptr[v]; ++k) ocol[optr[i] + k] = row_of((uint32_t)ob[k]);
        }
    };
    host_parallel(n_own, build_rows);
    for (uint64_t k = 0; k < icol.size() && e->n_ghost; ++k) {
        const uint32_t ru = icol[k] & gg::kColMask;
        if (ru >= e->ghost0) gcnt[ru - e->ghost0 + 1]++;
    }
    // ghost -> owned receivers (candidate marking from remote senders)
    std::vector<uint32_t> gocol;
    if (e->n_ghost) {
        for (uint64_t g = 0; g < e->n_ghost; ++g) gcnt[g + 1] += gcnt[g];
        gocol.resize(gcnt[e->n_ghost]);
        std::vector<int64_t> fill(gcnt.begin(), gcnt.end() - 1);
        for (uint64_t i = 0; i < n_own; ++i)
            for (int64_t k = iptr[i]; k < iptr[i + 1]; ++k) {
                const uint32_t ru = icol[k] & gg::kColMask;
                if (ru >= e->ghost0) gocol[fill[ru - e->ghost0]++] = (uint32_t)i;
            }
    }
    // device buffers
    e->n_in_edges = icol.size();
    e->n_out_edges = sym ? icol.size() : ocol.size();
    HIPCHK(hipMalloc(&e->d_in_ptr, (n_own + 1) * 8));
    HIPCHK(hipMalloc(&e->d_in_col, std::max<size_t>(1, icol.size()) * 4));
    HIPCHK(hipMemcpy(e->d_in_ptr, iptr.data(), (n_own + 1) * 8, hipMemcpyHostToDevice));
    if (!icol.empty()) HIPCHK(hipMemcpy(e->d_in_col, icol.data(), icol.size() * 4, hipMemcpyHostToDevice));
    if (sym) {
        // out-lists equal in-lists; readers of out_col mask off the recip bit
        e->d_out_ptr = e->d_in_ptr;
        e->d_out_col = e->d_in_col;
    } else {
        HIPCHK(hipMalloc(&e->d_out_ptr, (n_own + 1) * 8));
        HIPCHK(hipMalloc(&e->d_out_col, std::max<size_t>(1, ocol.size()) * 4));
        HIPCHK(hipMemcpy(e->d_out_ptr, optr.data(), (n_own + 1) * 8, hipMemcpyHostToDevice));
        if (!ocol.empty()) HIPCHK(hipMemcpy(e->d_out_col, ocol.data(), ocol.size() * 4, hipMemcpyHostToDevice));
    }
    if (perm) {
        HIPCHK(hipMalloc(&e->d_gid, e->rows * 4));
        HIPCHK(hipMemcpy(e->d_gid, e->gid.data(), e->rows * 4, hipMemcpyHostToDevice));
    }
    if (Wd > 1) {
        std::vector<uint32_t> sidx;
        for (uint32_t q = 0; q < Wd; ++q) sidx.insert(sidx.end(), sendl[q].begin(), sendl[q].end());
        HIPCHK(hipMalloc(&e->d_send_idx, std::max<size_t>(1, sidx.size()) * 4));
        if (!sidx.empty()) HIPCHK(hipMemcpy(e->d_send_idx, sidx.data(), sidx.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&e->d_gout_ptr, (e->n_ghost + 1) * 8));
        HIPCHK(hipMemcpy(e->d_gout_ptr, gcnt.data(), (e->n_ghost + 1) * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&e->d_gout_col, std::max<size_t>(1, gocol.size()) * 4));
        if (!gocol.empty())
            HIPCHK(hipMemcpy(e->d_gout_col, gocol.data(), gocol.size() * 4, hipMemcpyHostToDevice));
        // filtered exchange: the send entry of every ghost -> owned edge (the
        // owned node's position in the send list to the ghost's part), pack tiles,
        // segment capacities (header + an F and an S entry per send-list node)
        std::vector<uint32_t> gsidx(gocol.size());
        {
            uint32_t p = 0;
            for (uint64_t g = 0; g < e->n_ghost; ++g) {
                while (g >= e->recv_off[p + 1]) ++p;
                const auto& ids = send_ids[p];
                for (int64_t k = gcnt[g]; k < gcnt[g + 1]; ++k) {
                    const uint32_t id = e->gid[gocol[k]];
                    const auto it = std::lower_bound(ids.begin(), ids.end(), id);
                    if (it == ids.end() || *it != id) return e->fail(GG_EIO, "internal: ghost edge without a send entry");
                    gsidx[k] = (uint32_t)(e->send_off[p] + (it - ids.begin()));
                }
            }
        }
        HIPCHK(hipMalloc(&e->d_gout_sidx, std::max<size_t>(1, gsidx.size()) * 4));
        if (!gsidx.empty())
            HIPCHK(hipMemcpy(e->d_gout_sidx, gsidx.data(), gsidx.size() * 4, hipMemcpyHostToDevice));
        if (int rc = setup_exchange(e)) return rc;
    }
    return finish_topology(e, iptr.data(), sym ? nullptr : optr.data());
}

// gossip_gen.h: the spec's graph built in HBM (csrc/generate.hip) and installed
// as gg_topology would install the host builder's CSR. Single engine:
// symmetric, so the in-lists are the rows themselves with every entry
// reciprocal and nothing crosses PCIe. Sharded: built on the device, then the
// host partition path of gg_topology.
}  // extern "C"

// gg_topology_generate on a vertex-sharded engine: rank part of P owns the
// contiguous node range [plo[part], plo[part+1]) (native order, cut at
// multiples of 64) and builds only those rows of the generated graph, then
// its ghosts, send lists and ghost -> owned lists on the device
// (gg_gen::shard_csr): no rank holds the whole graph, in HBM or in host
// memory (host memory: the rank's ghost ids and per-part offsets only).
static int install_shard(gg_engine* e, gg_gen::Csr g, const std::vector<uint64_t>& plo, uint64_t* nnz_out);

// The lean digest on the vertex parts of a generated graph (hub graphs by
// default, GG_LSAT as for single engines): a component spans parts, so its
// labels come from the whole graph, built on this device in original ids and
// dropped after labelling; the labels stay on the host (the broadcasts'
// counts per component, ltab_sync) and the owned rows' on the device. They are
// built BEFORE the part allocates anything (lab_prepare, at the start of
// generate_sharded), so the whole-graph build meets the same free HBM at every
// N — two C4 lane halves at N = 2 once found none beside their parts — and
// kept per generator spec for the process: a second engine of the same graph
// (lane halves) takes them from the cache. A build that fails anyway is cached
// as a failure with its reason: the part then runs the digest against "every
// lane" (exact, no skips on a disconnected graph), its rounds report
// GG_PATH_LSAT without GG_PATH_LSAT_COMP, and the reason goes to stderr.
// GG_LSAT_LABELS_FAIL=1 forces that failure (test hook).
struct LabEntry {
    std::shared_ptr<const std::vector<uint32_t>> labs;  // empty vector: one component
    std::string fail;                                    // non-empty: the build failed
};
static std::mutex g_lab_mu;
static std::map<std::vector<uint64_t>, LabEntry> g_lab_cache;

static std::vector<uint64_t> lab_key(const gg_gen_spec* spec) {
    uint64_t ab[3];
    std::memcpy(ab, &spec->a, 8);
    std::memcpy(ab + 1, &spec->b, 8);
    std::memcpy(ab + 2, &spec->c, 8);
    return {spec->kind, spec->k, spec->n, spec->seed, ab[0], ab[1], ab[2]};
}

static bool lsat_wanted(const gg_engine* e, bool hubs_known) {
    const char* lk = test_knob("GG_LSAT");
    if (lk) return atoi(lk) != 0 && e->nwp >= 2;
    return e->nwp >= 2 && (!hubs_known || e->n_hubs > 0);  // before the install: hubs unknown, prepare anyway
}

// The whole graph's component labels into the cache (once per spec and process).
static void lab_prepare(gg_engine* e, const gg_gen_spec* spec) {
    if (!lsat_wanted(e, false) || spec->kind == GG_GEN_TREE) return;  // (a tree is connected)
    const auto key = lab_key(spec);
    {
        std::lock_guard<std::mutex> lk(g_lab_mu);
        if (g_lab_cache.count(key)) return;
    }
    LabEntry ent;
    gg_gen::Csr g{};
    std::string err;
    unsigned long long roots = 0;
    uint32_t* d_lab = nullptr;
    int rc = test_knob("GG_LSAT_LABELS_FAIL") ? GG_EIO : GG_OK;
    if (rc) err = "GG_LSAT_LABELS_FAIL";
    if (rc == GG_OK) rc = gg_gen::build_csr(*spec, e->stream, 0u, &g, &err);
    if (rc == GG_OK && hipMalloc(&d_lab, e->V * 4) != hipSuccess) rc = GG_EIO, err = "labels: hipMalloc";
    if (rc == GG_OK) {
        rc = cc_labels(e, g.row_ptr, g.col, e->V, d_lab, &roots, nullptr, 0, 0);
        if (rc) err = "cc_labels: " + e->err;
    }
    (void)hipFree(g.row_ptr);
    (void)hipFree(g.col);
    auto h = std::make_shared<std::vector<uint32_t>>();
    if (rc == GG_OK && roots > 1) {
        h->resize(e->V);
        if (hipMemcpy(h->data(), d_lab, e->V * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = GG_EIO, err = "labels: copy to host";
    }
    (void)hipFree(d_lab);
    (void)hipGetLastError();
    (void)hipStreamSynchronize(e->stream);
    e->err.clear();
    if (rc == GG_OK) {
        ent.labs = h;
    } else {
        ent.fail = err.empty() ? "whole-graph build failed" : err;
    }
    std::lock_guard<std::mutex> lk(g_lab_mu);
    if (g_lab_cache.size() > 4) g_lab_cache.clear();
    g_lab_cache[key] = ent;
}

static int lsat_parts(gg_engine* e, const gg_gen_spec* spec) {
    if (!(e->symmetric && e->d_gid && e->n_own && lsat_wanted(e, true))) return GG_OK;
    if (!e->d_lsat) {
        HIPCHK(hipMalloc(&e->d_lsat, e->rows));
        HIPCHK(hipMemsetAsync(e->d_lsat, 0, e->rows, e->stream));
    }
    LabEntry ent;
    if (spec->kind != GG_GEN_TREE) {
        lab_prepare(e, spec);  // (a no-op after generate_sharded's call)
        std::lock_guard<std::mutex> lk(g_lab_mu);
        auto it = g_lab_cache.find(lab_key(spec));
        if (it != g_lab_cache.end()) ent = it->second;
        else ent.fail = "labels evicted from the cache";
    }
    if (!ent.fail.empty()) {
        std::fprintf(stderr, "gg engine part %u: lean digest without component targets (every lane is the "
                             "target): %s\n", e->part, ent.fail.c_str());
        return hipStreamSynchronize(e->stream) == hipSuccess ? GG_OK : GG_EIO;
    }
    int rc = GG_OK;
    uint32_t* d_lab = nullptr;
    if (ent.labs && !ent.labs->empty()) {
        e->h_lab = *ent.labs;
        e->lab_global = true;
        HIPCHK(hipMalloc(&d_lab, e->V * 4));
        HIPCHK(hipMemcpy(d_lab, e->h_lab.data(), e->V * 4, hipMemcpyHostToDevice));
        if (hipMalloc(&e->d_llab, e->n_own * 4) != hipSuccess) {
            rc = e->fail(GG_EIO, "lean digest: labels");
        } else {
            hipLaunchKernelGGL(gg::llab_gather, dim3((unsigned)std::min<uint64_t>((e->n_own + 255) / 256, 8192)),
                               dim3(256), 0, e->stream, d_lab, e->d_gid, e->d_llab, e->n_own);
            rc = hipGetLastError() == hipSuccess ? lsat_targets_alloc(e) : GG_EIO;
        }
    }
    if (rc == GG_OK) rc = hipStreamSynchronize(e->stream) == hipSuccess ? GG_OK : GG_EIO;
    (void)hipFree(d_lab);
    return rc;
}

static uint64_t window_bytes(const gg_engine* e) {
    return gg::kWinHdr + 2 * std::max<uint64_t>((e->xroff[e->P] + 255) / 256 * 256, 256);
}

static int generate_sharded(gg_engine* e, const gg_gen_spec* spec, uint64_t* nnz_out) {
    const uint64_t V = e->V;
    const uint32_t P = e->P;
    std::vector<uint64_t> plo(P + 1);
    for (uint32_t p = 0; p < P; ++p) plo[p] = std::min<uint64_t>(V, (V * p / P) / 64 * 64);
    plo[P] = V;
    const uint64_t lo = plo[e->part], hi = plo[e->part + 1];
    lab_prepare(e, spec);  // the whole graph's labels while this part holds no HBM yet
    gg_gen::Csr g{};
    std::string err;
    int rc = gg_gen::build_csr_rows(*spec, e->stream, 0u, lo, hi, &g, &err);
    if (rc) return e->fail(rc, err);
    if ((rc = install_shard(e, g, plo, nnz_out))) return rc;
    return lsat_parts(e, spec);
}

// A rank's own rows [plo[part], plo[part+1]) of a symmetric graph (g: row_ptr
// from 0, global column ids, on the device; the engine takes both arrays) ->
// its ghosts, send lists and ghost -> owned lists on the device
// (gg_gen::shard_csr), then the engine's per-node state.
static int install_shard(gg_engine* e, gg_gen::Csr g, const std::vector<uint64_t>& plo, uint64_t* nnz_out) {
    const uint64_t lo = plo[e->part], hi = plo[e->part + 1];
    std::string err;
    int rc = 0;
    const uint64_t n_own = hi - lo;
    const uint64_t ghost0 = (n_own + 63) / 64 * 64;
    gg_gen::Shard sh;
    rc = gg_gen::shard_csr(&g, lo, hi, plo, ghost0, gg::kRecipBit, e->stream, &sh, &err);
    if (rc) {
        (void)hipFree(g.row_ptr);
        (void)hipFree(g.col);
        return e->fail(rc, err);
    }
    // until the engine owns them, every device array of the shard is freed on an
    // error (gg_topology_part hands its caller's rows in through this path)
    std::vector<uint32_t> own_row;
    uint32_t* d_grow = nullptr;
    auto drop = [&](int code, const std::string& m) {
        for (void* p : {(void*)g.row_ptr, (void*)g.col, (void*)sh.send_idx, (void*)sh.gout_ptr, (void*)sh.gout_col,
                        (void*)sh.gout_sidx, (void*)sh.gid, (void*)d_grow})
            if (p) (void)hipFree(p);
        return e->fail(code, m);
    };
    // rows in locality order (the single engine's degree order): hot rows together
    g.V = n_own;
    if (!test_knob("GG_SHARD_NATIVE")) {
        rc = gg_gen::shard_reorder(&g, &sh, ghost0, gg::kRecipBit, e->stream, &d_grow, &own_row, &err);
        if (rc) return drop(rc, err);
    }
    const uint64_t rows = std::max<uint64_t>(64, (ghost0 + sh.n_ghost + 63) / 64 * 64);
    if (rows > 0x7fffffffull) return drop(GG_EINVAL, "local rows exceed 2^31");
    e->gid.assign(rows, ~0u);
    if (own_row.empty()) {
        for (uint64_t i = 0; i < n_own; ++i) e->gid[i] = (uint32_t)(lo + i);
        for (uint64_t k = 0; k < sh.n_ghost; ++k) e->gid[ghost0 + k] = sh.ghosts_host[k];
    } else {  // the reordered rows' ids
        const hipError_t ce = hipMemcpy(e->gid.data(), sh.gid, rows * 4, hipMemcpyDeviceToHost);
        if (ce != hipSuccess) return drop(GG_EIO, std::string("hipMemcpy(gid): ") + hipGetErrorString(ce));
    }
    e->range_mode = true;
    e->range_lo = lo;
    e->range_hi = hi;
    e->loc_of.clear();
    e->symmetric = true;
    e->n_own = n_own;
    e->n_ghost = sh.n_ghost;
    e->ghost0 = ghost0;
    e->rows = rows;
    std::vector<uint32_t>().swap(sh.ghosts_host);
    e->own_row.swap(own_row);
    e->d_grow = d_grow;
    e->d_gid = sh.gid;
    e->d_in_ptr = g.row_ptr;
    e->d_in_col = g.col;
    e->d_out_ptr = g.row_ptr;
    e->d_out_col = g.col;
    e->n_in_edges = g.nnz;
    e->n_out_edges = g.nnz;
    if (nnz_out) *nnz_out = g.nnz;  // this rank's rows
    e->send_off = sh.send_off;
    e->recv_off = sh.recv_off;
    e->d_send_idx = sh.send_idx;
    e->d_gout_ptr = sh.gout_ptr;
    e->d_gout_col = sh.gout_col;
    e->d_gout_sidx = sh.gout_sidx;
    if ((rc = setup_exchange(e))) return rc;
    uint64_t dmax = 0;
    if ((rc = gg_gen::max_degree(g.row_ptr, n_own, e->stream, &dmax, &err))) return e->fail(rc, err);
    std::vector<int64_t> iptr;
    if (dmax > hub_threshold()) {  // hub chunks are planned on the host
        iptr.resize(n_own + 1);
        HIPCHK(hipMemcpy(iptr.data(), g.row_ptr, (n_own + 1) * 8, hipMemcpyDeviceToHost));
    }
    return finish_topology(e, iptr.empty() ? nullptr : iptr.data(), nullptr);
}

extern "C" {

int gg_topology_generate(gg_engine* e, const gg_gen_spec* spec, uint64_t* nnz_out) {
    if (!e || !spec) return GG_EINVAL;
    if (gg_gen::spec_nodes(*spec) != e->V) return e->fail(GG_EINVAL, "generator node count != engine n_nodes");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->free_topology();
    e->have_topo = false;
    e->host_rp.clear();
    e->windows.erase(std::remove_if(e->windows.begin(), e->windows.end(), [](const Window& w) { return w.edges; }),
                     e->windows.end());
    gg_gen::Csr g{};
    std::string err;
    if (e->P != 1) return generate_sharded(e, spec, nnz_out);
    e->range_mode = false;
    int rc = gg_gen::build_csr(*spec, e->stream, gg::kRecipBit, &g, &err);
    if (rc) return e->fail(rc, err);
    e->rows = std::max<uint64_t>(64, (e->V + 63) / 64 * 64);
    e->loc_of.clear();
    e->gid.clear();
    uint64_t dmax = 0;
    if ((rc = gg_gen::max_degree(g.row_ptr, e->V, e->stream, &dmax, &err))) {
        (void)hipFree(g.row_ptr);
        (void)hipFree(g.col);
        return e->fail(rc, err);
    }
    {  // degree_order's rule, on the device: power-law graphs get rows by descending degree
        const char* o = test_knob("GG_ORDER");
        const double mean = (double)g.nnz / (double)std::max<uint64_t>(1, e->V);
        const bool want = o && !strcmp(o, "degree") ? true
                          : o && !strcmp(o, "native") ? false
                                                      : (double)dmax > 16.0 * std::max(1.0, mean);
        if (want && (rc = gg_gen::degree_reorder(&g, e->rows, e->stream, gg::kRecipBit, &e->d_gid, &e->gid,
                                                 &e->loc_of, &err))) {
            (void)hipFree(g.row_ptr);
            (void)hipFree(g.col);
            return e->fail(rc, err);
        }
    }
    e->d_in_ptr = g.row_ptr;
    e->d_in_col = g.col;
    e->d_out_ptr = g.row_ptr;
    e->d_out_col = g.col;
    e->symmetric = true;
    e->n_own = e->V;
    e->n_ghost = 0;
    e->ghost0 = e->V;
    e->n_in_edges = g.nnz;
    e->n_out_edges = g.nnz;
    if (nnz_out) *nnz_out = g.nnz;
    std::vector<int64_t> iptr;
    if (dmax > hub_threshold()) {  // hub chunks are planned on the host
        iptr.resize(e->V + 1);
        HIPCHK(hipMemcpy(iptr.data(), g.row_ptr, (e->V + 1) * 8, hipMemcpyDeviceToHost));
    }
    return finish_topology(e, iptr.empty() ? nullptr : iptr.data(), nullptr);
}

// HandleTopology on a vertex-sharded engine from this rank's own rows only
// (broadcast.go:40-45: each node keeps its own row; here each rank its range):
// uploaded as they are, then the same device path as a generated shard.
int gg_topology_part(gg_engine* e, const uint64_t* part_lo, const int64_t* row_ptr, const int32_t* col,
                     uint64_t nnz) {
    if (!e || !part_lo || !row_ptr || (nnz && !col)) return GG_EINVAL;
    if (e->P < 2) return e->fail(GG_EINVAL, "gg_topology_part: not a vertex-sharded engine (use gg_topology)");
    const uint32_t P = e->P;
    std::vector<uint64_t> plo(part_lo, part_lo + P + 1);
    if (plo[0] != 0 || plo[P] != e->V) return e->fail(GG_EINVAL, "gg_topology_part: part_lo must run from 0 to n_nodes");
    for (uint32_t q = 0; q < P; ++q)
        if (plo[q + 1] < plo[q]) return e->fail(GG_EINVAL, "gg_topology_part: part_lo not ascending");
    const uint64_t lo = plo[e->part], hi = plo[e->part + 1], n = hi - lo;
    if (n == 0) return e->fail(GG_EINVAL, "gg_topology_part: empty part");
    if (row_ptr[0] != 0 || (uint64_t)row_ptr[n] != nnz) return e->fail(GG_EINVAL, "row_ptr[0]/row_ptr[n] mismatch");
    {
        std::atomic<int> bad{0};  // 1 monotone, 2 range, 3 order, 4 self-asymmetric
        host_parallel(n, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b && !bad.load(std::memory_order_relaxed); ++i) {
                if (row_ptr[i + 1] < row_ptr[i]) { bad = 1; return; }
                for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
                    if (col[k] < 0 || (uint64_t)col[k] >= e->V) { bad = 2; return; }
                    if (k > row_ptr[i] && col[k] <= col[k - 1]) { bad = 3; return; }
                    // links inside the part must be listed both ways (the rest is the caller's promise)
                    const uint64_t w = (uint64_t)col[k];
                    if (w >= lo && w < hi &&
                        !std::binary_search(col + row_ptr[w - lo], col + row_ptr[w - lo + 1], (int32_t)(lo + i))) {
                        bad = 4;
                        return;
                    }
                }
            }
        });
        if (bad == 1) return e->fail(GG_EINVAL, "row_ptr not monotone");
        if (bad == 2) return e->fail(GG_EINVAL, "neighbour id out of range");
        if (bad == 3) return e->fail(GG_EINVAL, "neighbour list not ascending/unique");
        if (bad == 4) return e->fail(GG_EINVAL, "gg_topology_part: the topology must be symmetric");
    }
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->free_topology();
    e->have_topo = false;
    e->host_rp.clear();
    e->windows.erase(std::remove_if(e->windows.begin(), e->windows.end(), [](const Window& w) { return w.edges; }),
                     e->windows.end());
    gg_gen::Csr g{};
    g.V = n;
    g.nnz = nnz;
    hipError_t ue = hipMalloc(&g.row_ptr, (n + 1) * 8);
    if (ue == hipSuccess) ue = hipMalloc(&g.col, std::max<uint64_t>(1, nnz) * 4);
    if (ue == hipSuccess) ue = hipMemcpy(g.row_ptr, row_ptr, (n + 1) * 8, hipMemcpyHostToDevice);
    if (ue == hipSuccess && nnz) ue = hipMemcpy(g.col, col, nnz * 4, hipMemcpyHostToDevice);
    if (ue != hipSuccess) {
        if (g.row_ptr) (void)hipFree(g.row_ptr);
        if (g.col) (void)hipFree(g.col);
        return e->fail(GG_EIO, std::string("gg_topology_part upload: ") + hipGetErrorString(ue));
    }
    const int rc = install_shard(e, g, plo, nullptr);
    if (rc == GG_OK) e->part_rows = true;  // per-edge window bits: over the caller's own rows
    return rc;
}

int gg_topology_export(gg_engine* e, int64_t* row_ptr, int32_t* col, uint64_t cap, uint64_t* nnz_out) {
    if (!e || !row_ptr) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P != 1) return e->fail(GG_EINVAL, "gg_topology_export: vertex-sharded engine");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (nnz_out) *nnz_out = e->n_in_edges;
    const uint64_t V = e->V;
    if (e->gid.empty()) {  // rows are node ids
        HIPCHK(hipMemcpy(row_ptr, e->d_in_ptr, (V + 1) * 8, hipMemcpyDeviceToHost));
        if (!col) return GG_OK;
        if (cap < e->n_in_edges) return e->fail(GG_EINVAL, "col buffer too small");
        if (e->n_in_edges) HIPCHK(hipMemcpy(col, e->d_in_col, e->n_in_edges * 4, hipMemcpyDeviceToHost));
        host_parallel(e->n_in_edges, [&](uint64_t lo, uint64_t hi) {
            for (uint64_t k = lo; k < hi; ++k) col[k] = (int32_t)((uint32_t)col[k] & gg::kColMask);
        });
        return GG_OK;
    }
    // degree-ordered rows: back to node ids (row v = local row loc_of[v], columns by gid)
    std::vector<int64_t> ip(V + 1);
    HIPCHK(hipMemcpy(ip.data(), e->d_in_ptr, (V + 1) * 8, hipMemcpyDeviceToHost));
    row_ptr[0] = 0;
    for (uint64_t v = 0; v < V; ++v) {
        const uint32_t l = e->loc_of[v];
        row_ptr[v + 1] = row_ptr[v] + (ip[l + 1] - ip[l]);
    }
    if (!col) return GG_OK;
    if (cap < e->n_in_edges) return e->fail(GG_EINVAL, "col buffer too small");
    std::vector<uint32_t> ic(e->n_in_edges);
    if (e->n_in_edges) HIPCHK(hipMemcpy(ic.data(), e->d_in_col, e->n_in_edges * 4, hipMemcpyDeviceToHost));
    host_parallel(V, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t v = lo; v < hi; ++v) {
            const uint32_t l = e->loc_of[v];
            for (int64_t k = ip[l]; k < ip[l + 1]; ++k)
                col[row_ptr[v] + (k - ip[l])] = (int32_t)e->gid[ic[k] & gg::kColMask];
        }
    });
    return GG_OK;
}

static int add_window(gg_engine* e, int64_t a, int64_t b, Window&& w) {
    if (a >= b) return e->fail(GG_EINVAL, "empty partition window");
    for (const auto& x : e->windows)  // per-edge windows may overlap group windows (and win)
        if (x.edges == w.edges && a < x.to && x.from < b) return e->fail(GG_EINVAL, "overlapping partition windows");
    w.from = a;
    w.to = b;
    e->windows.push_back(std::move(w));
    return GG_OK;
}

int gg_partition_seeded(gg_engine* e, int64_t a, int64_t b, uint64_t epoch_seed) {
    if (!e) return GG_EINVAL;
    Window w;
    w.seeded = true;
    w.epoch_seed = epoch_seed;
    return add_window(e, a, b, std::move(w));
}

// Per-edge partition window (Maelstrom's partition nemesis as arbitrary cut
// links; SURVEY.md Appendix A D7: an explicit per-edge bitset overrides the
// seeded plan). The caller's E bits follow its CSR (entry k of row u = the link
// u -> col[k]); a cut link drops messages both ways, so the topology and the
// mask must be symmetric. Converted here to this engine's local in-edge order.
int gg_set_partition(gg_engine* e, int64_t a, int64_t b, const uint64_t* bits) {
    if (!e || !bits) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "gg_set_partition: install the topology first");
    if (!e->symmetric) return e->fail(GG_EINVAL, "gg_set_partition: per-edge windows need a symmetric topology");
    if (e->P > 1 && e->host_rp.empty() && !e->part_rows)
        return e->fail(GG_EINVAL, "gg_set_partition: a shard built by gg_topology_generate holds no whole-graph "
                                  "row offsets (use gg_topology or gg_topology_part, or seeded/group windows)");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const uint64_t V = e->V, n_own = e->n_own;
    std::vector<int64_t> ip(n_own + 1);
    std::vector<uint32_t> ic(e->n_in_edges);
    HIPCHK(hipMemcpy(ip.data(), e->d_in_ptr, (n_own + 1) * 8, hipMemcpyDeviceToHost));
    if (e->n_in_edges) HIPCHK(hipMemcpy(ic.data(), e->d_in_col, e->n_in_edges * 4, hipMemcpyDeviceToHost));
    auto gid = [&](uint64_t row) -> uint64_t { return e->gid.empty() ? row : e->gid[row]; };
    // the caller's row offsets: every node's degree (sharded: kept from gg_topology)
    std::vector<int64_t> crp;
    const std::vector<int64_t>* rp = &e->host_rp;
    if (e->host_rp.empty()) {
        crp.assign(V + 1, 0);
        for (uint64_t i = 0; i < n_own; ++i) crp[gid(i) + 1] = ip[i + 1] - ip[i];
        for (uint64_t v = 0; v < V; ++v) crp[v + 1] += crp[v];
        rp = &crp;
    }
    auto bit = [&](uint64_t k) { return (bits[k >> 6] >> (k & 63)) & 1ull; };
    Window w;
    w.seeded = false;
    w.epoch_seed = 0;
    w.edges = true;
    w.ebits.assign((e->n_in_edges + 63) / 64, 0);
    for (uint64_t i = 0; i < n_own; ++i) {
        const uint64_t v = gid(i);
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
            if (!bit((uint64_t)((*rp)[v] + (k - ip[i])))) continue;
            w.ebits[k >> 6] |= 1ull << (k & 63);
            // symmetric mask: the reverse link u -> v (an owned u) must be cut too
            const uint32_t ru = ic[k] & gg::kColMask;
            if (ru >= n_own) continue;  // a ghost: its owner checks
            const uint64_t u = gid(ru);
            int64_t lo = ip[ru], hi = ip[ru + 1];
            while (lo < hi) {  // u's list ascends by node id
                const int64_t mid = (lo + hi) / 2;
                if (gid(ic[mid] & gg::kColMask) < v) lo = mid + 1;
                else hi = mid;
            }
            if (lo >= ip[ru + 1] || !bit((uint64_t)((*rp)[u] + (lo - ip[ru]))))
                return e->fail(GG_EINVAL, "gg_set_partition: the mask is not symmetric");
        }
    }
    return add_window(e, a, b, std::move(w));
}

int gg_partition_groups(gg_engine* e, int64_t a, int64_t b, const uint8_t* group) {
    if (!e || !group) return GG_EINVAL;
    Window w;
    w.seeded = false;
    w.epoch_seed = 0;
    w.group.assign(group, group + e->V);
    return add_window(e, a, b, std::move(w));
}

// One client broadcast into the round's list `dst` (e->inj[round]).
static int add_broadcast(gg_engine* e, uint32_t node, int64_t message, int64_t round,
                         std::vector<Injection>& dst) {
    if (node >= e->V) return e->fail(GG_EINVAL, "node out of range");
    if (round < e->round) return e->fail(GG_EINVAL, "broadcast scheduled in the past");
    uint32_t lane = e->lanes.find(message);
    if (lane == ~0u) {
        if (e->lane_value.size() >= e->cfg.n_lanes) return e->fail(GG_ENOSPC, "all message lanes in use");
        lane = (uint32_t)e->lane_value.size();
        e->lanes.insert(message, lane);
        e->lane_value.push_back(message);
    }
    dst.push_back({node, lane});
    if (e->inj_rounds.empty() || *e->inj_rounds.rbegin() != round) e->inj_rounds.insert(round);
    return GG_OK;
}

int gg_broadcast(gg_engine* e, uint32_t node, int64_t message, int64_t round) {
    if (!e) return GG_EINVAL;
    if (round < e->round) return e->fail(GG_EINVAL, "broadcast scheduled in the past");
    return add_broadcast(e, node, message, round, e->inj[round]);
}

int gg_broadcast_many(gg_engine* e, const uint32_t* nodes, const int64_t* messages,
                      const int64_t* rounds, uint64_t n) {
    if (!e || (n && (!nodes || !messages || !rounds))) return GG_EINVAL;
    std::vector<Injection>* dst = nullptr;
    int64_t dst_round = 0;
    for (uint64_t k = 0; k < n; ++k) {
        if (rounds[k] < e->round) return e->fail(GG_EINVAL, "broadcast scheduled in the past");
        if (!dst || rounds[k] != dst_round) {  // runs of one round: one map lookup
            dst = &e->inj[rounds[k]];
            dst_round = rounds[k];
            if (dst->empty()) dst->reserve(n - k);
        }
        int rc = add_broadcast(e, nodes[k], messages[k], rounds[k], *dst);
        if (rc) return rc;
    }
    return GG_OK;
}

int gg_lane_of(const gg_engine* e, int64_t message) {
    if (!e) return GG_EINVAL;
    const uint32_t lane = e->lanes.find(message);
    return lane == ~0u ? GG_EINVAL : (int)lane;
}

int64_t gg_current_round(const gg_engine* e) { return e ? e->round : -1; }

namespace {

// One batch of m <= kMaxBatch rounds from e->round, enqueued (captured once,
// replayed after): each round's 64 counter slots are folded on the device into
// one row at d_counters + kMaxBatch * kSlots * kCounters and copied to
// h_counters. wait: synchronise and time it (run_batch). paths: each round's
// path bits (host-known).
int enqueue_step_batch(gg_engine* e, uint32_t m, bool wait, std::vector<uint64_t>& paths) {
    const int64_t r0 = e->round;
    int rc = ensure_events(e, 2);
    if (rc) return rc;
    if (e->inj_ev_live) {  // h_inj reuse: only the copy out of it must be done (not e.g. a reset)
        HIPCHK(hipEventSynchronize(e->inj_ev));
        e->inj_ev_live = false;
    }
    std::vector<size_t> off;
    const size_t total = pack_injections(e, r0, m, off);
    if (total == (size_t)-1) return GG_EIO;
    const int64_t save_round = e->round;
    const bool save_db = e->db_active, save_fd = e->f_dirty;
    const int save_set = e->set_cur;
    const uint32_t save_solo = e->last_solo;
    auto enqueue_batch = [&]() -> int {
        e->db_active = save_db;  // (a failed capture may have run it once already)
        e->f_dirty = save_fd;
        e->set_cur = save_set;
        e->last_solo = save_solo;
        e->d_base = e->d_sets[save_set];
        // the slots are zero after a fold (fold_slots clears what it read): only a
        // batch after other users of the slots (sharded rounds, setup) zeroes them
        if (e->batch_zr)
            if (int rz = zero_async(e, e->d_counters, (size_t)e->batch_zr * gg::kSlots * gg::kCounters * 8)) return rz;
        for (uint32_t k = 0; k < m; ++k) {
            const uint32_t ni = (uint32_t)(off[k + 1] - off[k]);
            e->round = r0 + k;
            int rc2 = enqueue_round(e, e->d_inj, ni, e->d_counters + (size_t)k * gg::kSlots * gg::kCounters,
                                    e->d_injtab + k);
            if (rc2) return rc2;
        }
        // fold the 64 slots of each round on the device: one 256-byte row per round to the host
        unsigned long long* folded = e->d_counters + (size_t)kMaxBatch * gg::kSlots * gg::kCounters;
        hipLaunchKernelGGL(gg::fold_slots, dim3(m), dim3(gg::kCounters), 0, e->stream, e->d_counters, folded, 1u);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(e->h_counters, folded, (size_t)m * gg::kCounters * 8, hipMemcpyDeviceToHost,
                              e->stream));
        return GG_OK;
    };
    e->batch_zr = e->ctr_dirty ? std::max(e->ctr_dirty, m) : 0u;
    rc = run_batch(e, r0, m, off, total, enqueue_batch, wait);
    e->batch_zr = 0;
    e->ctr_dirty = rc ? kMaxBatch : 0u;  // (fold_slots zeroed the m rounds it read, the rest was zero)
    e->round = save_round + m;
    // the double-buffer state after the batch (a replayed graph enqueued nothing)
    e->db_active = save_db;
    e->f_dirty = save_fd;
    e->set_cur = save_set;
    e->last_solo = save_solo;
    paths.assign(m, 0);
    for (uint32_t k = 0; k < m; ++k) {
        const bool dbk = db_round(e, r0 + k);
        e->last_solo = solo_of(e, r0 + k, dbk);
        paths[k] = path_of(e, r0 + k, dbk) | (e->last_solo ? GG_PATH_SOLO : 0u);
        db_advance(e, r0 + k, dbk);
    }
    return rc;
}

// The host side of a batch's rounds once their folded counter rows are in `rows`.
void finish_step_batch(gg_engine* e, int64_t r0, uint32_t m, const std::vector<uint64_t>& paths,
                       const unsigned long long* rows, gg_round_stats* out, bool retire, bool learn = true) {
    for (uint32_t k = 0; k < m; ++k) {
        gg_round_stats s;
        fold_stats(e, rows + (size_t)k * gg::kCounters, r0 + k, &s, 1, learn);
        s.path = paths[k];
        e->quiet = s.new_bits ? 0 : e->quiet + 1;
        if (out) out[k] = s;
        if (retire) retire_round(e, r0 + k);
    }
}

// gg_reset's host part: round 0, no pending acks, no lane history; keep_schedule:
// the lanes and client broadcasts stay (gg_run_episodes restores them itself).
void reset_host_state(gg_engine* e, bool keep_schedule) {
    e->dist_k = 0;
    e->dist_done.clear();
    e->inj_off = 0;
    if (!keep_schedule) {
        e->lanes.clear();
        e->lane_value.clear();
        e->inj.clear();
        e->inj_rounds.clear();
    }
    e->dirty_parity = (int)(e->round & 1);
    e->round = 0;
    e->pend_acks = e->pend_ackdrop = 0;
    e->hash_total = 0;
    e->dist_open = false;
    e->u_hist.clear();
    e->u_bits.clear();
    e->lret.clear();
    e->last_solo = 0;
}

}  // namespace

int gg_step(gg_engine* e, uint32_t n, gg_round_stats* out) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P != 1) return e->fail(GG_EINVAL, "vertex-sharded engine: use gg_dist_round_begin/end");
    HIPCHK(hipSetDevice(e->device));
    int rc = materialize_windows(e);
    if (rc) return rc;
    if ((rc = ensure_db(e))) return rc;
    if ((rc = ensure_sync(e, e->round + (int64_t)n - 1))) return rc;
    uint32_t done = 0;
    std::vector<uint64_t> paths;
    e->step_event_ms = 0.0;
    while (done < n) {
        const uint32_t m = std::min<uint32_t>(kMaxBatch, n - done);
        const int64_t r0 = e->round;
        if ((rc = enqueue_step_batch(e, m, true, paths))) return rc;
        HIPCHK(hipStreamSynchronize(e->stream));
        finish_step_batch(e, r0, m, paths, e->h_counters, out ? out + done : nullptr, true);
        done += m;
    }
    return GG_OK;
}

int gg_run_episodes(gg_engine* e, uint32_t n, uint32_t episodes, gg_round_stats* out) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P != 1) return e->fail(GG_EINVAL, "vertex-sharded engine: use gg_dist_round_begin/end");
    if (e->round != 0) return e->fail(GG_EINVAL, "gg_run_episodes: call it right after gg_reset and the broadcasts");
    if (n < 1 || n > kMaxBatch || episodes < 1) return e->fail(GG_EINVAL, "gg_run_episodes: bad sizes");
    HIPCHK(hipSetDevice(e->device));
    int rc = materialize_windows(e);
    if (rc) return rc;
    if ((rc = ensure_db(e))) return rc;
    if ((rc = ensure_sync(e, (int64_t)n - 1))) return rc;
    if ((rc = ensure_events(e, 3))) return rc;
    // every episode's folded counter rows in a device ring, read back once
    const size_t rows_b = (size_t)n * gg::kCounters * 8, need = rows_b * episodes;
    if (need > e->ep_cap) {
        HIPCHK(hipStreamSynchronize(e->stream));
        dfree(e->d_ep);
        if (e->h_ep) (void)hipHostFree(e->h_ep);
        e->h_ep = nullptr;
        e->ep_cap = 0;
        HIPCHK(hipMalloc(&e->d_ep, need));
        HIPCHK(hipHostMalloc(&e->h_ep, need));
        e->ep_cap = need;
    }
    const auto inj0 = e->inj;
    const LaneTable lanes0 = e->lanes;
    const std::vector<int64_t> lv0 = e->lane_value;
    const int quiet0 = e->quiet;
    std::vector<std::vector<uint64_t>> paths(episodes);
    const unsigned long long* folded = e->d_counters + (size_t)kMaxBatch * gg::kSlots * gg::kCounters;
    int quiet_end = 0;  // trailing quiet rounds of an episode: every episode's, they are the same
    // the timed span (gg_step_device_ms): episodes t0k..K-1. Episode 1 can hold a
    // graph capture (the hints learned from episode 0 change the batch key), so
    // with three or more episodes the span starts at episode 2, whose batch
    // replays episode 1's graph; with two it is episode 1 (capture included)
    const uint32_t t0k = episodes > 2 ? 2 : (episodes > 1 ? 1 : 0);
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    for (uint32_t k = 0; k < episodes; ++k) {
        if (k == 2 && t0k == 2) HIPCHK(hipEventRecord(e->ev[2], e->stream));
        if (k) {  // gg_reset + the same broadcasts, without gg_reset's wait
            reset_host_state(e, true);
            e->inj = inj0;
            e->lanes = lanes0;
            e->lane_value = lv0;
            e->quiet = quiet_end;  // (reset clears the per-round F arrays only where they can be dirty)
            if ((rc = reset_device_state(e))) return rc;
        }
        if ((rc = enqueue_step_batch(e, n, false, paths[k]))) return rc;
        HIPCHK(hipMemcpyAsync(e->d_ep + (size_t)k * n * gg::kCounters, folded, rows_b, hipMemcpyDeviceToDevice,
                              e->stream));
        if (k == 0 && episodes > 1) {
            // the episodes are identical, so the first one's trailing quiet rounds
            // (its folded rows reach h_counters inside the replayed sequence) tell
            // every later reset how much of the F buffers an episode leaves dirty:
            // one host wait, after the first episode only
            HIPCHK(hipStreamSynchronize(e->stream));
            if (t0k == 1) HIPCHK(hipEventRecord(e->ev[2], e->stream));
            int q = 2;  // what a reset leaves
            for (uint32_t j = 0; j < n; ++j) q = e->h_counters[(size_t)j * gg::kCounters + gg::C_NEW] ? 0 : q + 1;
            quiet_end = q;
            // and which expand kernel each marking round needs (the later episodes: one each)
            for (uint32_t j = 0; j < n; ++j)
                learn_busy(e, j + 1, 2.0 * (double)e->h_counters[(size_t)j * gg::kCounters + gg::C_NACT] *
                                             (double)e->n_in_edges >= (double)e->n_own * (double)e->n_own);
        }
    }
    HIPCHK(hipEventRecord(e->ev[1], e->stream));
    HIPCHK(hipMemcpyAsync(e->h_ep, e->d_ep, need, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0.f;
    // per episode of the span t0k..K-1 (queued after the one host wait)
    HIPCHK(hipEventElapsedTime(&ms, e->ev[t0k ? 2 : 0], e->ev[1]));
    e->step_event_ms = (double)ms / (episodes - t0k);
    for (uint32_t k = 0; k < episodes; ++k) {  // each episode's stats from round 0's state
        e->hash_total = 0;
        e->pend_acks = e->pend_ackdrop = 0;
        e->quiet = k ? 2 : quiet0;  // (what a reset leaves)
        finish_step_batch(e, 0, n, paths[k], e->h_ep + (size_t)k * n * gg::kCounters, out ? out + (size_t)k * n : nullptr,
                          k + 1 == episodes, false);
    }
    return GG_OK;
}

int gg_step_device_ms(const gg_engine* e, double* ms) {
    if (!e || !ms) return GG_EINVAL;
    *ms = e->step_event_ms;
    return GG_OK;
}

int gg_dist_info(const gg_engine* e, uint64_t* n_own, uint64_t* n_ghost, uint64_t* n_send) {
    if (!e || !e->have_topo) return GG_EINVAL;
    if (n_own) *n_own = e->n_own;
    if (n_ghost) *n_ghost = e->n_ghost;
    if (n_send) *n_send = e->send_off.empty() ? 0 : e->send_off[e->P];
    return GG_OK;
}

int gg_dist_owned(const gg_engine* e, uint32_t* nodes, uint64_t cap, uint64_t* n_out) {
    if (!e || !e->have_topo) return GG_EINVAL;
    if (n_out) *n_out = e->n_own;
    if (nodes)
        for (uint64_t i = 0; i < e->n_own && i < cap; ++i) nodes[i] = e->gid.empty() ? (uint32_t)i : e->gid[i];
    return GG_OK;
}

// Counters of the pending sharded rounds -> dist_done (waits for the stream).
static int fold_pending(gg_engine* e) {
    if (e->dist_k) {
        const size_t slot = (size_t)gg::kSlots * gg::kCounters;
        HIPCHK(hipMemcpyAsync(e->h_counters, e->d_counters, e->dist_k * slot * 8, hipMemcpyDeviceToHost, e->stream));
        if (e->d_payload)
            HIPCHK(hipMemcpyAsync(e->dist_sent.data(), e->d_payload, e->dist_k * 8, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->ipc) {
        uint32_t err = 0;
        HIPCHK(hipMemcpy(&err, e->d_xticket + 1, 4, hipMemcpyDeviceToHost));
        if (err)
            return e->fail(GG_EIO, "device-driven exchange: a peer did not arrive within the wait bound (" +
                                       std::to_string(err) +
                                       " wait(s) ran out; the exchange stays dead: install a new topology and "
                                       "export/import again)");
    }
    for (uint32_t k = 0; k < e->dist_k; ++k) {
        gg_round_stats s;
        fold_stats(e, e->h_counters + (size_t)k * gg::kSlots * gg::kCounters, e->dist_round_of[k], &s);
        s.path = e->dist_path[k];
        s.sent_bytes = e->d_payload ? e->dist_sent[k] : 0;
        e->dist_done.push_back(s);
    }
    e->dist_k = 0;
    e->inj_off = 0;
    return GG_OK;
}

}  // extern "C"

// The device-driven exchange's kernel arguments for this round (peer_win null:
// no IPC exchange).
static gg::IpcArgs ipc_args(const gg_engine* e) {
    gg::IpcArgs ip{};
    if (!e->ipc) return ip;
    ip.peer_win = e->d_peer_win;
    ip.peer_off = e->d_peer_off;
    ip.peer_rbuf = e->d_peer_rbuf;
    ip.my_win = reinterpret_cast<uint64_t*>(e->d_win);
    ip.rbuf = e->win_rbuf;
    ip.send_mask = e->send_mask;
    ip.recv_mask = e->recv_mask;
    ip.seq = reinterpret_cast<uint64_t*>(e->d_xticket + 2);
    ip.ticket = e->d_xticket;
    ip.err = e->d_xticket + 1;
    static const uint32_t limit = test_knob("GG_IPC_SPIN_LIMIT") ? (uint32_t)strtoul(test_knob("GG_IPC_SPIN_LIMIT"), nullptr, 0)
                                                                  : gg::kSpinLimit;
    ip.spin_limit = limit;
    return ip;
}

// The pack of round r's ghost payloads (vertex parts): set marks, pack_ghosts
// (IPC: straight into the peers' receive buffers), finish_pack (headers, sizes,
// the payload bytes of counter slot `slot`; IPC: the peers' ready flags).
static int enqueue_pack(gg_engine* e, int64_t r, uint32_t slot) {
    // sets may be read in r+1 by callbacks (fired in r-1) and pushes (fired in r-2)
    const bool sync = e->cfg.enable_sync && r >= (int64_t)e->cfg.sync_base_ticks + 1;
    if (sync && e->n_ghost) {
        hipLaunchKernelGGL(gg::mark_set_needs, dim3((unsigned)((e->n_ghost + 255) / 256)), dim3(256), 0,
                           e->stream, e->d_fired[(r - 1) & 3], e->d_gout_ptr, e->d_gout_sidx, e->ghost0,
                           e->n_ghost, e->d_needmark);
        HIPCHK(hipGetLastError());
    }
    if (e->ipc && e->send_mask) {  // the peers' buffers of this round's parity are free
        hipLaunchKernelGGL(gg::ipc_wait, dim3(1), dim3(64), 0, e->stream, ipc_args(e), 0);
        HIPCHK(hipGetLastError());
    }
    if (e->ipc && e->need_produce && e->n_need_words) {  // our need bits of round r, for the peers' pack of r+1
        gg::NeedArgs na{};
        na.words = e->d_need_words;
        na.n_words = e->n_need_words;
        na.gfirst = e->d_gfirst;
        na.grow = e->d_grow;
        na.gout_ptr = e->d_gout_ptr;
        na.gout_col = e->d_gout_col;
        na.lsat = e->d_lsat;
        na.need_out = e->d_need_out;
        na.need_bytes = e->d_need_bytes;
        na.ipc = ipc_args(e);
        hipLaunchKernelGGL(gg::need_bits, dim3(std::min<uint32_t>((e->n_need_words + 3) / 4, 4096)), dim3(gg::kBlock), 0,
                           e->stream, na);
        HIPCHK(hipGetLastError());
    }
    if (e->n_xtiles) {
        gg::PackArgs pa{};
        // the peers' need bits of round r-1 (exact when no lane is injected in r-1 and r:
        // expand_kernels.hpp NeedWord)
        if (e->ipc && e->need_peers && r >= 1 && !e->inj_rounds.count(r) && !e->inj_rounds.count(r - 1)) {
            pa.need_in = e->d_need_in;
            pa.need_bytes_in = e->d_need_bytes + e->P;
            pa.need_peers = e->need_peers;
        }
        pa.F_cur = e->d_F[r & 1];
        pa.base = e->d_base;
        // a double-buffered round wrote no F rows: the payload's are set(r) & ~set(r-1)
        pa.set_prev = e->db_active ? e->d_sets[(r + 1) & 1] : nullptr;
        pa.flg_cur = e->d_flg[r & 1];
        pa.fired_m2 = e->d_fired[(r - 2) & 3];
        pa.needmark = e->d_needmark;
        pa.send_idx = e->d_send_idx;
        pa.tiles = e->d_xtiles;
        pa.n_tiles = e->n_xtiles;
        pa.cnt = e->d_xcnt;
        pa.out = e->d_xsend;
        pa.seg_off = e->d_xsoff;
        pa.nwp = (uint32_t)e->nwp;
        pa.stride = e->xstride;
        pa.sync = sync ? 1 : 0;
        pa.ipc = ipc_args(e);
        pa.ticket = e->d_xtk;  // finish_pack runs in the last block
        pa.parts = e->P;
        pa.self = e->part;
        pa.seg_bytes = e->d_segbytes;
        pa.payload = e->d_payload + slot;
        pa.sfirst = e->d_sfirst;
        hipLaunchKernelGGL(gg::pack_ghosts, dim3(std::min<uint32_t>(e->n_xtiles, 4096)), dim3(gg::kBlock), 0,
                           e->stream, pa);
        HIPCHK(hipGetLastError());
    } else {
        hipLaunchKernelGGL(gg::finish_pack, dim3(1), dim3(64), 0, e->stream, e->d_xcnt, e->d_xsend, e->d_xsoff, e->P,
                           e->part, e->xstride, e->d_segbytes, e->d_payload + slot, ipc_args(e), (uint32_t)e->nwp);
        HIPCHK(hipGetLastError());
    }
    return GG_OK;
}

// The received ghost payloads of round r into the ghost rows (IPC: once every
// source's ready flag says they landed; then the sources' consumed flags).
static int enqueue_unpack(gg_engine* e, int64_t r) {
    if (!e->n_ghost) return GG_OK;
    gg::UnpackArgs ua{};
    ua.F_cur = e->d_F[r & 1];
    ua.base = (e->cfg.batch_ticks && e->d_bset[0]) ? e->d_bset[r & 1] : e->d_base;
    ua.flg_cur = e->d_flg[r & 1];
    ua.stamp = e->d_stamp;
    ua.grow = e->d_grow;
    ua.act_cur = e->d_act_s + (r & 3) * gg::kSlots;
    ua.in = e->d_xrecv;
    ua.seg_off = e->d_xroff;
    ua.gfirst = e->d_gfirst;
    ua.parts = e->P;
    ua.self = e->part;
    ua.ghost0 = e->ghost0;
    ua.n_ghost = e->n_ghost;
    ua.nwp = (uint32_t)e->nwp;
    ua.stride = e->xstride;
    ua.round = (uint32_t)r;
    ua.ipc = ipc_args(e);
    if (e->last_mark) {  // round r+1 runs no round_prep: the active ghosts mark their owned receivers here
        ua.cand_mark = e->d_cand + (size_t)((r + 1) & 1) * e->rows;
        ua.gout_ptr = e->d_gout_ptr;
        ua.gout_col = e->d_gout_col;
    }
    if (e->ipc && e->recv_mask) {  // every source's segment of this round has landed
        hipLaunchKernelGGL(gg::ipc_wait, dim3(1), dim3(64), 0, e->stream, ua.ipc, 1);
        HIPCHK(hipGetLastError());
    }
    const uint64_t cap = 2 * e->n_ghost * (e->nwp >= 2 ? 1 + e->nwp / 2 : 1);  // 16-byte pieces, at most
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((cap + gg::kBlock - 1) / gg::kBlock, 2048));
    // few ghosts (trees, grids at small cuts): the stale-row clear rides in unpack's last block
    const bool fuse = e->n_ghost <= 16384;
    ua.stale_ticket = fuse ? e->d_xtk + 1 : nullptr;
    hipLaunchKernelGGL(gg::unpack_ghosts, dim3(blocks), dim3(gg::kBlock), 0, e->stream, ua);
    HIPCHK(hipGetLastError());
    if (!fuse) {
        hipLaunchKernelGGL(gg::clear_stale_ghosts, dim3((unsigned)((e->n_ghost + 255) / 256)), dim3(256), 0,
                           e->stream, e->d_F[r & 1], e->d_flg[r & 1], e->d_stamp, e->ghost0, e->n_ghost,
                           (uint32_t)e->nwp, (uint32_t)r);
        HIPCHK(hipGetLastError());
    }
    return GG_OK;
}

// One sharded round up to the exchange: the round's kernels, then (vertex
// parts) the pack of this round's ghost payloads. host_sizes: in exact mode,
// wait for the pack and return the segment sizes (the caller-driven exchange);
// the engine's own RCCL exchange moves the sizes on the device instead.
static int dist_begin(gg_engine* e, gg_exchange* x, bool host_sizes) {
    if (!e || !x) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->world < 2) return e->fail(GG_EINVAL, "not a sharded engine (world == 1): use gg_step");
    if (e->dist_open) return e->fail(GG_EINVAL, "round already open");
    HIPCHK(hipSetDevice(e->device));
    int rc = materialize_windows(e);
    if (rc) return rc;
    if ((rc = ensure_db(e))) return rc;
    if ((rc = ensure_sync(e, e->round))) return rc;
    if (e->dist_k == kMaxBatch && (rc = fold_pending(e))) return rc;
    const int64_t r = e->round;
    std::vector<size_t> off;
    const size_t total = pack_injections(e, r, 1, off, e->inj_off);
    if (total == (size_t)-1) return GG_EIO;
    const uint32_t* d_inj = nullptr;
    if (total) {
        e->inj_dev_hash = 0;  // d_inj now holds sharded rounds' pairs
        HIPCHK(hipMemcpyAsync(e->d_inj + 2 * e->inj_off, e->h_inj + 2 * e->inj_off, total * 8,
                              hipMemcpyHostToDevice, e->stream));
        d_inj = e->d_inj + 2 * e->inj_off;
        e->inj_off += total;
    }
    const size_t slot = (size_t)gg::kSlots * gg::kCounters;
    unsigned long long* ctr = e->d_counters + e->dist_k * slot;
    // the counter slots of a batch of rounds are cleared once, when it starts
    // (fold_pending has read the last one), and only as far as they were used:
    // a caller that folds every round (gg_dist_round_end with out) clears one slot
    if (e->dist_k == 0 && e->ctr_dirty) {
        if ((rc = zero_async(e, e->d_counters, e->ctr_dirty * slot * 8))) return rc;
        e->ctr_dirty = 0;
    }
    e->ctr_dirty = std::max(e->ctr_dirty, e->dist_k + 1);
    if ((rc = enqueue_round(e, d_inj, (uint32_t)total, ctr))) return rc;
    const uint32_t P = e->P;
    if (e->dist_round_of.size() < kMaxBatch) e->dist_round_of.resize(kMaxBatch);
    if (e->dist_path.size() < kMaxBatch) e->dist_path.resize(kMaxBatch);
    if (e->dist_sent.size() < kMaxBatch) e->dist_sent.resize(kMaxBatch);
    e->dist_round_of[e->dist_k] = r;
    e->dist_path[e->dist_k] = e->last_path;
    e->xsend_bytes.assign(e->world, 0);
    e->xrecv_bytes.assign(e->world, 0);
    e->xsend_off.assign(e->world, 0);
    e->xrecv_off.assign(e->world, 0);
    if (P > 1) {
        if ((rc = enqueue_pack(e, r, e->dist_k))) return rc;
        for (uint32_t q = 0; q < P; ++q) {  // peers: the parts of this lane group
            const uint32_t pr = e->peer_rank(q);
            e->xsend_off[pr] = e->xsoff[q];
            e->xrecv_off[pr] = e->xroff[q];
            e->xsend_bytes[pr] = e->xsoff[q + 1] - e->xsoff[q];
            e->xrecv_bytes[pr] = e->xroff[q + 1] - e->xroff[q];
        }
        if (e->ipc) {  // the pack kernels deliver the segments: nothing for a caller to move
            std::fill(e->xsend_bytes.begin(), e->xsend_bytes.end(), 0);
            std::fill(e->xrecv_bytes.begin(), e->xrecv_bytes.end(), 0);
        } else if (e->xexact && host_sizes) {
            HIPCHK(hipMemcpyAsync(e->h_segbytes, e->d_segbytes, P * 8, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            for (uint32_t q = 0; q < P; ++q)
                if (e->xexact_s[q]) e->xsend_bytes[e->peer_rank(q)] = e->h_segbytes[q];
        }
    }
    x->send = e->d_xsend;
    x->recv = e->d_xrecv;
    x->send_bytes = e->xsend_bytes.data();
    x->recv_bytes = e->xrecv_bytes.data();
    x->send_off = e->xsend_off.data();
    x->recv_off = e->xrecv_off.data();
    x->send_total = P > 1 ? e->xsoff[P] : 0;
    x->recv_total = P > 1 ? e->xroff[P] : 0;
    x->on_device = 1;
    x->exact = (P > 1 && e->xexact) ? 1 : 0;
    x->stream = (void*)e->stream;
    e->dist_open = true;
    return GG_OK;
}

extern "C" {

int gg_dist_round_begin(gg_engine* e, gg_exchange* x) { return dist_begin(e, x, true); }

int gg_dist_round_end(gg_engine* e, gg_round_stats* out) {
    if (!e || !e->dist_open) return GG_EINVAL;
    HIPCHK(hipSetDevice(e->device));
    const int64_t r = e->round;
    int rc = enqueue_unpack(e, r);
    if (rc) return rc;
    e->dist_k++;
    retire_round(e, r);
    e->round++;
    e->dist_open = false;
    if (out) {
        if ((rc = fold_pending(e))) return rc;
        *out = e->dist_done.back();
        e->dist_done.pop_back();
    }
    return GG_OK;
}

int gg_dist_flush(gg_engine* e, gg_round_stats* out, uint64_t cap, uint64_t* n_out) {
    if (!e) return GG_EINVAL;
    if (e->dist_open) return e->fail(GG_EINVAL, "round still open");
    HIPCHK(hipSetDevice(e->device));
    int rc = fold_pending(e);
    if (rc) return rc;
    const uint64_t n = e->dist_done.size();
    if (n_out) *n_out = n;
    if (!out) return GG_OK;
    if (cap < n) return e->fail(GG_EINVAL, "stats buffer too small");
    for (uint64_t i = 0; i < n; ++i) out[i] = e->dist_done[i];
    e->dist_done.clear();
    return GG_OK;
}

// ---- engine-owned RCCL exchange ------------------------------------------------
// The ghost exchange as grouped ncclSend/ncclRecv on the engine stream, one pair
// per peer rank with a non-empty segment (sizes match pairwise: rank p's send
// segment to q is q's receive segment from p). The RCCL entry points are
// resolved at run time from the copy already loaded in the process (PyTorch's,
// when it drives the ranks; same soname), else librccl.so.1 (or GG_RCCL_LIB),
// so a process never holds two RCCL builds.
}  // extern "C"
namespace {
struct RcclApi {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*errstr)(ncclResult_t) = nullptr;
};

RcclApi load_rccl() {
    RcclApi r;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) {
        const char* path = getenv("GG_RCCL_LIB");
        h = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) {
        r.why = std::string("RCCL not loadable: ") + dlerror();
        return r;
    }
    bool all = true;
    auto get = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) {
            all = false;
            r.why = std::string("RCCL symbol missing: ") + name;
        }
    };
    get(r.get_id, "ncclGetUniqueId");
    get(r.init_rank, "ncclCommInitRank");
    get(r.destroy, "ncclCommAbort");  // local teardown: no wait on peers at exit
    get(r.send, "ncclSend");
    get(r.recv, "ncclRecv");
    get(r.group_start, "ncclGroupStart");
    get(r.group_end, "ncclGroupEnd");
    get(r.errstr, "ncclGetErrorString");
    r.ok = all;
    return r;
}

const RcclApi& rccl() {
    static const RcclApi api = load_rccl();
    return api;
}
}  // namespace

// (the engine stream is synchronised first, so no operation of ours is pending)
static void rccl_destroy(ncclComm_t c) {
    if (rccl().ok) (void)rccl().destroy(c);
}
extern "C" {

#define NCCLCHK(x)                                                                         \
    do {                                                                                   \
        ncclResult_t r_ = (x);                                                             \
        if (r_ != ncclSuccess) return e->fail(GG_EIO, std::string(#x) + ": " + rccl().errstr(r_)); \
    } while (0)

int gg_dist_comm_available(char* why, uint64_t cap) {
    const RcclApi& r = rccl();
    if (why && cap) {
        std::snprintf(why, cap, "%s", r.ok ? "" : r.why.c_str());
    }
    return r.ok ? GG_OK : GG_EIO;
}

// The id carries the lane group and part count it was made for in its last 12
// bytes (RCCL's bootstrap handle — a magic and a socket address — leaves them
// zero; gg_dist_comm_id checks that), so gg_dist_comm_init can refuse an id of
// another lane group before ncclCommInitRank, where ranks of two groups with
// the same part numbers would fail or hang undetectably.
constexpr size_t kIdTag = 116;
constexpr uint32_t kIdMagic = 0x474c4747u;  // "GGLG"

int gg_dist_comm_id(const gg_engine* e, uint8_t* id_out) {
    if (!e || !id_out) return GG_EINVAL;
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    const RcclApi& r = rccl();
    if (!r.ok) return GG_EIO;
    ncclUniqueId id;
    if (r.get_id(&id) != ncclSuccess) return GG_EIO;
    std::memcpy(id_out, &id, sizeof(id));
    for (size_t k = kIdTag; k < 128; ++k)
        if (id_out[k]) return GG_EIO;  // this RCCL uses the bytes the tag would take
    const uint32_t tag[3] = {kIdMagic, e->lgrp, e->P};
    std::memcpy(id_out + kIdTag, tag, sizeof(tag));
    return GG_OK;
}

int gg_dist_comm_init(gg_engine* e, const uint8_t* id_in) {
    if (!e || !id_in) return GG_EINVAL;
    if (e->world < 2) return e->fail(GG_EINVAL, "not a sharded engine (world == 1)");
    if (e->comm || e->have_xport) return e->fail(GG_EINVAL, "exchange transport already set");
    if (e->P < 2) return e->fail(GG_EINVAL, "no vertex parts (lane_groups == world): nothing to exchange");
    uint32_t tag[3];
    std::memcpy(tag, id_in + kIdTag, sizeof(tag));
    if (tag[0] != kIdMagic) return e->fail(GG_EINVAL, "gg_dist_comm_init: not an id from gg_dist_comm_id");
    if (tag[1] != e->lgrp || tag[2] != e->P)
        return e->fail(GG_EINVAL, "gg_dist_comm_init: the id was made for lane group " + std::to_string(tag[1]) +
                                      " of " + std::to_string(tag[2]) + " parts, this engine is lane group " +
                                      std::to_string(e->lgrp) + " of " + std::to_string(e->P) +
                                      " (one id per lane group)");
    const RcclApi& r = rccl();
    if (!r.ok) return e->fail(GG_EIO, r.why);
    HIPCHK(hipSetDevice(e->device));
    ncclUniqueId id;
    std::memcpy(&id, id_in, sizeof(id));
    std::memset(reinterpret_cast<uint8_t*>(&id) + kIdTag, 0, 128 - kIdTag);  // RCCL's own bytes only
    ncclComm_t c = nullptr;
    // one communicator per lane group: its P parts, rank = part (lane groups never
    // exchange anything, and a process may hold engines of several lane groups)
    NCCLCHK(r.init_rank(&c, (int)e->P, id, (int)e->part));
    e->comm = c;
    return GG_OK;
}

// ---- device-driven exchange (IPC-mapped windows) ----------------------------
namespace {
struct IpcBlob {
    uint32_t magic, part, parts, lgrp;
    uint32_t need, pad;     // the exporting engine writes need bits (it holds the lean digest)
    uint64_t rbuf;          // receive buffer bytes of the exporting engine
    uint64_t roff[64];      // where source part q's segment lands in its receive buffer (xroff[q])
    hipIpcMemHandle_t handle;
};
static_assert(sizeof(IpcBlob) <= GG_IPC_BLOB_BYTES, "IPC blob size");
constexpr uint32_t kIpcMagic = 0x43504947u;  // "GIPC"
}  // namespace

// Window pool and mapping cache (round 6). On this ROCm (dmabuf IPC), a window
// freed after its peers had mapped and unmapped it, followed by a new window
// allocated and exported, sometimes failed: hipIpcGetMemHandle returned
// "invalid argument" on the new window and the peer process blocked in the
// runtime — the new allocation can take the address range of a mapping just
// closed (tools/ipc_reopen_repro.hip, scenario 5; intermittent: one run in two).
// That is what stalled the 8-rank rehearsal between the C2 headline and the C5
// leg (every engine freed its window, the next leg exported new ones). So no
// window is freed and no mapping is closed while the process lives: an engine
// takes the smallest free pooled window of its device that is large enough
// (else allocates and exports a new one, once), returns it when it is destroyed,
// and a peer window already mapped by this process is mapped again from the
// cache (keyed by its handle), never reopened. A reused window's flag area is
// zeroed before it is exported again (the new exchange's sequence numbers start
// at 0; every peer has left the old exchange: gg_dist_ipc_close + barrier).
namespace {
struct PooledWin {
    uint8_t* ptr;
    uint64_t bytes;
    int device;
    bool busy;
    hipIpcMemHandle_t handle;
};
std::mutex g_ipc_mu;
std::vector<PooledWin> g_win_pool;
std::map<std::string, void*> g_peer_maps;  // handle bytes -> this process's mapping

// A new window above 1 GiB is allocated in whole GiB. Measured on the 2-rank C4 leg
// at 2^24 nodes (two lane halves per rank, windows of 3.741 GiB): a window of that
// exact size, or rounded up to 2 MiB or 256 MiB, could not be mapped by the peer
// (hipIpcOpenMemHandle never returned, in every allocation order tried); rounded up
// to 4 GiB it mapped in milliseconds, every time. Windows up to
// 1 GiB (2^22 nodes) always mapped and keep their exact size.
// GG_IPC_WINDOW_ALIGN_MB overrides the granularity (0: exact sizes; the A/B).
uint64_t win_round(uint64_t bytes) {
    const char* s = test_knob("GG_IPC_WINDOW_ALIGN_MB");
    const uint64_t a = s ? (uint64_t)(atof(s) * 1048576.0) : (bytes > (1ull << 30) ? 1ull << 30 : 0);
    return a ? (bytes + a - 1) / a * a : bytes;
}

int win_acquire(gg_engine* e, uint64_t bytes) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    PooledWin* best = nullptr;
    for (auto& w : g_win_pool)
        if (!w.busy && w.device == e->device && w.bytes >= bytes && (!best || w.bytes < best->bytes)) best = &w;
    if (best) {
        best->busy = true;
        e->d_win = best->ptr;
        HIPCHK(hipMemset(e->d_win, 0, gg::kWinHdr));  // the flags of its last exchange
        return GG_OK;
    }
    PooledWin w{};
    bytes = win_round(bytes);
    // uncached: stores from the peers' pack kernels and this engine's reads meet in HBM
    HIPCHK(hipExtMallocWithFlags(reinterpret_cast<void**>(&w.ptr), bytes, hipDeviceMallocUncached));
    HIPCHK(hipMemset(w.ptr, 0, bytes));
    HIPCHK(hipIpcGetMemHandle(&w.handle, w.ptr));
    w.bytes = bytes;
    w.device = e->device;
    w.busy = true;
    g_win_pool.push_back(w);
    e->d_win = w.ptr;
    return GG_OK;
}

void win_release(uint8_t* p) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto& w : g_win_pool)
        if (w.ptr == p) w.busy = false;
}

uint64_t win_size(const uint8_t* p) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto& w : g_win_pool)
        if (w.ptr == p) return w.bytes;
    return 0;
}

bool win_handle(const uint8_t* p, hipIpcMemHandle_t* h) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto& w : g_win_pool)
        if (w.ptr == p) {
            *h = w.handle;
            return true;
        }
    return false;
}
}  // namespace

int gg_dist_ipc_export(gg_engine* e, uint8_t* blob) {
    if (!e || !blob) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P < 2) return e->fail(GG_EINVAL, "no vertex parts: nothing to exchange");
    if (e->ipc) return e->fail(GG_EINVAL, "exchange transport already set");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->win_rbuf = (e->xroff[e->P] + 255) / 256 * 256;
    if (e->d_win && win_size(e->d_win) < window_bytes(e)) {  // (a preallocated window too small)
        win_release(e->d_win);
        e->d_win = nullptr;
    }
    if (!e->d_win)  // a pooled window, or a new one exported once
        if (int rc = win_acquire(e, window_bytes(e))) return rc;
    if (!e->d_xticket) {
        HIPCHK(hipMalloc(&e->d_xticket, 16));
        HIPCHK(hipMemset(e->d_xticket, 0, 16));
    }
    IpcBlob b{};
    b.magic = kIpcMagic;
    b.part = e->part;
    b.parts = e->P;
    b.lgrp = e->lgrp;
    b.rbuf = std::max<uint64_t>(e->win_rbuf, 256);
    // need bits: with the lean digest, unless GG_NEED_BITS=0 (A/B)
    {
        const char* nk = test_knob("GG_NEED_BITS");
        e->need_produce = e->d_lsat != nullptr && e->symmetric && e->n_need_words && !(nk && atoi(nk) == 0);
    }
    b.need = e->need_produce ? 1u : 0u;
    for (uint32_t q = 0; q < e->P; ++q) b.roff[q] = e->xroff[q];
    if (!win_handle(e->d_win, &b.handle)) return e->fail(GG_EIO, "gg_dist_ipc_export: window not in the pool");
    std::memset(blob, 0, GG_IPC_BLOB_BYTES);
    std::memcpy(blob, &b, sizeof(b));
    return GG_OK;
}

int gg_dist_ipc_import(gg_engine* e, const uint8_t* blobs) {
    if (!e || !blobs) return GG_EINVAL;
    if (!e->d_win) return e->fail(GG_EINVAL, "gg_dist_ipc_import: call gg_dist_ipc_export first");
    if (e->ipc) return e->fail(GG_EINVAL, "exchange transport already set");
    const uint32_t P = e->P;
    std::vector<IpcBlob> b(P);
    for (uint32_t q = 0; q < P; ++q) {
        std::memcpy(&b[q], blobs + (size_t)q * GG_IPC_BLOB_BYTES, sizeof(IpcBlob));
        if (b[q].magic != kIpcMagic || b[q].part != q || b[q].parts != P || b[q].lgrp != e->lgrp)
            return e->fail(GG_EINVAL, "gg_dist_ipc_import: blob " + std::to_string(q) +
                                          " is not part " + std::to_string(q) + " of this lane group");
    }
    HIPCHK(hipSetDevice(e->device));
    std::vector<uint8_t*> win(P, nullptr);
    std::vector<uint64_t> off(P, 0), rb(P, 0);
    e->peer_map.assign(P, nullptr);
    e->send_mask = e->recv_mask = 0;
    e->need_peers = 0;
    const bool dbg = test_knob("GG_IPC_DEBUG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto note = [&](const char* what, uint32_t q) {
        if (dbg)
            std::fprintf(stderr, "gg_dist_ipc_import part %u: %s %u at %.3f s\n", e->part, what, q,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    };
    if (dbg) {
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        std::fprintf(stderr,
                     "gg_dist_ipc_import part %u: HBM free %.2f of %.2f GiB, own window %.3f GiB (allocated %.3f)\n",
                     e->part, fr / 1073741824.0, tot / 1073741824.0,
                     (gg::kWinHdr + 2.0 * std::max<uint64_t>(e->win_rbuf, 256)) / 1073741824.0,
                     win_size(e->d_win) / 1073741824.0);
    }
    double limit_s = 30.0;
    if (const char* s = test_knob("GG_IPC_OPEN_TIMEOUT_S")) limit_s = std::max(1.0, atof(s));
    for (uint32_t q = 0; q < P; ++q) {
        const bool snd = q != e->part && e->xsoff[q + 1] > e->xsoff[q];
        const bool rcv = q != e->part && e->xroff[q + 1] > e->xroff[q];
        if (!snd && !rcv) continue;
        void* m = nullptr;
        const std::string key(reinterpret_cast<const char*>(&b[q].handle), sizeof(hipIpcMemHandle_t));
        {
            std::lock_guard<std::mutex> lk(g_ipc_mu);
            auto it = g_peer_maps.find(key);
            if (it != g_peer_maps.end()) m = it->second;
        }
        if (m) note("mapped already (cache)", q);
        else note("open", q);
        if (!m) {  // bounded: a mapping that never returns fails this rank instead of hanging it
            struct Open {
                std::mutex mu;
                std::condition_variable cv;
                bool done = false;
                hipError_t rc = hipSuccess;
                void* m = nullptr;
            };
            auto st = std::make_shared<Open>();
            const int dev = e->device;
            const hipIpcMemHandle_t h = b[q].handle;
            std::thread([st, h, dev] {
                (void)hipSetDevice(dev);
                void* mm = nullptr;
                const hipError_t rc = hipIpcOpenMemHandle(&mm, h, hipIpcMemLazyEnablePeerAccess);
                std::lock_guard<std::mutex> lk(st->mu);
                st->rc = rc;
                st->m = mm;
                st->done = true;
                st->cv.notify_all();
            }).detach();
            std::unique_lock<std::mutex> lk(st->mu);
            if (!st->cv.wait_for(lk, std::chrono::duration<double>(limit_s), [&] { return st->done; })) {
                e->peer_map.assign(P, nullptr);  // (the mappings made so far stay in the cache)
                return e->fail(GG_EIO, "gg_dist_ipc_import: hipIpcOpenMemHandle of part " + std::to_string(q) +
                                           "'s window did not return within " + std::to_string((int)limit_s) +
                                           " s (GG_IPC_OPEN_TIMEOUT_S)");
            }
            if (st->rc != hipSuccess) {
                e->peer_map.assign(P, nullptr);
                return e->fail(GG_EIO, std::string("gg_dist_ipc_import: hipIpcOpenMemHandle: ") +
                                           hipGetErrorString(st->rc));
            }
            m = st->m;
            std::lock_guard<std::mutex> lk2(g_ipc_mu);
            g_peer_maps[key] = m;
        }
        note("opened", q);
        e->peer_map[q] = m;
        win[q] = static_cast<uint8_t*>(m);
        off[q] = b[q].roff[e->part];
        rb[q] = b[q].rbuf;
        if (snd) e->send_mask |= 1ull << q;
        if (rcv) e->recv_mask |= 1ull << q;
        if (snd && rcv && b[q].need) e->need_peers |= 1ull << q;  // q's bits cover our sends to q
    }
    HIPCHK(hipMalloc(&e->d_peer_win, P * sizeof(uint8_t*)));
    HIPCHK(hipMalloc(&e->d_peer_off, P * 8));
    HIPCHK(hipMalloc(&e->d_peer_rbuf, P * 8));
    HIPCHK(hipMemcpy(e->d_peer_win, win.data(), P * sizeof(uint8_t*), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->d_peer_off, off.data(), P * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->d_peer_rbuf, rb.data(), P * 8, hipMemcpyHostToDevice));
    note("tables done", P);
    e->ipc = true;
    return GG_OK;
}

int gg_dist_ipc_close(gg_engine* e) {
    if (!e) return GG_EINVAL;
    if (!e->ipc && e->peer_map.empty()) return GG_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));  // (waits are bounded: a dead exchange drains)
    if (e->dist_exec) (void)hipGraphExecDestroy(e->dist_exec);  // its kernels name the peer windows
    e->dist_exec = nullptr;
    e->peer_map.clear();  // (the mappings stay in the process's cache: never reopened, never closed)
    dfree(e->d_peer_win);
    dfree(e->d_peer_off);
    dfree(e->d_peer_rbuf);
    e->send_mask = e->recv_mask = 0;
    e->need_peers = 0;
    e->ipc = false;
    return GG_OK;
}

int gg_dist_transport_init(gg_engine* e, const gg_transport* t) {
    if (!e || !t || !t->group_start || !t->send || !t->recv || !t->group_end) return GG_EINVAL;
    if (e->world < 2) return e->fail(GG_EINVAL, "not a sharded engine (world == 1)");
    if (e->comm || e->have_xport || e->ipc) return e->fail(GG_EINVAL, "exchange transport already set");
    e->xport = *t;
    e->have_xport = true;
    return GG_OK;
}

}  // extern "C"

namespace {
// One group of point-to-point transfers of gg_dist_step, enqueued on the engine
// stream over RCCL or the caller's transport; peers are part indices of the
// engine's lane group. The group is closed even after a failed call.
struct XGroup {
    gg_engine* e;
    int rc = GG_OK;
    std::string what;
    explicit XGroup(gg_engine* eng) : e(eng) {
        if (e->comm) {
            const ncclResult_t x = rccl().group_start();
            if (x != ncclSuccess) fail(std::string("ncclGroupStart: ") + rccl().errstr(x));
        } else if (e->xport.group_start(e->xport.user)) {
            fail("transport group_start failed");
        }
    }
    void fail(const std::string& m) {
        if (rc == GG_OK) {
            rc = GG_EIO;
            what = m;
        }
    }
    void send(const void* p, uint64_t n, uint32_t q) {
        if (rc) return;
        if (e->comm) {
            const ncclResult_t x = rccl().send(p, n, ncclUint8, (int)q, e->comm, e->stream);
            if (x != ncclSuccess) fail(std::string("ncclSend: ") + rccl().errstr(x));
        } else if (e->xport.send(e->xport.user, p, n, q, (void*)e->stream)) {
            fail("transport send failed");
        }
    }
    void recv(void* p, uint64_t n, uint32_t q) {
        if (rc) return;
        if (e->comm) {
            const ncclResult_t x = rccl().recv(p, n, ncclUint8, (int)q, e->comm, e->stream);
            if (x != ncclSuccess) fail(std::string("ncclRecv: ") + rccl().errstr(x));
        } else if (e->xport.recv(e->xport.user, p, n, q, (void*)e->stream)) {
            fail("transport recv failed");
        }
    }
    int close() {
        if (e->comm) {
            const ncclResult_t x = rccl().group_end();
            if (x != ncclSuccess) fail(std::string("ncclGroupEnd: ") + rccl().errstr(x));
        } else if (e->xport.group_end(e->xport.user)) {
            fail("transport group_end failed");
        }
        return rc ? e->fail(rc, what) : GG_OK;
    }
};
}  // namespace

extern "C" {

}  // extern "C"

// ---- gg_topology_part_directed: a rank's own rows of a directed topology -----
// Each node keeps only its own row (broadcast.go:40-45); a receiver's in-list is
// made of other ranks' rows, so the ranks hand each other the reverse of their
// cut edges (one exchange of (receiver, sender) pairs over the engine's RCCL
// communicator or the caller's transport, staged through device memory), and
// every rank then builds its owned rows, ghosts (remote nodes adjacent in or out),
// send lists and ghost -> owned lists from local data only.
static int exchange_reverse_edges(gg_engine* e, const std::vector<uint64_t>& plo, const int64_t* orp,
                                  const int32_t* ocol, std::vector<int64_t>& irp, std::vector<uint32_t>& icol) {
    const uint32_t P = e->P, me = e->part;
    const uint64_t lo = plo[me], hi = plo[me + 1], n = hi - lo;
    auto owner = [&](uint64_t u) -> uint32_t {
        return (uint32_t)(std::upper_bound(plo.begin(), plo.end(), u) - plo.begin()) - 1;
    };
    std::vector<std::vector<uint64_t>> out(P);  // (receiver << 32 | sender) per receiver's part
    for (uint64_t i = 0; i < n; ++i)
        for (int64_t k = orp[i]; k < orp[i + 1]; ++k) {
            const uint64_t u = (uint64_t)ocol[k];
            out[owner(u)].push_back(u << 32 | (lo + i));
        }
    std::vector<uint64_t> scnt(P), rcnt(P, 0);
    for (uint32_t q = 0; q < P; ++q) scnt[q] = out[q].size();
    uint64_t* d_cnt = nullptr;
    HIPCHK(hipMalloc(&d_cnt, 2 * P * 8));
    HIPCHK(hipMemcpy(d_cnt, scnt.data(), P * 8, hipMemcpyHostToDevice));
    {
        XGroup g(e);
        for (uint32_t q = 0; q < P; ++q) {
            if (q == me) continue;
            g.send(d_cnt + q, 8, q);
            g.recv(d_cnt + P + q, 8, q);
        }
        const int rc = g.close();
        if (rc) {
            dfree(d_cnt);
            return rc;
        }
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(rcnt.data(), d_cnt + P, P * 8, hipMemcpyDeviceToHost));
    dfree(d_cnt);
    rcnt[me] = 0;
    uint64_t stot = 0, rtot = 0;
    std::vector<uint64_t> soff(P + 1, 0), roff(P + 1, 0);
    for (uint32_t q = 0; q < P; ++q) {
        soff[q + 1] = soff[q] + (q == me ? 0 : scnt[q]);
        roff[q + 1] = roff[q] + rcnt[q];
    }
    stot = soff[P];
    rtot = roff[P];
    std::vector<uint64_t> pairs(out[me]);  // this part's own links
    uint64_t *d_s = nullptr, *d_r = nullptr;
    HIPCHK(hipMalloc(&d_s, std::max<uint64_t>(1, stot) * 8));
    HIPCHK(hipMalloc(&d_r, std::max<uint64_t>(1, rtot) * 8));
    for (uint32_t q = 0; q < P; ++q)
        if (q != me && scnt[q]) HIPCHK(hipMemcpy(d_s + soff[q], out[q].data(), scnt[q] * 8, hipMemcpyHostToDevice));
    int rc = GG_OK;
    {
        XGroup g(e);
        for (uint32_t q = 0; q < P; ++q) {
            if (q == me) continue;
            if (scnt[q]) g.send(d_s + soff[q], scnt[q] * 8, q);
            if (rcnt[q]) g.recv(d_r + roff[q], rcnt[q] * 8, q);
        }
        rc = g.close();
    }
    if (rc == GG_OK) {
        pairs.resize(pairs.size() + rtot);
        const hipError_t ce = hipStreamSynchronize(e->stream);
        const hipError_t ce2 = ce == hipSuccess && rtot
                                   ? hipMemcpy(pairs.data() + out[me].size(), d_r, rtot * 8, hipMemcpyDeviceToHost)
                                   : ce;
        if (ce2 != hipSuccess) rc = e->fail(GG_EIO, std::string("reverse edges: ") + hipGetErrorString(ce2));
    }
    dfree(d_s);
    dfree(d_r);
    if (rc) return rc;
    std::sort(pairs.begin(), pairs.end());  // by receiver, then sender: in-lists ascending by sender id
    irp.assign(n + 1, 0);
    icol.resize(pairs.size());
    for (size_t k = 0; k < pairs.size(); ++k) {
        const uint64_t u = pairs[k] >> 32;
        if (u < lo || u >= hi) return e->fail(GG_EIO, "internal: a reverse edge for another part");
        irp[u - lo + 1]++;
        icol[k] = (uint32_t)pairs[k];
    }
    for (uint64_t i = 0; i < n; ++i) irp[i + 1] += irp[i];
    return GG_OK;
}

// The sharded install of gg_topology, from one part's own out-lists and in-lists
// (global ids, ascending) instead of the whole graph: owned rows in id order
// (range mode), ghosts by source part and id, send lists, ghost -> owned lists.
static int install_part_rows(gg_engine* e, const std::vector<uint64_t>& plo, const int64_t* orp, const int32_t* ocolg,
                             const std::vector<int64_t>& irp, const std::vector<uint32_t>& icolg) {
    const uint32_t P = e->P, me = e->part;
    const uint64_t lo = plo[me], hi = plo[me + 1], n_own = hi - lo;
    auto owner = [&](uint64_t u) -> uint32_t {
        return (uint32_t)(std::upper_bound(plo.begin(), plo.end(), u) - plo.begin()) - 1;
    };
    bool sym = true;  // this part's rows: every out-list equals its in-list
    for (uint64_t i = 0; i < n_own && sym; ++i) {
        if (orp[i + 1] - orp[i] != irp[i + 1] - irp[i]) sym = false;
        for (int64_t k = 0; sym && k < orp[i + 1] - orp[i]; ++k)
            if ((uint32_t)ocolg[orp[i] + k] != icolg[irp[i] + k]) sym = false;
    }
    e->symmetric = sym;
    e->range_mode = true;
    e->range_lo = lo;
    e->range_hi = hi;
    e->own_row.clear();
    e->loc_of.clear();
    e->n_own = n_own;
    std::vector<std::vector<uint32_t>> gfrom(P), sendl(P);
    std::vector<uint32_t> peers;
    for (uint64_t i = 0; i < n_own; ++i) {
        peers.clear();
        auto visit = [&](uint32_t u) {
            const uint32_t q = owner(u);
            if (q == me) return;
            gfrom[q].push_back(u);
            peers.push_back(q);
        };
        for (int64_t k = orp[i]; k < orp[i + 1]; ++k) visit((uint32_t)ocolg[k]);
        for (int64_t k = irp[i]; k < irp[i + 1]; ++k) visit(icolg[k]);
        std::sort(peers.begin(), peers.end());
        peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
        for (uint32_t q : peers) sendl[q].push_back((uint32_t)i);  // owned rows ascend with ids
    }
    std::vector<uint32_t> ghosts;
    e->send_off.assign(P + 1, 0);
    e->recv_off.assign(P + 1, 0);
    for (uint32_t q = 0; q < P; ++q) {
        auto& g = gfrom[q];
        std::sort(g.begin(), g.end());
        g.erase(std::unique(g.begin(), g.end()), g.end());
        ghosts.insert(ghosts.end(), g.begin(), g.end());
        e->recv_off[q + 1] = e->recv_off[q] + g.size();
        e->send_off[q + 1] = e->send_off[q] + sendl[q].size();
    }
    e->n_ghost = ghosts.size();
    e->ghost0 = (n_own + 63) / 64 * 64;
    e->rows = std::max<uint64_t>(64, (e->ghost0 + e->n_ghost + 63) / 64 * 64);
    if (e->rows > 0x7fffffffull) return e->fail(GG_EINVAL, "local rows exceed 2^31");
    e->gid.assign(e->rows, ~0u);
    for (uint64_t i = 0; i < n_own; ++i) e->gid[i] = (uint32_t)(lo + i);
    for (uint64_t k = 0; k < ghosts.size(); ++k) e->gid[e->ghost0 + k] = ghosts[k];
    auto row_of = [&](uint32_t u) -> uint32_t {
        if (u >= lo && u < hi) return (uint32_t)(u - lo);
        const uint32_t q = owner(u);
        const uint32_t* g0 = ghosts.data() + e->recv_off[q];
        const uint32_t* g1 = ghosts.data() + e->recv_off[q + 1];
        return (uint32_t)(e->ghost0 + e->recv_off[q] + (std::lower_bound(g0, g1, u) - g0));
    };
    std::vector<uint32_t> icol(irp[n_own]), ocol(sym ? 0 : orp[n_own]);
    host_parallel(n_own, [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) {
            const int32_t* ob = ocolg + orp[i];
            const int32_t* oe = ocolg + orp[i + 1];
            for (int64_t k = irp[i]; k < irp[i + 1]; ++k) {
                const uint32_t u = icolg[k];
                const bool recip = sym || std::binary_search(ob, oe, (int32_t)u);
                icol[k] = row_of(u) | (recip ? gg::kRecipBit : 0u);
            }
            if (!sym)
                for (int64_t k = orp[i]; k < orp[i + 1]; ++k) ocol[k] = row_of((uint32_t)ocolg[k]);
        }
    });
    std::vector<int64_t> gcnt(e->n_ghost + 1, 0);
    for (uint64_t k = 0; k < icol.size() && e->n_ghost; ++k) {
        const uint32_t ru = icol[k] & gg::kColMask;
        if (ru >= e->ghost0) gcnt[ru - e->ghost0 + 1]++;
    }
    std::vector<uint32_t> gocol;
    if (e->n_ghost) {
        for (uint64_t g = 0; g < e->n_ghost; ++g) gcnt[g + 1] += gcnt[g];
        gocol.resize(gcnt[e->n_ghost]);
        std::vector<int64_t> fill(gcnt.begin(), gcnt.end() - 1);
        for (uint64_t i = 0; i < n_own; ++i)
            for (int64_t k = irp[i]; k < irp[i + 1]; ++k) {
                const uint32_t ru = icol[k] & gg::kColMask;
                if (ru >= e->ghost0) gocol[fill[ru - e->ghost0]++] = (uint32_t)i;
            }
    }
    e->n_in_edges = icol.size();
    e->n_out_edges = sym ? icol.size() : ocol.size();
    HIPCHK(hipMalloc(&e->d_in_ptr, (n_own + 1) * 8));
    HIPCHK(hipMalloc(&e->d_in_col, std::max<size_t>(1, icol.size()) * 4));
    HIPCHK(hipMemcpy(e->d_in_ptr, irp.data(), (n_own + 1) * 8, hipMemcpyHostToDevice));
    if (!icol.empty()) HIPCHK(hipMemcpy(e->d_in_col, icol.data(), icol.size() * 4, hipMemcpyHostToDevice));
    if (sym) {
        e->d_out_ptr = e->d_in_ptr;
        e->d_out_col = e->d_in_col;
    } else {
        HIPCHK(hipMalloc(&e->d_out_ptr, (n_own + 1) * 8));
        HIPCHK(hipMalloc(&e->d_out_col, std::max<size_t>(1, ocol.size()) * 4));
        HIPCHK(hipMemcpy(e->d_out_ptr, orp, (n_own + 1) * 8, hipMemcpyHostToDevice));
        if (!ocol.empty()) HIPCHK(hipMemcpy(e->d_out_col, ocol.data(), ocol.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc(&e->d_gid, e->rows * 4));
    HIPCHK(hipMemcpy(e->d_gid, e->gid.data(), e->rows * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> sidx;
    for (uint32_t q = 0; q < P; ++q) sidx.insert(sidx.end(), sendl[q].begin(), sendl[q].end());
    HIPCHK(hipMalloc(&e->d_send_idx, std::max<size_t>(1, sidx.size()) * 4));
    if (!sidx.empty()) HIPCHK(hipMemcpy(e->d_send_idx, sidx.data(), sidx.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_gout_ptr, (e->n_ghost + 1) * 8));
    HIPCHK(hipMemcpy(e->d_gout_ptr, gcnt.data(), (e->n_ghost + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&e->d_gout_col, std::max<size_t>(1, gocol.size()) * 4));
    if (!gocol.empty()) HIPCHK(hipMemcpy(e->d_gout_col, gocol.data(), gocol.size() * 4, hipMemcpyHostToDevice));
    // the send entry of every ghost -> owned edge: the owned row's position in the
    // send list to the ghost's part (send lists hold owned rows, ascending)
    std::vector<uint32_t> gsidx(gocol.size());
    {
        uint32_t p = 0;
        for (uint64_t g = 0; g < e->n_ghost; ++g) {
            while (g >= e->recv_off[p + 1]) ++p;
            const auto& sl = sendl[p];
            for (int64_t k = gcnt[g]; k < gcnt[g + 1]; ++k) {
                const auto it = std::lower_bound(sl.begin(), sl.end(), gocol[k]);
                if (it == sl.end() || *it != gocol[k]) return e->fail(GG_EIO, "internal: ghost edge without a send entry");
                gsidx[k] = (uint32_t)(e->send_off[p] + (it - sl.begin()));
            }
        }
    }
    HIPCHK(hipMalloc(&e->d_gout_sidx, std::max<size_t>(1, gsidx.size()) * 4));
    if (!gsidx.empty()) HIPCHK(hipMemcpy(e->d_gout_sidx, gsidx.data(), gsidx.size() * 4, hipMemcpyHostToDevice));
    if (int rc = setup_exchange(e)) return rc;
    e->part_rows = true;
    return finish_topology(e, irp.data(), sym ? nullptr : orp);
}

extern "C" int gg_topology_part_directed(gg_engine* e, const uint64_t* part_lo, const int64_t* row_ptr,
                                         const int32_t* col, uint64_t nnz) {
    if (!e || !part_lo || !row_ptr || (nnz && !col)) return GG_EINVAL;
    if (e->P < 2) return e->fail(GG_EINVAL, "gg_topology_part_directed: not a vertex-sharded engine");
    if (!e->comm && !e->have_xport)
        return e->fail(GG_EINVAL, "gg_topology_part_directed: the reverse edges need gg_dist_comm_init or "
                                  "gg_dist_transport_init first");
    const uint32_t P = e->P;
    std::vector<uint64_t> plo(part_lo, part_lo + P + 1);
    if (plo[0] != 0 || plo[P] != e->V) return e->fail(GG_EINVAL, "part_lo must run from 0 to n_nodes");
    for (uint32_t q = 0; q < P; ++q)
        if (plo[q + 1] < plo[q]) return e->fail(GG_EINVAL, "part_lo not ascending");
    const uint64_t lo = plo[e->part], hi = plo[e->part + 1], n = hi - lo;
    if (n == 0) return e->fail(GG_EINVAL, "empty part");
    if (row_ptr[0] != 0 || (uint64_t)row_ptr[n] != nnz) return e->fail(GG_EINVAL, "row_ptr[0]/row_ptr[n] mismatch");
    for (uint64_t i = 0; i < n; ++i) {
        if (row_ptr[i + 1] < row_ptr[i]) return e->fail(GG_EINVAL, "row_ptr not monotone");
        for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            if (col[k] < 0 || (uint64_t)col[k] >= e->V) return e->fail(GG_EINVAL, "neighbour id out of range");
            if (k > row_ptr[i] && col[k] <= col[k - 1]) return e->fail(GG_EINVAL, "neighbour list not ascending/unique");
        }
    }
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->free_topology();
    e->have_topo = false;
    e->host_rp.clear();
    e->windows.erase(std::remove_if(e->windows.begin(), e->windows.end(), [](const Window& w) { return w.edges; }),
                     e->windows.end());
    std::vector<int64_t> irp;
    std::vector<uint32_t> icol;
    int rc = exchange_reverse_edges(e, plo, row_ptr, col, irp, icol);
    if (rc) return rc;
    return install_part_rows(e, plo, row_ptr, col, irp, icol);
}

// gg_dist_step when the exchange needs no host: the device-driven exchange (IPC)
// or none (lane groups only). Rounds go in batches that fill the pending counter
// slots; a batch is captured once into a hipGraph (kernels, the exchange's pack
// and unpack, the counter clear) and replayed while its shape — first round,
// length, first counter slot, the rounds that inject, lanes injected so far,
// windows, buffers — is unchanged; the injections and each round's offsets into
// them are uploaded before the launch and read on the device (as in gg_step). No
// host wait anywhere: the counters come back with gg_dist_flush.
static int dist_step_batched(gg_engine* e, uint32_t n_rounds) {
    HIPCHK(hipSetDevice(e->device));
    int rc = materialize_windows(e);
    if (rc) return rc;
    if ((rc = ensure_db(e))) return rc;
    if ((rc = ensure_sync(e, e->round + (int64_t)n_rounds - 1))) return rc;
    if (e->dist_round_of.size() < kMaxBatch) e->dist_round_of.resize(kMaxBatch);
    if (e->dist_path.size() < kMaxBatch) e->dist_path.resize(kMaxBatch);
    if (e->dist_sent.size() < kMaxBatch) e->dist_sent.resize(kMaxBatch);
    if (!e->d_injtab) {
        HIPCHK(hipMalloc(&e->d_injtab, (kMaxBatch + 1) * sizeof(uint32_t)));
        HIPCHK(hipHostMalloc(&e->h_injtab, (kMaxBatch + 1) * sizeof(uint32_t)));
    }
    static const bool no_graph = ab_knob("GG_NO_GRAPH") != nullptr;
    const size_t slot = (size_t)gg::kSlots * gg::kCounters;
    uint32_t done = 0;
    while (done < n_rounds) {
        if (e->dist_k == kMaxBatch && (rc = fold_pending(e))) return rc;
        const uint32_t k0 = e->dist_k;
        const uint32_t m = std::min<uint32_t>(n_rounds - done, kMaxBatch - k0);
        const int64_t r0 = e->round;
        // injections of the batch behind the pending rounds' (their kernels may not have run)
        std::vector<size_t> off;
        const size_t base = e->inj_off;
        const size_t total = pack_injections(e, r0, m, off, base);
        if (total == (size_t)-1) return GG_EIO;
        e->inj_dev_hash = 0;  // d_inj holds sharded rounds' pairs
        if (total)
            HIPCHK(hipMemcpyAsync(e->d_inj + 2 * base, e->h_inj + 2 * base, total * 8, hipMemcpyHostToDevice,
                                  e->stream));
        // the pinned table slots of this batch are not those of a pending batch (slots k0..k0+m)
        for (uint32_t k = 0; k <= m; ++k) e->h_injtab[k0 + k] = (uint32_t)(base + off[k]);
        HIPCHK(hipMemcpyAsync(e->d_injtab + k0, e->h_injtab + k0, (m + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                              e->stream));
        e->inj_off += total;
        e->injtab_dev_hash = ~0ull;  // gg_step's table cache no longer matches d_injtab
        const bool save_db = e->db_active, save_fd = e->f_dirty;
        const int save_set = e->set_cur;
        const uint32_t save_solo = e->last_solo;
        auto enqueue = [&]() -> int {
            e->db_active = save_db;
            e->f_dirty = save_fd;
            e->set_cur = save_set;
            e->last_solo = save_solo;
            e->d_base = e->d_sets[save_set];
            if (int rz = zero_async(e, e->d_counters + k0 * slot, (size_t)m * slot * 8)) return rz;
            for (uint32_t k = 0; k < m; ++k) {
                e->round = r0 + k;
                const uint32_t ni = (uint32_t)(off[k + 1] - off[k]);
                int rc2 = enqueue_round(e, e->d_inj, ni, e->d_counters + (k0 + k) * slot, e->d_injtab + k0 + k);
                if (rc2) return rc2;
                if (e->P > 1) {
                    if ((rc2 = enqueue_pack(e, r0 + k, k0 + k))) return rc2;
                    if ((rc2 = enqueue_unpack(e, r0 + k))) return rc2;
                }
            }
            return GG_OK;
        };
        BatchKey key;
        key.r0 = r0;
        key.m = m;
        key.windows = e->windows.size();
        key.inj_buf = e->d_inj;
        key.db_state = (e->db_active ? 2 : 0) | e->set_cur;
        key.solo_hash = solo_sched_hash(e, r0, m);
        {
            uint64_t p = gg_mix64(m);
            for (size_t k = 0; k < m; ++k) p = gg_mix64(p ^ (off[k + 1] > off[k] ? 2 * k + 1 : 2 * k));
            key.inj_hash = p;
            uint64_t u = gg_mix64(~0ull);
            for (int64_t q = r0 - 1; q < r0 + (int64_t)m; ++q) u = gg_mix64(u ^ lanes_through(e, q));
            key.u_hash = u;
        }
        if (no_graph || e->graph_broken || m < 4) {  // (a capture costs more than a few rounds' launches)
            if ((rc = enqueue())) return rc;
        } else {
            if (!(e->dist_exec && key == e->dist_key && k0 == e->dist_key_k0)) {
                if (e->dist_exec) (void)hipGraphExecDestroy(e->dist_exec);
                e->dist_exec = nullptr;
                hipGraph_t g = nullptr;
                bool ok = hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
                const int rc2 = ok ? enqueue() : GG_OK;
                if (ok) ok = hipStreamEndCapture(e->stream, &g) == hipSuccess && g && rc2 == GG_OK;
                hipGraphExec_t ge = nullptr;
                if (ok) ok = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
                if (g) (void)hipGraphDestroy(g);
                if (!ok) {
                    (void)hipGetLastError();
                    e->graph_broken = true;  // direct launches from now on
                    if ((rc = enqueue())) return rc;
                } else {
                    e->dist_exec = ge;
                    e->dist_key = key;
                    e->dist_key_k0 = k0;
                }
            }
            if (e->dist_exec) HIPCHK(hipGraphLaunch(e->dist_exec, e->stream));
        }
        // host state after the batch (a replayed graph enqueued nothing)
        e->db_active = save_db;
        e->f_dirty = save_fd;
        e->set_cur = save_set;
        e->last_solo = save_solo;
        for (uint32_t k = 0; k < m; ++k) {
            const bool dbk = db_round(e, r0 + k);
            e->dist_round_of[k0 + k] = r0 + k;
            e->last_solo = solo_of(e, r0 + k, dbk);
            e->dist_path[k0 + k] = path_of(e, r0 + k, dbk) | (e->last_solo ? GG_PATH_SOLO : 0u);
            db_advance(e, r0 + k, dbk);
            retire_round(e, r0 + k);
        }
        e->round = r0 + m;
        e->dist_k = k0 + m;
        e->ctr_dirty = std::max(e->ctr_dirty, e->dist_k);
        done += m;
    }
    return GG_OK;
}

extern "C" {

int gg_dist_step(gg_engine* e, uint32_t n_rounds) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->world < 2) return e->fail(GG_EINVAL, "not a sharded engine (world == 1): use gg_step");
    if (e->dist_open) return e->fail(GG_EINVAL, "round already open");
    const uint32_t P = e->P;
    if (e->ipc || P == 1) return dist_step_batched(e, n_rounds);
    if (P > 1 && !e->comm && !e->have_xport && !e->ipc)
        return e->fail(GG_EINVAL, "no communicator (gg_dist_comm_init, gg_dist_transport_init or gg_dist_ipc_import)");
    auto peer = [&](uint32_t q) {  // shares edges with part q (capacities are non-zero both ways)
        return q != e->part && e->xsoff.size() > q + 1 && e->xsoff[q + 1] > e->xsoff[q];
    };
    std::vector<uint64_t> sb(P, 0), rb(P, 0);
    for (uint32_t k = 0; k < n_rounds; ++k) {
        gg_exchange x{};
        int rc = dist_begin(e, &x, false);
        if (rc) return rc;
        if (P > 1 && !e->ipc) {  // (IPC: the pack kernels delivered the segments already)
            for (uint32_t q = 0; q < P; ++q) {
                sb[q] = e->xsoff[q + 1] - e->xsoff[q];
                rb[q] = e->xroff[q + 1] - e->xroff[q];
            }
            if (e->xexact) {
                // exact directions: this round's segment sizes first (8 bytes each way),
                // then one host wait for them (the payload counts are host arguments)
                XGroup g(e);
                for (uint32_t q = 0; q < P; ++q) {
                    if (q == e->part) continue;
                    if (e->xexact_s[q]) g.send(e->d_segbytes + q, 8, q);
                    if (e->xexact_r[q]) g.recv(e->d_segbytes + P + q, 8, q);
                }
                if ((rc = g.close())) return rc;
                HIPCHK(hipMemcpyAsync(e->h_segbytes, e->d_segbytes, 2 * P * 8, hipMemcpyDeviceToHost, e->stream));
                HIPCHK(hipStreamSynchronize(e->stream));
                for (uint32_t q = 0; q < P; ++q) {
                    if (e->xexact_s[q]) sb[q] = e->h_segbytes[q];
                    if (e->xexact_r[q]) rb[q] = e->h_segbytes[P + q];
                    if (sb[q] > e->xsoff[q + 1] - e->xsoff[q] || rb[q] > e->xroff[q + 1] - e->xroff[q])
                        return e->fail(GG_EIO, "exchange segment larger than its capacity");
                }
            }
            XGroup g(e);
            for (uint32_t q = 0; q < P; ++q) {
                if (!peer(q)) continue;  // own part / no shared edges: nothing either way
                if (sb[q]) g.send(e->d_xsend + e->xsoff[q], sb[q], q);
                if (rb[q]) g.recv(e->d_xrecv + e->xroff[q], rb[q], q);
            }
            if ((rc = g.close())) return rc;
        }
        if ((rc = gg_dist_round_end(e, nullptr))) return rc;
    }
    return GG_OK;
}

int gg_dist_run_episodes(gg_engine* e, uint32_t n, uint32_t episodes, gg_round_stats* out) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->world < 2) return e->fail(GG_EINVAL, "not a sharded engine (world == 1): use gg_run_episodes");
    if (!(e->ipc || e->P == 1)) return e->fail(GG_EINVAL, "gg_dist_run_episodes: needs the device-driven exchange");
    if (e->dist_open || e->dist_k || e->round != 0)
        return e->fail(GG_EINVAL, "gg_dist_run_episodes: call it right after gg_reset and the broadcasts");
    if (n < 1 || n > kMaxBatch || episodes < 1) return e->fail(GG_EINVAL, "gg_dist_run_episodes: bad sizes");
    HIPCHK(hipSetDevice(e->device));
    // every episode's raw counter slots (and payload bytes) in a device ring, read back once
    const size_t slot = (size_t)gg::kSlots * gg::kCounters;
    const size_t ctr_b = (size_t)n * slot * 8, pay_b = (size_t)n * 8, per = ctr_b + pay_b, need = per * episodes;
    if (need > e->ep_cap) {
        HIPCHK(hipStreamSynchronize(e->stream));
        dfree(e->d_ep);
        if (e->h_ep) (void)hipHostFree(e->h_ep);
        e->h_ep = nullptr;
        e->ep_cap = 0;
        HIPCHK(hipMalloc(&e->d_ep, need));
        HIPCHK(hipHostMalloc(&e->h_ep, need));
        e->ep_cap = need;
    }
    const auto inj0 = e->inj;
    const LaneTable lanes0 = e->lanes;
    const std::vector<int64_t> lv0 = e->lane_value;
    int rc = ensure_events(e, 2);
    if (rc) return rc;
    HIPCHK(hipEventRecord(e->ev[0], e->stream));
    for (uint32_t k = 0; k < episodes; ++k) {
        if (k) {  // gg_reset + the same broadcasts, without gg_reset's wait
            reset_host_state(e, true);
            e->inj = inj0;
            e->lanes = lanes0;
            e->lane_value = lv0;
            e->quiet = 0;
            if ((rc = reset_device_state(e))) return rc;
        }
        // (episode k > 0 packs the same pairs into the same pinned ring slots an
        // earlier episode's copy may still be reading: identical bytes)
        if ((rc = dist_step_batched(e, n))) return rc;
        auto* dst = reinterpret_cast<uint8_t*>(e->d_ep) + (size_t)k * per;
        HIPCHK(hipMemcpyAsync(dst, e->d_counters, ctr_b, hipMemcpyDeviceToDevice, e->stream));
        if (e->d_payload) HIPCHK(hipMemcpyAsync(dst + ctr_b, e->d_payload, pay_b, hipMemcpyDeviceToDevice, e->stream));
    }
    HIPCHK(hipEventRecord(e->ev[1], e->stream));
    HIPCHK(hipMemcpyAsync(e->h_ep, e->d_ep, need, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
    e->step_event_ms = (double)ms / episodes;
    if (e->ipc) {
        uint32_t err = 0;
        HIPCHK(hipMemcpy(&err, e->d_xticket + 1, 4, hipMemcpyDeviceToHost));
        if (err)
            return e->fail(GG_EIO, "device-driven exchange: a peer did not arrive within the wait bound (" +
                                       std::to_string(err) +
                                       " wait(s) ran out; the exchange stays dead: install a new topology and "
                                       "export/import again)");
    }
    for (uint32_t k = 0; k < episodes; ++k) {
        e->hash_total = 0;
        e->pend_acks = e->pend_ackdrop = 0;
        const auto* src = reinterpret_cast<const uint8_t*>(e->h_ep) + (size_t)k * per;
        const auto* ctr = reinterpret_cast<const unsigned long long*>(src);
        const auto* pay = reinterpret_cast<const unsigned long long*>(src + ctr_b);
        for (uint32_t j = 0; j < n; ++j) {
            gg_round_stats s;
            fold_stats(e, ctr + (size_t)j * slot, e->dist_round_of[j], &s);
            s.path = e->dist_path[j];
            s.sent_bytes = e->d_payload ? pay[j] : 0;
            e->quiet = s.new_bits ? 0 : e->quiet + 1;
            if (out) out[(size_t)k * n + j] = s;
        }
    }
    e->dist_k = 0;  // (folded here: gg_dist_flush has nothing pending)
    e->inj_off = 0;
    return GG_OK;
}

}  // extern "C"

// Local rows of owned nodes (GG_EINVAL if one is not owned).
static int rows_of(gg_engine* e, const uint32_t* nodes, uint64_t n, std::vector<uint32_t>& rows) {
    rows.resize(n);
    for (uint64_t k = 0; k < n; ++k) {
        const uint32_t l = local_row(e, nodes[k]);
        if (l == ~0u || l >= e->n_own) return e->fail(GG_EINVAL, "node not owned by this engine");
        rows[k] = l;
    }
    return GG_OK;
}

// Gather rows[0..n) on the device, kChunk rows per pass: sets (base | F of the
// last round where LAG) or delivery rounds; the rows may be anywhere in the
// local order (degree-ordered or sharded engines).
template <class T, class Launch>
static int gather_chunks(gg_engine* e, const std::vector<uint32_t>& rows, uint64_t per_row, std::vector<T>& h,
                         Launch&& launch) {
    constexpr uint64_t kChunk = 1 << 20;
    const uint64_t n = rows.size();
    h.resize(n * per_row);
    if (!n) return GG_OK;
    HIPCHK(hipStreamSynchronize(e->stream));
    uint32_t* d_rows = nullptr;
    T* d_out = nullptr;
    const uint64_t c = std::min(n, kChunk);
    hipError_t err = hipMalloc(&d_rows, c * 4);
    if (err == hipSuccess) err = hipMalloc(&d_out, c * per_row * sizeof(T));
    for (uint64_t k0 = 0; k0 < n && err == hipSuccess; k0 += kChunk) {
        const uint64_t m = std::min(kChunk, n - k0);
        err = hipMemcpyAsync(d_rows, rows.data() + k0, m * 4, hipMemcpyHostToDevice, e->stream);
        if (err == hipSuccess) {
            launch(d_rows, m, d_out);
            err = hipGetLastError();
        }
        if (err == hipSuccess)
            err = hipMemcpyAsync(h.data() + k0 * per_row, d_out, m * per_row * sizeof(T), hipMemcpyDeviceToHost,
                                 e->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    }
    if (d_rows) (void)hipFree(d_rows);
    if (d_out) (void)hipFree(d_out);
    HIPCHK(err);
    return GG_OK;
}

static int read_bits_rows(gg_engine* e, const uint32_t* nodes, uint64_t n, uint64_t* out) {
    std::vector<uint32_t> rows;
    int rc = rows_of(e, nodes, n, rows);
    if (rc) return rc;
    HIPCHK(hipSetDevice(e->device));
    std::vector<uint64_t> h;
    const int last = (int)((e->round - 1) & 1);
    const uint64_t* F = e->round ? e->d_F[last] : nullptr;
    const uint8_t* fl = e->round ? e->d_flg[last] : nullptr;
    rc = gather_chunks(e, rows, e->nwp, h, [&](const uint32_t* d_rows, uint64_t m, uint64_t* d_out) {
        const uint64_t t = m * e->nwp;
        hipLaunchKernelGGL(gg::gather_sets, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, e->stream, d_rows, m,
                           e->d_base, F, fl, (uint32_t)e->nwp, d_out);
    });
    if (rc) return rc;
    // whole-job words per node; a lane-group engine fills only its own words
    for (uint64_t k = 0; k < n; ++k) {
        if (e->L > 1) std::memset(out + k * e->nw_g, 0, e->nw_g * 8);
        std::memcpy(out + k * e->nw_g + e->w0, h.data() + k * e->nwp, e->nw * 8);
    }
    return GG_OK;
}

static int delivery_rows(gg_engine* e, const uint32_t* nodes, uint64_t n, int32_t* out) {
    if (!e->d_dr) return e->fail(GG_EINVAL, "GG_TRACK_DELIVERY not enabled");
    std::vector<uint32_t> rows;
    int rc = rows_of(e, nodes, n, rows);
    if (rc) return rc;
    HIPCHK(hipSetDevice(e->device));
    const uint64_t W = e->cfg.n_lanes, Wl = e->nw * 64;  // whole-job lanes, this engine's lanes
    std::vector<int32_t> h;
    rc = gather_chunks(e, rows, Wl, h, [&](const uint32_t* d_rows, uint64_t m, int32_t* d_out) {
        const uint64_t t = m * Wl;
        hipLaunchKernelGGL(gg::gather_rounds, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, e->stream, d_rows, m,
                           e->d_dr, (uint32_t)Wl, d_out);
    });
    if (rc) return rc;
    for (uint64_t k = 0; k < n; ++k) {
        if (e->L > 1) std::fill(out + k * W, out + (k + 1) * W, -1);
        std::memcpy(out + k * W + 64 * e->w0, h.data() + k * Wl, Wl * 4);
    }
    return GG_OK;
}

extern "C" {

static std::vector<uint32_t> node_range(uint32_t a, uint32_t b) {
    std::vector<uint32_t> v;
    for (uint32_t x = a; x < b; ++x) v.push_back(x);
    return v;
}

int gg_read(gg_engine* e, uint32_t node, int64_t* out, uint64_t cap, uint64_t* n_out) {
    if (!e || !e->have_topo) return GG_EINVAL;
    std::vector<uint64_t> h(e->nw_g);
    int rc = read_bits_rows(e, &node, 1, h.data());
    if (rc) return rc;
    std::vector<int64_t> vals;  // a lane-group engine: the values of its own lanes
    for (uint64_t j = 0; j < e->nw_g; ++j) {
        uint64_t x = h[j];
        while (x) {
            const int b = __builtin_ctzll(x);
            x &= x - 1;
            const uint64_t lane = j * 64 + b;
            if (lane < e->lane_value.size()) vals.push_back(e->lane_value[lane]);
        }
    }
    std::sort(vals.begin(), vals.end());
    if (n_out) *n_out = vals.size();
    if (out)
        for (uint64_t i = 0; i < vals.size() && i < cap; ++i) out[i] = vals[i];
    return GG_OK;
}

int gg_read_bits(gg_engine* e, uint32_t a, uint32_t b, uint64_t* out) {
    if (!e || !e->have_topo || !out || a > b) return GG_EINVAL;
    const auto v = node_range(a, b);
    return read_bits_rows(e, v.data(), v.size(), out);
}

int gg_read_bits_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, uint64_t* out) {
    if (!e || !e->have_topo || (n && (!nodes || !out))) return GG_EINVAL;
    return read_bits_rows(e, nodes, n, out);
}

int gg_delivery_rounds(gg_engine* e, uint32_t a, uint32_t b, int32_t* out, uint64_t cap) {
    if (!e || !e->have_topo || !out || a > b) return GG_EINVAL;
    if (cap < (uint64_t)(b - a) * e->cfg.n_lanes) return e->fail(GG_EINVAL, "output buffer too small");
    const auto v = node_range(a, b);
    return delivery_rows(e, v.data(), v.size(), out);
}

int gg_delivery_rounds_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, int32_t* out) {
    if (!e || !e->have_topo || (n && (!nodes || !out))) return GG_EINVAL;
    return delivery_rows(e, nodes, n, out);
}

int gg_reset(gg_engine* e) {
    if (!e) return GG_EINVAL;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    reset_host_state(e, false);
    if (!e->have_topo) return GG_OK;
    HIPCHK(hipSetDevice(e->device));
    return reset_device_state(e);
}

int gg_device_bytes(const gg_engine* e, uint64_t* total, uint64_t* sync_part) {
    if (!e) return GG_EINVAL;
    if (hipSetDevice(e->device) != hipSuccess) return GG_EIO;
    auto size_of = [](const void* p) -> uint64_t {
        size_t n = 0;
        return (p && hipMemPtrGetInfo(const_cast<void*>(p), &n) == hipSuccess) ? (uint64_t)n : 0ull;
    };
    const void* sync_ptrs[] = {e->d_srec, e->d_pushb, e->d_rev, e->d_sstate, e->d_ibits,
                               e->d_sat, e->d_sat_new, e->d_pushany, e->d_nmeta};
    const void* other[] = {
        e->d_gid, e->d_grow, e->d_send_idx, e->d_gout_ptr, e->d_gout_col, e->d_xsend, e->d_xrecv, e->d_xsoff,
        e->d_xroff, e->d_gfirst, e->d_xtiles, e->d_gout_sidx, e->d_needmark, e->d_stamp, e->d_xcnt, e->d_segbytes,
        e->d_payload, e->d_in_ptr, e->d_in_col, e->d_out_ptr == e->d_in_ptr ? nullptr : e->d_out_ptr,
        e->d_out_col == e->d_in_col ? nullptr : e->d_out_col, e->d_sets[0] ? e->d_sets[0] : e->d_base,
        e->d_sets[1], e->d_F[0], e->d_F[1], e->d_flg[0], e->d_flg[1], e->d_cand, e->d_zmark, e->d_tile_cand,
        e->d_work, e->d_n_work, e->d_bcount, e->d_nodes, e->d_act, e->d_act_deg, e->d_tot, e->d_act_s,
        e->d_act_deg_s, e->d_tot_s, e->d_abits, e->d_lsat, e->d_llab, e->d_lreach, e->d_ltab, e->d_hubs, e->d_hub_c0, e->d_hchunks, e->d_mchunks, e->d_pend,
        e->d_pend_src, e->d_bset[0], e->d_bset[1], e->d_hscratch, e->d_hflag, e->d_hlive, e->d_fired[0],
        e->d_fired[1], e->d_fired[2], e->d_fired[3], e->d_sync_next, e->d_sync_k, e->d_dr, e->d_counters,
        e->d_inj, e->d_injtab};
    uint64_t s = 0, o = 0;
    for (const void* p : sync_ptrs) s += size_of(p);
    for (const void* p : other) o += size_of(p);
    for (const auto& w : e->windows) o += size_of(w.d_grp) + size_of(w.d_ebits);
    if (total) *total = s + o;
    if (sync_part) *sync_part = s;
    return GG_OK;
}

}  // extern "C"
