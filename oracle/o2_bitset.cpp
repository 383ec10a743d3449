// O2 — bitset CPU restatement of the reference broadcast handlers.
//
// TEST INFRASTRUCTURE ONLY: built into oracle/_build/libgossip_cpu.so and loaded
// by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. It exports
// the same C ABI (include/gossip.h) as the product library libgossip_hip.so so a
// parity test can drive both with identical calls. Nothing in the product links it.
//
// Parity status: parity unpinned by reference tests (there are none: SURVEY.md §4,
// §8c). O2 is checked against the message-level literal restatement O1
// (oracle/o1_literal.py) on randomized small graphs, partitions and sync
// schedules, and against the analytic KATs of SURVEY.md §8c (tests/).
//
// Semantics, per node v in round r:
//   S  = seen_prev(v) | client broadcasts of round r          HandleBroadcast :59-79
//   for in-neighbour u ascending whose message was not dropped in round r-1:
//        contrib = seen_prev(u) if u pushed to v in r-1 else F_prev(u)
//        claim_u = contrib & ~S ;  S |= claim_u                first deliverer = u
//   if v's sync fired in r-2: for out-neighbour w ascending whose read (r-2) and
//        read_ok (r-1) both arrived:  R = seen_prev(w)         SyncBroadcast :82-117
//        new = R & ~S (forwarded to all but w, :97-100); push = S & ~R (to w,
//        :104-108); S |= R (:110-114)
//   seen_cur(v) = S ; F_cur(v) = S & ~seen_prev(v)             rebroadcastAllExcept :50-57
// Message counts use per-claimer popcounts (forward exclusion, :52) and the
// partition masks at the send round. Acks of round r are the broadcasts
// delivered in round r; they are counted by the sender in round r-1.
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gossip.h"
#include "gossip_spec.h"

namespace {

struct Window {
    int64_t from, to;
    bool seeded;
    uint64_t epoch_seed;
    std::vector<uint8_t> group;  // global node -> group (explicit windows)
    bool edges = false;          // gg_set_partition: cut links, in the caller's CSR order
    std::vector<uint64_t> bits;
};

struct Injection {
    uint32_t node;  // global id
    uint32_t lane;
};

struct alignas(128) Acc {  // per-thread counters (a cache line pair each: no false sharing)
    uint64_t new_bits = 0, fwd_sent = 0, fwd_deliv = 0, pushes = 0, push_deliv = 0;
    uint64_t reads = 0, read_oks = 0, dropped = 0, fired = 0, hash = 0;
    uint64_t node_dropped = 0;  // dropped reads / read_oks (node-level, not per lane)
    uint64_t next_acks = 0, next_ackdrop = 0;
    void add(const Acc& o) {
        new_bits += o.new_bits; fwd_sent += o.fwd_sent; fwd_deliv += o.fwd_deliv;
        pushes += o.pushes; push_deliv += o.push_deliv; reads += o.reads;
        read_oks += o.read_oks; dropped += o.dropped; fired += o.fired; hash += o.hash;
        node_dropped += o.node_dropped;
        next_acks += o.next_acks; next_ackdrop += o.next_ackdrop;
    }
};

inline int popc(uint64_t x) { return __builtin_popcountll(x); }

// Storage that is not zeroed at allocation: the full-size configs (C5: 2^30
// nodes, 6.4e9 adjacency entries) fill their buffers once, with every thread
// (reset_state), instead of twice on one.
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <class U>
    NoInit(const NoInit<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
using Words = std::vector<uint64_t, NoInit<uint64_t>>;

// A read-only window on CSR storage held elsewhere in the engine: a symmetric
// topology on one vertex part keeps ONE copy of the caller's rows and reads it
// as in-lists, out-lists and (per-edge windows) the caller's CSR alike.
template <class T>
struct View {
    const T* p = nullptr;
    uint64_t n = 0;
    const T& operator[](uint64_t i) const { return p[i]; }
    const T* data() const { return p; }
    uint64_t size() const { return n; }
    template <class V>
    void of(const V& v) { p = reinterpret_cast<const T*>(v.data()); n = v.size(); }
};

// n items over T threads, contiguous ranges: f(t, begin, end)
template <class Fn>
void pfor(int T, uint64_t n, Fn&& f) {
    if (T <= 1 || n < 65536) {
        f(0, 0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(t, n * t / T, n * (t + 1) / T); });
    for (auto& x : th) x.join();
}

// Host threads: the CPUs this process may run on, capped by the runtime's
// declared share (OMP_NUM_THREADS: the GPU box's per-GPU share of its host
// cores); GG_CPU_THREADS overrides both.
int default_threads() {
    int n = 0;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    if (const char* s = getenv("OMP_NUM_THREADS"))
        if (atoi(s) > 0) n = std::min(n, atoi(s));
    if (const char* s = getenv("GG_CPU_THREADS")) n = std::max(1, atoi(s));
    return n;
}

}  // namespace

struct gg_engine {
    gg_config cfg{};
    std::string err;
    uint64_t V = 0, nw = 0;
    uint32_t rank = 0, world = 1;
    // 2-D sharding (gg_config.lane_groups): L lane groups x P vertex parts; this
    // engine holds lane words [w0, w0 + nw) of nw_g for the nodes of part `part`
    uint32_t L = 1, P = 1, lgrp = 0, part = 0;
    uint64_t nw_g = 0, w0 = 0;
    uint32_t peer_rank(uint32_t q) const { return lgrp * P + q; }
    uint64_t lo = 0, hi = 0, slice = 0;    // owned range, rows per rank slice
    std::vector<uint64_t> rank_lo;         // [world+1]
    bool have_topo = false, symmetric = true;
    // owned rows; columns are replica indices (rank * slice + offset)
    View<int64_t> crp;                     // the caller's CSR (per-edge windows)
    View<int32_t> ccol;
    View<int64_t> in_ptr, out_ptr;
    View<uint32_t> in_col, out_col;
    std::vector<uint8_t> in_recip;         // empty: every in-edge is reciprocal (symmetric topology)
    bool recip(int64_t e) const { return in_recip.empty() || in_recip[e]; }
    // the storage behind the views (a symmetric topology on one part: only s_ptr, s_col)
    std::vector<int64_t, NoInit<int64_t>> s_ptr, s_optr, s_crp;
    std::vector<uint32_t, NoInit<uint32_t>> s_col, s_ocol;
    std::vector<int32_t, NoInit<int32_t>> s_ccol;
    // replicas [world*slice][nw]
    Words seen[2], F[2];
    // act[b][rep] = 1 iff F[b]'s row is not zero (a sender with nothing new is skipped)
    std::vector<uint8_t, NoInit<uint8_t>> act[2];
    std::vector<uint64_t> fired[4];        // [world*slice/64]
    bool fired_nz[4] = {false, false, false, false};  // slot holds some fired bit
    bool fired_any(int64_t r) const { return r >= 0 && fired_nz[r & 3]; }
    std::vector<int64_t, NoInit<int64_t>> sync_next;  // owned (filled by reset_state)
    std::vector<uint32_t, NoInit<uint32_t>> sync_k;
    std::vector<int32_t> dr;               // owned rows * W
    // batched gossip (cfg.batch_ticks): pending values, and who delivered them
    std::vector<uint64_t> pend;            // owned rows * nw
    std::vector<uint32_t> pend_src;        // owned: kNone, kMixed, or the only sender (global id)
    std::vector<Window> windows;
    std::unordered_map<int64_t, uint32_t> lanes;
    std::vector<int64_t> lane_value;
    std::map<int64_t, std::vector<Injection>> inj;
    int64_t round = 0;
    uint64_t pend_acks = 0, pend_ackdrop = 0;
    uint64_t hash_total = 0;  // seen_hash: all rounds' new-bit words so far
    int threads = 1;
    bool dist_open = false;
    Acc dist_acc;
    // sharded exchange (dense: every owned node's seen row, F row and fired
    // bit to every other rank; the HIP engine sends ghosts only)
    std::vector<uint8_t> xsend, xrecv;
    std::vector<uint64_t> xsend_bytes, xrecv_bytes, xsend_off, xrecv_off;
    std::vector<gg_round_stats> dist_pending;
    uint64_t xsend_sent = 0;  // payload bytes of the open round

    int fail(int code, const std::string& m) { err = m; return code; }

    uint64_t global_of(uint64_t rep) const {
        uint64_t r = rep / slice;
        return rank_lo[r] + (rep - r * slice);
    }
    uint64_t rep_of(uint64_t g) const {
        uint32_t r = (uint32_t)(std::upper_bound(rank_lo.begin(), rank_lo.end(), g) - rank_lo.begin()) - 1;
        return (uint64_t)r * slice + (g - rank_lo[r]);
    }
    const Window* window_at(int64_t r) const {
        for (const auto& w : windows)  // a per-edge window overrides a group window
            if (w.edges && w.from <= r && r < w.to) return &w;
        for (const auto& w : windows)
            if (!w.edges && w.from <= r && r < w.to) return &w;
        return nullptr;
    }
    int group_of(const Window* w, uint64_t g) const {
        return w->seeded ? (int)gg_part_group(cfg.seed, w->epoch_seed, g) : (int)w->group[g];
    }
    // message from global a to global b sent in round r dropped?
    bool masked(int64_t r, uint64_t a, uint64_t b) const { return masked_in(window_at(r), a, b); }
    // the same under the window of its round (window_at, hoisted out of a round's loops)
    bool masked_in(const Window* w, uint64_t a, uint64_t b) const {
        if (!w) return false;
        if (w->edges) {  // the link a -> b (symmetric topology: it exists both ways)
            const int32_t* r0 = ccol.data() + crp[a];
            const int32_t* r1 = ccol.data() + crp[a + 1];
            const uint64_t k = (uint64_t)crp[a] + (uint64_t)(std::lower_bound(r0, r1, (int32_t)b) - r0);
            return (w->bits[k >> 6] >> (k & 63)) & 1ull;
        }
        return group_of(w, a) != group_of(w, b);
    }
    bool fired_at(int64_t r, uint64_t rep) const {
        if (r < 0) return false;
        return (fired[r & 3][rep >> 6] >> (rep & 63)) & 1ull;
    }
    void reset_state() {
        for (int b = 0; b < 2; ++b) {
            pfor(threads, seen[b].size(), [&](int, uint64_t i0, uint64_t i1) {
                std::fill(seen[b].begin() + i0, seen[b].begin() + i1, 0ull);
                std::fill(F[b].begin() + i0, F[b].begin() + i1, 0ull);
            });
            std::fill(act[b].begin(), act[b].end(), (uint8_t)0);
        }
        for (int b = 0; b < 4; ++b) {
            std::fill(fired[b].begin(), fired[b].end(), 0ull);
            fired_nz[b] = false;
        }
        pfor(threads, hi - lo, [&](int, uint64_t i0, uint64_t i1) {
            for (uint64_t i = i0; i < i1; ++i) {
                sync_k[i] = 0;
                sync_next[i] = gg_sync_interval(cfg.seed, lo + i, 0, cfg.sync_base_ticks, cfg.sync_jitter_ticks);
            }
        });
        std::fill(dr.begin(), dr.end(), -1);
        std::fill(pend.begin(), pend.end(), 0ull);
        std::fill(pend_src.begin(), pend_src.end(), ~0u);
        lanes.clear();
        lane_value.clear();
        inj.clear();
        round = 0;
        pend_acks = pend_ackdrop = 0;
        hash_total = 0;
        dist_open = false;
    }
    void compute_round(Acc& total);
    void compute_round_batched(Acc& total);
};

// Batched gossip (gg_config.batch_ticks = B >= 1; new semantics, not the
// reference's; message-level restatement: oracle/o1_batched.py): per node v in
// round r, (1) client broadcasts, (2) the messages sent to v in r-1 and not
// dropped, ascending sender: the sender's batch (its F row of r-1) and, on a
// push edge, its push (its whole set after r-1: the push carried every value it
// held that v's read_ok of r-2 lacked, and v's set has grown past that reply);
// a value's first deliverer is its claimer and new values join v's pending set
// P; (3) if v's timer fired in r-2, the read_oks of its peers, ascending (sent
// in r-1 with the peer's set after r-1): new values join S and P (deliverer:
// the peer); then one push per such peer carrying S & ~R if not empty; (5) the
// timer (reads to every neighbour); (6) at the end of a round with
// (r+1) % B == 0, v sends P to every out-neighbour w in one message, except to
// a w that delivered every value of P first (rebroadcastAllExcept's exclusion,
// per batch). pend_src tracks that: kNone (P empty), kMixed (several
// deliverers or a client), or the one deliverer. Partition windows drop
// messages as in parity mode; every delivered message is acked.
void gg_engine::compute_round_batched(Acc& a) {
    constexpr uint32_t kNone = ~0u, kMixed = ~0u - 1;
    const int64_t r = round;
    const uint64_t n_own = hi - lo;
    const bool sync = cfg.enable_sync != 0;
    const uint32_t W = (uint32_t)(nw * 64);
    auto& sp_all = seen[(r + 1) & 1];
    auto& sc_all = seen[r & 1];
    auto& Fp_all = F[(r + 1) & 1];
    auto& Fc_all = F[r & 1];
    std::fill(fired[r & 3].begin(), fired[r & 3].end(), 0ull);
    std::unordered_map<uint32_t, std::vector<uint32_t>> inj_by_node;
    {
        auto it = inj.find(r);
        if (it != inj.end()) {
            for (const auto& x : it->second) inj_by_node[x.node].push_back(x.lane);
            inj.erase(it);
        }
    }
    fired_nz[r & 3] = false;
    const bool tick = (r + 1) % (int64_t)cfg.batch_ticks == 0;
    std::vector<uint64_t> S(nw), sp(nw);
    std::vector<uint64_t> firedw;
    for (uint64_t i = 0; i < n_own; ++i) {
        const uint64_t g = lo + i;
        for (uint64_t j = 0; j < nw; ++j) sp[j] = S[j] = sp_all[i * nw + j];
        uint32_t& src = pend_src[i];
        auto deliver = [&](uint32_t d) { src = src == kNone ? d : (src == d ? src : kMixed); };
        auto ij = inj_by_node.find((uint32_t)g);  // (1) client broadcasts
        if (ij != inj_by_node.end())
            for (uint32_t lane : ij->second) {
                const uint64_t b = 1ull << (lane & 63);
                if (!(S[lane >> 6] & b)) src = kMixed;  // a client value goes to every neighbour
                S[lane >> 6] |= b;
            }
        for (int64_t e = in_ptr[i]; e < in_ptr[i + 1]; ++e) {  // (2) batches and pushes, ascending sender
            const uint64_t u = in_col[e];
            if (sync && fired_at(r - 1, u) && !masked(r - 1, u, g)) {  // u's read arrives, read_ok sent now
                a.read_oks++;
                if (masked(r, g, u)) a.node_dropped++;
            }
            if (masked(r - 1, u, g)) continue;  // dropped in flight
            const bool push = sync && fired_at(r - 3, u) && !masked(r - 3, u, g) && !masked(r - 2, g, u);
            const uint64_t* x = &Fp_all[u * nw];
            const uint64_t* y = &sp_all[u * nw];
            bool got = false;
            for (uint64_t j = 0; j < nw; ++j) {
                const uint64_t c = (x[j] | (push ? y[j] : 0ull)) & ~S[j];
                S[j] |= c;
                got |= c != 0;
            }
            if (got) deliver((uint32_t)u);
        }
        if (sync && fired_at(r - 2, g)) {  // (3) read_ok callbacks, ascending peer, then the pushes
            for (int pass = 0; pass < 2; ++pass)
                for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e) {
                    const uint64_t w = out_col[e];
                    if (masked(r - 2, g, w) || masked(r - 1, w, g)) continue;
                    const uint64_t* R = &sp_all[w * nw];
                    if (pass == 0) {
                        bool got = false;
                        for (uint64_t j = 0; j < nw; ++j) {
                            got |= (R[j] & ~S[j]) != 0;
                            S[j] |= R[j];
                        }
                        if (got) deliver((uint32_t)w);
                    } else {
                        bool any = false;
                        for (uint64_t j = 0; j < nw; ++j) any |= (S[j] & ~R[j]) != 0;
                        if (!any) continue;
                        a.pushes++;
                        if (masked(r, g, w)) {
                            a.dropped++;
                        } else {
                            a.push_deliv++;
                            a.next_acks++;
                            if (masked(r + 1, w, g)) a.next_ackdrop++;
                        }
                    }
                }
        }
        uint64_t* sc = &sc_all[i * nw];
        uint64_t* fc = &Fc_all[i * nw];
        uint64_t* P = &pend[i * nw];
        bool pend_any = false;
        for (uint64_t j = 0; j < nw; ++j) {
            sc[j] = S[j];
            const uint64_t f = S[j] & ~sp[j];
            a.new_bits += popc(f);
            if (f) a.hash += gg_word_hash(g * nw_g + w0 + j, f);
            if (f && !dr.empty()) {
                uint64_t y = f;
                while (y) {
                    int b = __builtin_ctzll(y);
                    y &= y - 1;
                    dr[i * W + j * 64 + b] = (int32_t)r;
                }
            }
            P[j] |= f;
            pend_any |= P[j] != 0;
            fc[j] = 0;
        }
        const uint64_t deg = (uint64_t)(out_ptr[i + 1] - out_ptr[i]);
        if (sync && r == sync_next[i]) {  // (5) sync timer: read RPC to every neighbour
            a.fired++;
            a.reads += deg;
            for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e)
                if (masked(r, g, out_col[e])) a.node_dropped++;
            firedw.push_back(g);
            sync_k[i]++;
            sync_next[i] = r + gg_sync_interval(cfg.seed, g, sync_k[i], cfg.sync_base_ticks, cfg.sync_jitter_ticks);
        }
        if (tick) {  // (6) the batch
            if (pend_any) {
                for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e) {
                    const uint64_t w = out_col[e];
                    if (src == (uint32_t)w) continue;  // w delivered every pending value: no message
                    a.fwd_sent++;
                    if (masked(r, g, w)) {
                        a.dropped++;
                    } else {
                        a.fwd_deliv++;
                        a.next_acks++;
                        if (masked(r + 1, w, g)) a.next_ackdrop++;
                    }
                }
                for (uint64_t j = 0; j < nw; ++j) {
                    fc[j] = P[j];
                    P[j] = 0;
                }
            }
            src = kNone;
        }
    }
    a.dropped += a.node_dropped;
    a.node_dropped = 0;
    for (uint64_t g : firedw) fired[r & 3][g >> 6] |= 1ull << (g & 63);
    fired_nz[r & 3] = !firedw.empty();
}

void gg_engine::compute_round(Acc& total) {
    const int64_t r = round;
    const uint64_t n_own = hi - lo;
    const uint64_t own0 = (uint64_t)part * slice;
    const bool sync = cfg.enable_sync != 0;
    const uint32_t W = (uint32_t)(nw * 64);  // this engine's lanes
    auto& sp_all = seen[(r + 1) & 1];  // seen_prev (round r-1)
    auto& sc_all = seen[r & 1];        // seen_cur
    auto& Fp_all = F[(r + 1) & 1];
    auto& Fc_all = F[r & 1];
    const uint8_t* act_p = act[(r + 1) & 1].data();
    uint8_t* act_c = act[r & 1].data();
    // fired slot of round r: owned words cleared here (world slices are refreshed by the exchange)
    {
        auto& fr = fired[r & 3];
        std::fill(fr.begin() + own0 / 64, fr.begin() + (own0 + slice) / 64, 0ull);
    }
    // injections of round r for owned nodes, grouped per node (call order kept)
    std::unordered_map<uint32_t, std::vector<uint32_t>> inj_by_node;
    {
        auto it = inj.find(r);
        if (it != inj.end()) {
            for (const auto& x : it->second)  // owned nodes, this lane group's values
                if (x.node >= lo && x.node < hi && (x.lane >> 6) >= w0 && (x.lane >> 6) < w0 + nw)
                    inj_by_node[x.node].push_back(x.lane - 64 * (uint32_t)w0);
            inj.erase(it);
        }
    }
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, n_own / 256 + 1));
    std::vector<Acc> accs(T);
    std::vector<std::vector<uint64_t>> firedw(T);
    // the windows of the rounds this one reads, and whether any timer fired in
    // r-1 (reads arriving now) and r-3 (pushes arriving now): hoisted out of the
    // per-edge loop, which is then one sender row per edge in lean rounds
    const Window *wm3 = window_at(r - 3), *wm2 = window_at(r - 2), *wm1 = window_at(r - 1);
    const Window *w00 = window_at(r), *wp1 = window_at(r + 1);
    const bool any_w = wm3 || wm2 || wm1 || w00 || wp1;
    const bool f1 = sync && fired_any(r - 1), f2 = sync && fired_any(r - 2), f3 = sync && fired_any(r - 3);
    const bool any_inj = !inj_by_node.empty();
    // nodes handed out in chunks (a sparse round's frontier sits in a few
    // ranges of ids): the counters are sums, so the order of the chunks is free
    std::atomic<uint64_t> next_chunk{0};
    constexpr uint64_t kChunk = 4096;
    auto work = [&](int t) {
        Acc& a = accs[t];
        std::vector<uint64_t> S(nw), sp(nw);
        constexpr uint64_t kAhead = 8;  // sender rows prefetched this many nodes ahead
        for (;;) {
        const uint64_t b0 = next_chunk.fetch_add(kChunk, std::memory_order_relaxed);
        if (b0 >= n_own) break;
        const uint64_t b1 = std::min(n_own, b0 + kChunk);
        for (uint64_t i = b0; i < b1; ++i) {
            const uint64_t g = lo + i, rep = own0 + i;
            if (i + kAhead < b1)
                for (int64_t e = in_ptr[i + kAhead]; e < in_ptr[i + kAhead + 1]; ++e) {
                    const uint64_t u = in_col[e];
                    if (act_p[u])
                        for (uint64_t j = 0; j < nw; j += 8) __builtin_prefetch(&Fp_all[u * nw + j]);
                }
            // A quiet node: nothing can reach it this round (no client broadcast, no
            // in-neighbour with an F row or a push, no sync callback) and its rows
            // did not change in r-1 or r-2, so both set buffers already hold its set
            // and its F row of r-2 is zero: the rows are neither read nor written
            // (the full path below would store the same bytes). Its counters are
            // the read_oks arriving and its own timer.
            bool quiet = !act_p[rep] && !act_c[rep] && !(f2 && fired_at(r - 2, rep)) &&
                         !(any_inj && inj_by_node.count((uint32_t)g));
            for (int64_t e = in_ptr[i]; quiet && e < in_ptr[i + 1]; ++e) {
                const uint64_t urep = in_col[e];
                if (act_p[urep] || (f3 && fired_at(r - 3, urep))) quiet = false;
            }
            if (quiet) {
                if (f1)
                    for (int64_t e = in_ptr[i]; e < in_ptr[i + 1]; ++e) {
                        const uint64_t urep = in_col[e];
                        const uint64_t u = any_w ? global_of(urep) : urep;
                        if (fired_at(r - 1, urep) && !masked_in(wm1, u, g)) {  // read arrives
                            a.read_oks++;                                      // HandleRead :131
                            if (masked_in(w00, g, u)) a.node_dropped++;
                        }
                    }
                if (sync && r == sync_next[i]) {  // (5) as below, with Tn = 0
                    const uint64_t deg = (uint64_t)(out_ptr[i + 1] - out_ptr[i]);
                    uint64_t mdrop = 0;
                    if (w00 || wp1)
                        for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e)
                            if (masked_in(w00, g, global_of(out_col[e]))) mdrop++;
                    a.fired++;
                    a.reads += deg;  // RPC read :120
                    a.node_dropped += mdrop;
                    firedw[t].push_back(rep);
                    sync_k[i]++;
                    sync_next[i] = r + gg_sync_interval(cfg.seed, g, sync_k[i], cfg.sync_base_ticks,
                                                        cfg.sync_jitter_ticks);
                }
                continue;
            }
            const uint64_t* spv = &sp_all[rep * nw];
            for (uint64_t j = 0; j < nw; ++j) sp[j] = S[j] = spv[j];
            // (1) client broadcasts
            if (any_inj) {
                auto ij = inj_by_node.find((uint32_t)g);
                if (ij != inj_by_node.end())
                    for (uint32_t lane : ij->second) S[lane >> 6] |= 1ull << (lane & 63);
            }
            // (2) node broadcasts, ascending sender
            uint64_t cl_recip = 0, cl_deliv = 0, cl_ackdrop = 0;
            for (int64_t e = in_ptr[i]; e < in_ptr[i + 1]; ++e) {
                const uint64_t urep = in_col[e];
                const uint64_t u = any_w ? global_of(urep) : urep;  // (only the masks read it)
                if (f1 && fired_at(r - 1, urep) && !masked_in(wm1, u, g)) {  // read arrives
                    a.read_oks++;                                          // HandleRead :131
                    if (masked_in(w00, g, u)) a.node_dropped++;
                }
                if (masked_in(wm1, u, g)) continue;                        // dropped in flight
                const bool push = f3 && fired_at(r - 3, urep) && !masked_in(wm3, u, g) &&
                                  !masked_in(wm2, g, u);
                if (!push && !act_p[urep]) continue;  // its F row is zero: nothing to claim
                const uint64_t* src = push ? &sp_all[urep * nw] : &Fp_all[urep * nw];
                uint64_t pc = 0;
                for (uint64_t j = 0; j < nw; ++j) {
                    uint64_t c = src[j] & ~S[j];
                    S[j] |= c;
                    pc += popc(c);
                }
                if (pc && recip(e)) {
                    cl_recip += pc;
                    if (!masked_in(w00, g, u)) {
                        cl_deliv += pc;
                        if (masked_in(wp1, u, g)) cl_ackdrop += pc;
                    }
                }
            }
            // (3) sync callback: fired in r-2, peers ascending
            uint64_t cb_new = 0, cb_new_deliv = 0, cb_new_ackdrop = 0;
            uint64_t push_sent = 0, push_deliv = 0, push_ackdrop = 0;
            if (f2 && fired_at(r - 2, rep)) {
                for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e) {
                    const uint64_t wrep = out_col[e];
                    const uint64_t w = global_of(wrep);
                    if (masked_in(wm2, g, w) || masked_in(wm1, w, g)) continue;
                    const uint64_t* R = &sp_all[wrep * nw];
                    uint64_t pn = 0, pp = 0;
                    for (uint64_t j = 0; j < nw; ++j) {
                        pn += popc(R[j] & ~S[j]);
                        pp += popc(S[j] & ~R[j]);
                        S[j] |= R[j];
                    }
                    cb_new += pn;
                    push_sent += pp;
                    if (!masked_in(w00, g, w)) {
                        cb_new_deliv += pn;
                        push_deliv += pp;
                        if (masked_in(wp1, w, g)) {
                            cb_new_ackdrop += pn;
                            push_ackdrop += pp;
                        }
                    }
                }
            }
            // state
            uint64_t* sc = &sc_all[rep * nw];
            uint64_t* fc = &Fc_all[rep * nw];
            uint64_t Tn = 0;
            for (uint64_t j = 0; j < nw; ++j) {
                sc[j] = S[j];
                uint64_t f = S[j] & ~sp[j];
                fc[j] = f;
                Tn += popc(f);
                if (f) a.hash += gg_word_hash(g * nw_g + w0 + j, f);
                if (f && !dr.empty()) {
                    uint64_t x = f;
                    while (x) {
                        int b = __builtin_ctzll(x);
                        x &= x - 1;
                        dr[i * W + j * 64 + b] = (int32_t)r;
                    }
                }
            }
            act_c[rep] = Tn != 0;
            a.new_bits += Tn;
            // counts of what v sends in round r
            const uint64_t deg = (uint64_t)(out_ptr[i + 1] - out_ptr[i]);
            uint64_t U = deg, AD = 0, mdrop = 0;
            if (w00 || wp1) {
                U = 0;
                for (int64_t e = out_ptr[i]; e < out_ptr[i + 1]; ++e) {
                    const uint64_t w = global_of(out_col[e]);
                    if (!masked_in(w00, g, w)) {
                        U++;
                        if (masked_in(wp1, w, g)) AD++;
                    } else {
                        mdrop++;
                    }
                }
            }
            const uint64_t fs = deg * Tn - cl_recip - cb_new;
            const uint64_t fd = U * Tn - cl_deliv - cb_new_deliv;
            a.fwd_sent += fs;
            a.fwd_deliv += fd;
            a.pushes += push_sent;
            a.push_deliv += push_deliv;
            a.dropped += (fs - fd) + (push_sent - push_deliv);
            a.next_acks += fd + push_deliv;
            a.next_ackdrop += AD * Tn - cl_ackdrop - cb_new_ackdrop + push_ackdrop;
            // (5) sync timer
            if (sync && r == sync_next[i]) {
                a.fired++;
                a.reads += deg;                                          // RPC read :120
                a.node_dropped += mdrop;
                firedw[t].push_back(rep);
                sync_k[i]++;
                sync_next[i] = r + gg_sync_interval(cfg.seed, g, sync_k[i], cfg.sync_base_ticks,
                                                    cfg.sync_jitter_ticks);
            }
        }
        }  // chunks
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t) {
        if (lgrp != 0) {  // node-level events are counted by lane group 0 only
            accs[t].reads = accs[t].read_oks = accs[t].fired = accs[t].node_dropped = 0;
        }
        accs[t].dropped += accs[t].node_dropped;
        accs[t].node_dropped = 0;
        total.add(accs[t]);
        for (uint64_t rep : firedw[t]) fired[r & 3][rep >> 6] |= 1ull << (rep & 63);
    }
    // the slot's own words; a vertex part ORs its peers' in at gg_dist_round_end
    fired_nz[r & 3] = false;
    for (int t = 0; t < T; ++t) fired_nz[r & 3] |= !firedw[t].empty();
}

// --------------------------------------------------------------------------

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
    if (cfg->world / L > 63) return GG_EINVAL;  // the HIP engine's exchange limit (same ABI)
    if (cfg->batch_ticks && cfg->world != 1) return GG_EINVAL;  // batched gossip: one engine
    auto* e = new gg_engine();
    e->cfg = *cfg;
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
    e->threads = default_threads();
    *out = e;
    return GG_OK;
}

void gg_destroy(gg_engine* e) { delete e; }

const char* gg_last_error(const gg_engine* e) { return e ? e->err.c_str() : "null engine"; }

int gg_topology(gg_engine* e, const int64_t* row_ptr, const int32_t* col, uint64_t nnz) {
    if (!e || !row_ptr || (nnz && !col)) return GG_EINVAL;
    const uint64_t V = e->V;
    const int T = e->threads;
    if (row_ptr[0] != 0 || (uint64_t)row_ptr[V] != nnz) return e->fail(GG_EINVAL, "row_ptr[0]/row_ptr[V] mismatch");
    {  // rows monotone, ids in range, each row ascending and unique (the first bad row reports)
        std::vector<uint64_t> bad_v(std::max(T, 1), V);
        std::vector<const char*> bad_m(std::max(T, 1), nullptr);
        pfor(T, V, [&](int t, uint64_t v0, uint64_t v1) {
            for (uint64_t v = v0; v < v1; ++v) {
                const char* m = nullptr;
                if (row_ptr[v + 1] < row_ptr[v]) {
                    m = "row_ptr not monotone";
                } else {
                    for (int64_t k = row_ptr[v]; k < row_ptr[v + 1] && !m; ++k) {
                        if (col[k] < 0 || (uint64_t)col[k] >= V) m = "neighbour id out of range";
                        else if (k > row_ptr[v] && col[k] <= col[k - 1]) m = "neighbour list not ascending/unique";
                    }
                }
                if (m) {
                    bad_v[t] = v;
                    bad_m[t] = m;
                    return;
                }
            }
        });
        uint64_t bv = V;
        const char* bm = nullptr;
        for (size_t t = 0; t < bad_v.size(); ++t)
            if (bad_m[t] && bad_v[t] < bv) bv = bad_v[t], bm = bad_m[t];
        if (bm) return e->fail(GG_EINVAL, bm);
    }
    // symmetric iff every link u -> v has its v -> u (rows are ascending and unique)
    bool sym = true;
    {
        std::atomic<bool> asym{false};
        pfor(T, V, [&](int, uint64_t u0, uint64_t u1) {
            for (uint64_t u = u0; u < u1 && !asym.load(std::memory_order_relaxed); ++u)
                for (int64_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) {
                    const int32_t v = col[k];
                    if (!std::binary_search(col + row_ptr[v], col + row_ptr[v + 1], (int32_t)u)) {
                        asym = true;
                        break;
                    }
                }
        });
        sym = !asym;
    }
    e->symmetric = sym;
    e->windows.erase(std::remove_if(e->windows.begin(), e->windows.end(), [](const Window& w) { return w.edges; }),
                     e->windows.end());
    // in-lists ascending by sender: the rows themselves when symmetric, else the transpose
    std::vector<int64_t> tin_s;
    std::vector<uint32_t> tcol_s;
    const int64_t* tin = row_ptr;
    const uint32_t* tcol = reinterpret_cast<const uint32_t*>(col);
    if (!sym) {
        tin_s.assign(V + 1, 0);
        for (uint64_t k = 0; k < nnz; ++k) tin_s[col[k] + 1]++;
        for (uint64_t v = 0; v < V; ++v) tin_s[v + 1] += tin_s[v];
        tcol_s.resize(nnz);
        std::vector<int64_t> pos(tin_s.begin(), tin_s.end() - 1);
        for (uint64_t u = 0; u < V; ++u)
            for (int64_t k = row_ptr[u]; k < row_ptr[u + 1]; ++k) tcol_s[pos[col[k]]++] = (uint32_t)u;
        tin = tin_s.data();
        tcol = tcol_s.data();
    }
    // edge-balanced vertex ranges over the in-lists (pull work)
    const uint32_t Wd = e->P;  // vertex parts of this lane group
    e->rank_lo.assign(Wd + 1, V);
    e->rank_lo[0] = 0;
    {
        const uint64_t total = nnz + V;
        uint32_t p = 1;
        for (uint64_t v = 0; v < V && p < Wd; ++v) {
            uint64_t cum = (uint64_t)tin[v + 1] + v + 1;
            while (p < Wd && cum >= total * p / Wd) e->rank_lo[p++] = v + 1;
        }
        while (p < Wd) e->rank_lo[p++] = V;
    }
    uint64_t maxrows = 0;
    for (uint32_t p = 0; p < Wd; ++p) maxrows = std::max<uint64_t>(maxrows, e->rank_lo[p + 1] - e->rank_lo[p]);
    e->slice = std::max<uint64_t>(64, (maxrows + 63) / 64 * 64);
    e->lo = e->rank_lo[e->part];
    e->hi = e->rank_lo[e->part + 1];
    const uint64_t n_own = e->hi - e->lo;
    // copy helpers (every thread: the full-size configs hold 6.4e9 entries)
    auto copy_ptr = [&](auto& dst, const int64_t* src, uint64_t n) {
        dst.resize(n);
        pfor(T, n, [&](int, uint64_t i0, uint64_t i1) { std::copy(src + i0, src + i1, dst.begin() + i0); });
    };
    e->s_optr.clear(); e->s_ocol.clear(); e->s_crp.clear(); e->s_ccol.clear();
    e->in_recip.clear();
    if (Wd == 1 && sym) {
        // one part (replica index = global id) of a symmetric graph: ONE copy of the
        // caller's rows serves as in-lists, out-lists and the per-edge window CSR
        copy_ptr(e->s_ptr, row_ptr, V + 1);
        e->s_col.resize(nnz);
        pfor(T, nnz, [&](int, uint64_t i0, uint64_t i1) {
            for (uint64_t k = i0; k < i1; ++k) e->s_col[k] = (uint32_t)col[k];
        });
        e->in_ptr.of(e->s_ptr);
        e->in_col.of(e->s_col);
        e->out_ptr = e->in_ptr;
        e->out_col = e->in_col;
        e->crp.of(e->s_ptr);
        e->ccol.of(e->s_col);
    } else {
        copy_ptr(e->s_crp, row_ptr, V + 1);
        e->s_ccol.assign(col, col + nnz);
        e->crp.of(e->s_crp);
        e->ccol.of(e->s_ccol);
        // owned rows with replica column ids
        e->s_ptr.assign(n_own + 1, 0);
        e->s_optr.assign(n_own + 1, 0);
        for (uint64_t i = 0; i < n_own; ++i) {
            e->s_ptr[i + 1] = e->s_ptr[i] + (tin[e->lo + i + 1] - tin[e->lo + i]);
            e->s_optr[i + 1] = e->s_optr[i] + (row_ptr[e->lo + i + 1] - row_ptr[e->lo + i]);
        }
        e->s_col.resize(e->s_ptr[n_own]);
        if (!sym) e->in_recip.resize(e->s_ptr[n_own]);  // symmetric: every in-edge is reciprocal
        e->s_ocol.resize(e->s_optr[n_own]);
        for (uint64_t i = 0; i < n_own; ++i) {
            const uint64_t v = e->lo + i;
            const int32_t* ob = col + row_ptr[v];
            const int32_t* oe = col + row_ptr[v + 1];
            for (int64_t k = 0; k < tin[v + 1] - tin[v]; ++k) {
                uint32_t u = tcol[tin[v] + k];
                e->s_col[e->s_ptr[i] + k] = (uint32_t)e->rep_of(u);
                if (!sym) e->in_recip[e->s_ptr[i] + k] = std::binary_search(ob, oe, (int32_t)u) ? 1 : 0;
            }
            for (int64_t k = 0; k < row_ptr[v + 1] - row_ptr[v]; ++k)
                e->s_ocol[e->s_optr[i] + k] = (uint32_t)e->rep_of((uint64_t)ob[k]);
        }
        e->in_ptr.of(e->s_ptr);
        e->in_col.of(e->s_col);
        e->out_ptr.of(e->s_optr);
        e->out_col.of(e->s_ocol);
    }
    const uint64_t rows = (uint64_t)Wd * e->slice;
    for (int b = 0; b < 2; ++b) {  // zeroed by reset_state below
        e->seen[b].resize(rows * e->nw);
        e->F[b].resize(rows * e->nw);
        e->act[b].resize(rows);
    }
    for (int b = 0; b < 4; ++b) e->fired[b].assign(rows / 64, 0);
    e->sync_next.resize(n_own);
    e->sync_k.resize(n_own);
    if (e->cfg.flags & GG_TRACK_DELIVERY) e->dr.assign(n_own * e->nw * 64, -1);
    else e->dr.clear();
    e->pend.assign(e->cfg.batch_ticks ? n_own * e->nw : 0, 0ull);
    e->pend_src.assign(e->cfg.batch_ticks ? n_own : 0, ~0u);
    e->have_topo = true;
    e->reset_state();
    return GG_OK;
}

static int add_window(gg_engine* e, int64_t a, int64_t b, Window&& w) {
    if (!e) return GG_EINVAL;
    if (a >= b) return e->fail(GG_EINVAL, "empty partition window");
    for (const auto& x : e->windows)  // per-edge windows may overlap group windows (and win)
        if (x.edges == w.edges && a < x.to && x.from < b) return e->fail(GG_EINVAL, "overlapping partition windows");
    w.from = a;
    w.to = b;
    e->windows.push_back(std::move(w));
    return GG_OK;
}

int gg_partition_seeded(gg_engine* e, int64_t a, int64_t b, uint64_t epoch_seed) {
    Window w;
    w.seeded = true;
    w.epoch_seed = epoch_seed;
    return add_window(e, a, b, std::move(w));
}

int gg_set_partition(gg_engine* e, int64_t a, int64_t b, const uint64_t* bits) {
    if (!e || !bits) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "gg_set_partition: install the topology first");
    if (!e->symmetric) return e->fail(GG_EINVAL, "gg_set_partition: per-edge windows need a symmetric topology");
    const uint64_t E = e->ccol.size();
    Window w;
    w.seeded = false;
    w.epoch_seed = 0;
    w.edges = true;
    w.bits.assign(bits, bits + (E + 63) / 64);
    auto bit = [&](uint64_t k) { return (bits[k >> 6] >> (k & 63)) & 1ull; };
    for (uint64_t u = 0; u < e->V; ++u)
        for (int64_t k = e->crp[u]; k < e->crp[u + 1]; ++k) {
            const uint64_t v = (uint64_t)e->ccol[k];
            const int32_t* r0 = e->ccol.data() + e->crp[v];
            const int32_t* r1 = e->ccol.data() + e->crp[v + 1];
            const uint64_t kr = (uint64_t)e->crp[v] + (uint64_t)(std::lower_bound(r0, r1, (int32_t)u) - r0);
            if (bit((uint64_t)k) != bit(kr)) return e->fail(GG_EINVAL, "gg_set_partition: the mask is not symmetric");
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

int gg_broadcast(gg_engine* e, uint32_t node, int64_t message, int64_t round) {
    if (!e) return GG_EINVAL;
    if (node >= e->V) return e->fail(GG_EINVAL, "node out of range");
    if (round < e->round) return e->fail(GG_EINVAL, "broadcast scheduled in the past");
    auto it = e->lanes.find(message);
    uint32_t lane;
    if (it == e->lanes.end()) {
        if (e->lane_value.size() >= e->cfg.n_lanes) return e->fail(GG_ENOSPC, "all message lanes in use");
        lane = (uint32_t)e->lane_value.size();
        e->lanes.emplace(message, lane);
        e->lane_value.push_back(message);
    } else {
        lane = it->second;
    }
    e->inj[round].push_back({node, lane});
    return GG_OK;
}

int gg_broadcast_many(gg_engine* e, const uint32_t* nodes, const int64_t* messages,
                      const int64_t* rounds, uint64_t n) {
    if (!e || (n && (!nodes || !messages || !rounds))) return GG_EINVAL;
    for (uint64_t k = 0; k < n; ++k) {
        int rc = gg_broadcast(e, nodes[k], messages[k], rounds[k]);
        if (rc) return rc;
    }
    return GG_OK;
}

int gg_lane_of(const gg_engine* e, int64_t message) {
    if (!e) return GG_EINVAL;
    auto it = e->lanes.find(message);
    return it == e->lanes.end() ? GG_EINVAL : (int)it->second;
}

int64_t gg_current_round(const gg_engine* e) { return e ? e->round : -1; }

static void fill_stats(gg_engine* e, const Acc& a, gg_round_stats* s) {
    s->round = e->round;
    s->new_bits = a.new_bits;
    s->fwd_sent = a.fwd_sent;
    s->fwd_delivered = a.fwd_deliv;
    s->pushes = a.pushes;
    s->push_delivered = a.push_deliv;
    s->acks = e->pend_acks;
    s->reads = a.reads;
    s->read_oks = a.read_oks;
    s->dropped = a.dropped + e->pend_ackdrop;
    s->syncs_fired = a.fired;
    e->hash_total += a.hash;
    s->seen_hash = e->hash_total;
    s->kernel_ms = 0.0;
    s->work_rows = 0;
    s->work_gathers = 0;
    s->prep_ms = s->expand_ms = s->stream_ms = 0.0;
    s->prep_bytes = s->expand_bytes = s->stream_bytes = 0;
    s->sent_bytes = e->dist_open ? e->xsend_sent : 0;
    s->path = 0;
}

int gg_step(gg_engine* e, uint32_t n, gg_round_stats* out) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P != 1) return e->fail(GG_EINVAL, "vertex-sharded engine: use gg_dist_round_begin/end");
    for (uint32_t k = 0; k < n; ++k) {
        Acc a;
        if (e->cfg.batch_ticks) e->compute_round_batched(a);
        else e->compute_round(a);
        gg_round_stats s;
        fill_stats(e, a, &s);
        if (out) out[k] = s;
        e->pend_acks = a.next_acks;
        e->pend_ackdrop = a.next_ackdrop;
        e->round++;
    }
    return GG_OK;
}

int gg_step_device_ms(const gg_engine* e, double* ms) {
    if (!e || !ms) return GG_EINVAL;
    *ms = 0.0;  // no device
    return GG_OK;
}

// gossip.h: episodes x (gg_reset; the schedule held now; gg_step(n_rounds)).
int gg_run_episodes(gg_engine* e, uint32_t n_rounds, uint32_t episodes, gg_round_stats* out) {
    if (!e) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->P != 1) return e->fail(GG_EINVAL, "vertex-sharded engine: use gg_dist_round_begin/end");
    if (e->round != 0) return e->fail(GG_EINVAL, "gg_run_episodes: call it right after gg_reset and the broadcasts");
    if (n_rounds < 1 || n_rounds > 256 || episodes < 1) return e->fail(GG_EINVAL, "gg_run_episodes: bad sizes");
    const auto inj0 = e->inj;
    const auto lanes0 = e->lanes;
    const auto lv0 = e->lane_value;
    for (uint32_t k = 0; k < episodes; ++k) {
        if (k) {
            int rc = gg_reset(e);
            if (rc) return rc;
            e->inj = inj0;
            e->lanes = lanes0;
            e->lane_value = lv0;
        }
        int rc = gg_step(e, n_rounds, out ? out + (size_t)k * n_rounds : nullptr);
        if (rc) return rc;
    }
    return GG_OK;
}

int gg_dist_info(const gg_engine* e, uint64_t* n_own, uint64_t* n_ghost, uint64_t* n_send) {
    if (!e || !e->have_topo) return GG_EINVAL;
    const uint64_t n = e->hi - e->lo;
    if (n_own) *n_own = n;
    if (n_ghost) *n_ghost = e->P > 1 ? e->V - n : 0;  // full replicas
    if (n_send) *n_send = e->P > 1 ? n * (e->P - 1) : 0;
    return GG_OK;
}

int gg_dist_owned(const gg_engine* e, uint32_t* nodes, uint64_t cap, uint64_t* n_out) {
    if (!e || !e->have_topo) return GG_EINVAL;
    const uint64_t n = e->hi - e->lo;
    if (n_out) *n_out = n;
    if (nodes)
        for (uint64_t i = 0; i < n && i < cap; ++i) nodes[i] = (uint32_t)(e->lo + i);
    return GG_OK;
}

// payload of one node: seen row, F row (nw words each), fired byte (8-byte slot)
static uint64_t node_payload(const gg_engine* e) { return (2 * e->nw + 1) * 8; }

int gg_dist_round_begin(gg_engine* e, gg_exchange* x) {
    if (!e || !x) return GG_EINVAL;
    if (!e->have_topo) return e->fail(GG_EINVAL, "no topology");
    if (e->dist_open) return e->fail(GG_EINVAL, "round already open");
    e->dist_acc = Acc();
    e->compute_round(e->dist_acc);
    const int64_t r = e->round;
    const uint64_t pb = node_payload(e), n_own = e->hi - e->lo, own0 = (uint64_t)e->part * e->slice;
    e->xsend_bytes.assign(e->world, 0);
    e->xrecv_bytes.assign(e->world, 0);
    uint64_t st = 0, rt = 0;
    for (uint32_t q = 0; q < e->P; ++q) {  // peers: the other parts of this lane group
        if (q == e->part) continue;
        e->xsend_bytes[e->peer_rank(q)] = n_own * pb;
        e->xrecv_bytes[e->peer_rank(q)] = (e->rank_lo[q + 1] - e->rank_lo[q]) * pb;
        st += n_own * pb;
        rt += (e->rank_lo[q + 1] - e->rank_lo[q]) * pb;
    }
    e->xsend.assign(std::max<uint64_t>(1, st), 0);
    e->xsend_sent = st;
    e->xrecv.assign(std::max<uint64_t>(1, rt), 0);
    uint8_t* p = e->xsend.data();
    for (uint32_t q = 0; q < e->P; ++q) {
        if (q == e->part) continue;
        for (uint64_t i = 0; i < n_own; ++i, p += pb) {
            const uint64_t rep = own0 + i;
            std::memcpy(p, &e->seen[r & 1][rep * e->nw], e->nw * 8);
            std::memcpy(p + e->nw * 8, &e->F[r & 1][rep * e->nw], e->nw * 8);
            p[2 * e->nw * 8] = e->fired_at(r, rep) ? 1 : 0;
        }
    }
    e->xsend_off.assign(e->world, 0);  // segments contiguous in rank order (static sizes)
    e->xrecv_off.assign(e->world, 0);
    for (uint32_t q = 1; q < e->world; ++q) {
        e->xsend_off[q] = e->xsend_off[q - 1] + e->xsend_bytes[q - 1];
        e->xrecv_off[q] = e->xrecv_off[q - 1] + e->xrecv_bytes[q - 1];
    }
    x->send = e->xsend.data();
    x->recv = e->xrecv.data();
    x->send_bytes = e->xsend_bytes.data();
    x->recv_bytes = e->xrecv_bytes.data();
    x->send_off = e->xsend_off.data();
    x->recv_off = e->xrecv_off.data();
    x->exact = 0;
    x->send_total = st;
    x->recv_total = rt;
    x->on_device = 0;
    x->stream = nullptr;
    e->dist_open = true;
    return GG_OK;
}

int gg_dist_round_end(gg_engine* e, gg_round_stats* out) {
    if (!e || !e->dist_open) return GG_EINVAL;
    const int64_t r = e->round;
    const uint64_t pb = node_payload(e);
    const uint8_t* p = e->xrecv.data();
    for (uint32_t q = 0; q < e->P; ++q) {
        if (q == e->part) continue;
        for (uint64_t g = e->rank_lo[q]; g < e->rank_lo[q + 1]; ++g, p += pb) {
            const uint64_t rep = (uint64_t)q * e->slice + (g - e->rank_lo[q]);
            std::memcpy(&e->seen[r & 1][rep * e->nw], p, e->nw * 8);
            std::memcpy(&e->F[r & 1][rep * e->nw], p + e->nw * 8, e->nw * 8);
            e->act[r & 1][rep] = 0;
            for (uint64_t j = 0; j < e->nw; ++j) e->act[r & 1][rep] |= e->F[r & 1][rep * e->nw + j] != 0;
            uint64_t& w = e->fired[r & 3][rep >> 6];
            if (p[2 * e->nw * 8]) {
                w |= 1ull << (rep & 63);
                e->fired_nz[r & 3] = true;
            } else {
                w &= ~(1ull << (rep & 63));
            }
        }
    }
    gg_round_stats s;
    fill_stats(e, e->dist_acc, &s);
    if (out) *out = s;
    else e->dist_pending.push_back(s);
    e->pend_acks = e->dist_acc.next_acks;
    e->pend_ackdrop = e->dist_acc.next_ackdrop;
    e->round++;
    e->dist_open = false;
    return GG_OK;
}

int gg_dist_flush(gg_engine* e, gg_round_stats* out, uint64_t cap, uint64_t* n_out) {
    if (!e) return GG_EINVAL;
    const uint64_t n = e->dist_pending.size();
    if (n_out) *n_out = n;
    if (!out) return GG_OK;  // count only
    if (cap < n) return e->fail(GG_EINVAL, "stats buffer too small");
    for (uint64_t i = 0; i < n; ++i) out[i] = e->dist_pending[i];
    e->dist_pending.clear();
    return GG_OK;
}

// The engine-owned RCCL exchange is GPU-only: the oracle's ranks exchange
// through the caller (gg_dist_round_begin/end) and these report GG_EIO.
int gg_dist_comm_available(char* why, uint64_t cap) {
    if (why && cap) std::snprintf(why, cap, "%s", "CPU oracle: no RCCL");
    return GG_EIO;
}
int gg_dist_comm_id(const gg_engine*, uint8_t*) { return GG_EIO; }
int gg_dist_ipc_export(gg_engine*, uint8_t*) { return GG_EIO; }  // no device memory to map
int gg_dist_ipc_import(gg_engine*, const uint8_t*) { return GG_EIO; }
int gg_dist_ipc_close(gg_engine* e) { return e ? GG_OK : GG_EINVAL; }  // nothing mapped
int gg_dist_comm_init(gg_engine* e, const uint8_t*) { return e ? e->fail(GG_EIO, "CPU oracle: no RCCL") : GG_EINVAL; }
int gg_dist_step(gg_engine* e, uint32_t) { return e ? e->fail(GG_EIO, "CPU oracle: no RCCL") : GG_EINVAL; }
int gg_dist_run_episodes(gg_engine* e, uint32_t, uint32_t, gg_round_stats*) {
    return e ? e->fail(GG_EIO, "CPU oracle: no device-driven exchange") : GG_EINVAL;
}
int gg_topology_part(gg_engine* e, const uint64_t*, const int64_t*, const int32_t*, uint64_t) {
    return e ? e->fail(GG_ENOSYS, "CPU oracle: sharded engines take the whole graph (gg_topology)") : GG_EINVAL;
}
int gg_topology_part_directed(gg_engine* e, const uint64_t*, const int64_t*, const int32_t*, uint64_t) {
    return e ? e->fail(GG_ENOSYS, "CPU oracle: sharded engines take the whole graph (gg_topology)") : GG_EINVAL;
}
int gg_dist_transport_init(gg_engine* e, const gg_transport*) {
    return e ? e->fail(GG_EIO, "CPU oracle: the engine-driven exchange is the HIP engine's") : GG_EINVAL;
}

static bool owned(const gg_engine* e, uint64_t a, uint64_t b) { return a <= b && a >= e->lo && b <= e->hi; }

int gg_read(gg_engine* e, uint32_t node, int64_t* out, uint64_t cap, uint64_t* n_out) {
    if (!e || !e->have_topo) return GG_EINVAL;
    if (!owned(e, node, (uint64_t)node + 1)) return e->fail(GG_EINVAL, "node not owned by this engine");
    const uint64_t rep = (uint64_t)e->part * e->slice + (node - e->lo);
    const auto& sc = e->seen[(e->round + 1) & 1];  // last completed round
    std::vector<int64_t> vals;  // a lane-group engine: the values of its own lanes
    for (uint64_t j = 0; j < e->nw; ++j) {
        uint64_t x = sc[rep * e->nw + j];
        while (x) {
            int b = __builtin_ctzll(x);
            x &= x - 1;
            uint64_t lane = (e->w0 + j) * 64 + b;
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
    if (!e || !e->have_topo || !out) return GG_EINVAL;
    if (!owned(e, a, b)) return e->fail(GG_EINVAL, "range not owned by this engine");
    const auto& sc = e->seen[(e->round + 1) & 1];
    const uint64_t rep = (uint64_t)e->part * e->slice + (a - e->lo);
    for (uint64_t k = 0; k < (uint64_t)(b - a); ++k) {  // whole-job words, own window filled
        std::fill(out + k * e->nw_g, out + (k + 1) * e->nw_g, 0ull);
        std::memcpy(out + k * e->nw_g + e->w0, &sc[(rep + k) * e->nw], e->nw * 8);
    }
    return GG_OK;
}

int gg_delivery_rounds(gg_engine* e, uint32_t a, uint32_t b, int32_t* out, uint64_t cap) {
    if (!e || !e->have_topo || !out) return GG_EINVAL;
    if (e->dr.empty()) return e->fail(GG_EINVAL, "GG_TRACK_DELIVERY not enabled");
    if (!owned(e, a, b)) return e->fail(GG_EINVAL, "range not owned by this engine");
    const uint64_t W = e->cfg.n_lanes, Wl = e->nw * 64;
    const uint64_t n = (uint64_t)(b - a) * W;
    if (cap < n) return e->fail(GG_EINVAL, "output buffer too small");
    std::fill(out, out + n, -1);
    for (uint64_t k = 0; k < (uint64_t)(b - a); ++k)
        std::memcpy(out + k * W + 64 * e->w0, &e->dr[(a - e->lo + k) * Wl], Wl * 4);
    return GG_OK;
}

int gg_read_bits_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, uint64_t* out) {
    if (!e || !e->have_topo || (n && (!nodes || !out))) return GG_EINVAL;
    for (uint64_t k = 0; k < n; ++k) {
        int rc = gg_read_bits(e, nodes[k], nodes[k] + 1, out + k * e->nw_g);
        if (rc) return rc;
    }
    return GG_OK;
}

int gg_delivery_rounds_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, int32_t* out) {
    if (!e || !e->have_topo || (n && (!nodes || !out))) return GG_EINVAL;
    for (uint64_t k = 0; k < n; ++k) {
        int rc = gg_delivery_rounds(e, nodes[k], nodes[k] + 1, out + k * e->cfg.n_lanes, e->cfg.n_lanes);
        if (rc) return rc;
    }
    return GG_OK;
}

int gg_reset(gg_engine* e) {
    if (!e) return GG_EINVAL;
    if (e->have_topo) e->reset_state();
    e->dist_pending.clear();
    return GG_OK;
}

int gg_device_bytes(const gg_engine* e, uint64_t* total, uint64_t* sync_part) {  // no device memory
    if (!e) return GG_EINVAL;
    if (total) *total = 0;
    if (sync_part) *sync_part = 0;
    return GG_OK;
}

}  // extern "C"
