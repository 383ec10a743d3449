/*
 * gossip.h — C ABI of the MI355X gossip-propagation engine.
 *
 * Drop-in boundary for the hot path of dshebib/gossip-glomers-distributed-systems
 * `broadcast/` (the Gossip Glomers "broadcast" challenge solution). The reference
 * registers five maelstrom handlers per node (`broadcast/main.go:22-40`) and runs
 * one OS process per node; this engine runs every node of a topology in lockstep
 * 100 ms rounds (one round = one simulated latency tick) on one or more GPUs.
 *
 * Entry point                 replaces (reference file:line)
 * ---------------------------------------------------------------------------
 * gg_create                   maelstrom.NewNode + Context{} + handler table
 *                             `broadcast/main.go:17-40`; sync timer `main.go:42-51`
 * gg_topology                 HandleTopology `broadcast/broadcast.go:36-48`
 *                             (every node keeps its own row; here: all rows at once)
 * gg_partition_seeded /       Maelstrom `--nemesis partition` (external harness,
 * gg_partition_groups /       `README.md:18`): messages across groups (or over cut
 * gg_set_partition            links) are dropped; no retry (`broadcast.go:55`)
 * gg_broadcast                client `broadcast` -> HandleBroadcast `broadcast.go:59-79`
 * gg_step                     n lockstep rounds: every HandleBroadcast /
 *                             rebroadcastAllExcept (`:50-57`) / SyncBroadcast
 *                             (`:81-122`) / HandleRead (`:124-132`) / broadcast_ok
 *                             (`main.go:38-40`) event of those rounds
 * gg_run_episodes             repeated gg_reset + broadcasts + gg_step with one host
 *                             wait (a workload replayed many times; new)
 * gg_read / gg_read_bits      client `read` -> HandleRead `broadcast.go:124-132`
 * gg_delivery_rounds          observation only (first round each value was seen)
 * gg_dist_*                   one engine per GPU: locality-ordered vertex ranges with
 *                             ghost copies of adjacent remote nodes (new)
 *
 * Determinization contract (restated in DESIGN.md §2):
 * one round per 100 ms tick; every message sent in round r is delivered in
 * round r+1 unless the partition plan drops it (evaluated at the send round);
 * within a round a node handles client broadcasts, then node broadcasts in
 * ascending sender id, then sync read_ok callbacks in ascending peer id, then
 * read requests (answered with the end-of-round set), then its sync timer.
 *
 * Conventions: 0 = success; negative errno on failure (GG_EINVAL, GG_ENOMEM,
 * GG_EIO for HIP/driver failures, GG_ENOSPC when more distinct message values
 * than lanes were broadcast) and gg_last_error() describes it — the analogue of a
 * handler returning an error. All inputs are caller-owned and copied; outputs go
 * to caller buffers. One engine is driven by one host thread.
 *
 * Two libraries export exactly these symbols: libgossip_hip.so (the product,
 * HIP kernels for gfx950) and oracle/_build/libgossip_cpu.so (the CPU bitset
 * restatement, used only by tests and the CPU baseline).
 */
#ifndef GOSSIP_H_
#define GOSSIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GG_ABI_VERSION 7

#define GG_OK 0
#define GG_EIO (-5)
#define GG_ENOMEM (-12)
#define GG_EINVAL (-22)
#define GG_ENOSPC (-28)
#define GG_ENOSYS (-38)

/* gg_config.flags */
#define GG_TRACK_DELIVERY 1u /* keep the first-seen round of every (node,lane) */

typedef struct gg_engine gg_engine; /* opaque; owns all device memory */

typedef struct {
    uint64_t n_nodes;           /* V: node ids 0..V-1 ("n0".."n<V-1>") */
    uint32_t n_lanes;           /* W: message lanes, multiple of 64, 64..8192 */
    uint32_t flags;             /* GG_TRACK_DELIVERY */
    uint64_t seed;              /* sync schedule + seeded partitions */
    uint32_t sync_base_ticks;   /* 20  (= 2 s,  `main.go:47`) */
    uint32_t sync_jitter_ticks; /* 10  (= rand.Intn(1000) ms, `main.go:46`) */
    int32_t enable_sync;        /* 1 = run SyncBroadcast timers */
    int32_t device;             /* HIP device ordinal; -1 = current device */
    uint32_t rank;              /* sharded mode: this engine's rank (0 if single) */
    uint32_t world;             /* sharded mode: number of engines (1 = single) */
    uint32_t lane_groups;       /* sharded mode: the ranks split the message lanes into this many
                                   groups of whole 64-lane words (0 or 1: every rank has every lane).
                                   world = lane_groups * parts; rank = group * parts + part. Ranks of
                                   one group split the nodes into `parts` vertex ranges (below); ranks
                                   of different groups never exchange anything (a value's propagation
                                   depends on no other value), so lane_groups == world needs no
                                   exchange at all and such an engine runs with gg_step. */
    uint32_t batch_ticks;       /* 0: the reference's semantics (parity mode). B >= 1: batched gossip,
                                   new semantics: a node keeps the
                                   values it learns as pending and, at the end of every round r with
                                   (r+1) % B == 0, sends ONE `broadcast` message per out-neighbour
                                   carrying its pending values (none to a neighbour that delivered all
                                   of them first); fwd_sent/fwd_delivered/acks count messages, not
                                   values. Sync timers: the read_ok callback adds what it lacked to
                                   the pending values and sends each peer one push with everything the
                                   peer's reply lacked; partition windows drop batches as in parity
                                   mode. One engine, or vertex parts (world > 1, lane_groups == 1:
                                   each engine runs its ghosts' timers, the exchange ships batches as
                                   F rows and the sets callbacks and pushes read as kind S); lane
                                   groups are refused (GG_EINVAL). The CPU oracle O2 is one engine. */
} gg_config;

typedef struct {
    int64_t round;           /* round these counters belong to */
    uint64_t new_bits;       /* (node,msg) deliveries in this round */
    uint64_t fwd_sent;       /* node->node `broadcast` forwards sent (:55, :99) */
    uint64_t fwd_delivered;  /* ... of which not dropped */
    uint64_t pushes;         /* sync pushes sent (:106) */
    uint64_t push_delivered; /* ... of which not dropped */
    uint64_t acks;           /* broadcast_ok replies to nodes sent (:69, :78) */
    uint64_t reads;          /* sync `read` RPCs sent (:120) */
    uint64_t read_oks;       /* `read_ok` replies to nodes sent (:131) */
    uint64_t dropped;        /* messages of every kind sent this round and dropped */
    uint64_t syncs_fired;    /* sync timers that fired this round */
    uint64_t seen_hash;      /* fingerprint of every round's new bits so far */
    double kernel_ms;        /* device time of the round (0 for the CPU oracle) */
    uint64_t work_rows;      /* diagnostics, engine-specific (not part of parity): */
    uint64_t work_gathers;   /*   nodes that moved rows, sender rows gathered */
    double prep_ms;          /*   device time of the round's kernels by kind: timers/marking, */
    double expand_ms;        /*   sparse/sync expand, dense streaming expand (first block */
    double stream_ms;        /*   start to last block end; 0 for the CPU oracle) */
    uint64_t prep_bytes;     /*   algorithmic bytes each kind had to move this round */
    uint64_t expand_bytes;   /*   (DESIGN.md §4), counted by the kernels */
    uint64_t stream_bytes;
    uint64_t sent_bytes;     /*   sharded: payload bytes this engine sent to other ranks */
    uint64_t path;           /*   GG_PATH_* bits: the kernel path the round took (0 for the CPU oracle) */
} gg_round_stats;

/* gg_round_stats.path (diagnostics) */
#define GG_PATH_STREAM 1u       /* lean round, F-row streaming kernels (expand_stream*, hub_*) */
#define GG_PATH_DB 2u           /* lean round, double-buffered sets (expand_stream_db) */
#define GG_PATH_SYNC_STREAM 4u  /* streamed sync round (sync_records, expand_stream_sync, hub_sync_*) */
#define GG_PATH_TILES 8u        /* tile path (expand_round) */
#define GG_PATH_MASKED 16u      /* a partition window touches rounds r-3..r+1 */
#define GG_PATH_BATCHED 32u     /* batched gossip (expand_batched) */
#define GG_PATH_NO_PREP 64u     /* no round_prep launch: the previous round's expand marked this round's
                                   candidates (double-buffered rounds of a single engine before the timers) */
#define GG_PATH_SOLO 128u       /* marking round with one expand kernel: the one the last run of this round
                                   needed (busy or not), instead of both with one exiting at once */
#define GG_PATH_LSAT 256u       /* the engine holds the lean saturation digest */
#define GG_PATH_LSAT_COMP 512u  /* ... with per-component targets (else every injected lane is the target) */

/* Inter-node messages of a round = fwd_sent + pushes + acks + reads + read_oks. */

int gg_create(const gg_config* cfg, gg_engine** out);
void gg_destroy(gg_engine* e);
const char* gg_last_error(const gg_engine* e);
int gg_abi_version(void);

/* Adjacency: row v lists topology[v] = the nodes v sends to, ascending and
 * unique (HandleTopology keeps topology[own id], missing row = empty list).
 * Directed lists are allowed; symmetric ones take a faster path. */
int gg_topology(gg_engine* e, const int64_t* row_ptr, const int32_t* col, uint64_t nnz);

/* Vertex-sharded engines (world / lane_groups = P > 1): HandleTopology from this
 * rank's own node range only (broadcast.go:40-45 keeps each node's own row; here
 * each rank keeps its range and no rank ever holds another's rows). Every rank of
 * a lane group passes the same part boundaries part_lo[0..P] (0 = part_lo[0] <=
 * ... <= part_lo[P] = n_nodes; part p owns nodes [part_lo[p], part_lo[p+1])) and
 * only its own rows: row_ptr[0..n] from 0 (n = its node count), col = global node
 * ids, ascending and unique per row. The topology must be symmetric (u lists v
 * iff v lists u), as Maelstrom's are: links inside the part are checked, links to
 * other parts are the caller's promise. Ghosts and send lists are built on the
 * device. */
int gg_topology_part(gg_engine* e, const uint64_t* part_lo, const int64_t* row_ptr, const int32_t* col,
                     uint64_t nnz);
/* The same for rows that may be directed (u lists v without v listing u): a
 * receiver's in-list is made of other parts' rows, so the ranks of the lane group
 * exchange the reverse of their cut edges once, over the engine's RCCL
 * communicator or the caller's transport — call gg_dist_comm_init or
 * gg_dist_transport_init first (collective over the lane group). No rank holds
 * another's rows; owned nodes keep id order. Per-edge windows (gg_set_partition)
 * on an engine built by either function take bits over the caller's own rows (a
 * symmetric topology and mask; links to other parts are the caller's promise). */
int gg_topology_part_directed(gg_engine* e, const uint64_t* part_lo, const int64_t* row_ptr, const int32_t* col,
                              uint64_t nnz);

/* Partition windows [round_from, round_to): a message sent in such a round
 * between nodes of different groups is dropped. Windows must not overlap.
 * Seeded: group(v) = bisection bit from (seed, epoch_seed, v). */
int gg_partition_seeded(gg_engine* e, int64_t round_from, int64_t round_to, uint64_t epoch_seed);
int gg_partition_groups(gg_engine* e, int64_t round_from, int64_t round_to, const uint8_t* group);
/* Per-edge window: edge_mask_bits holds one bit per
 * adjacency entry in the caller's CSR order (entry k of row u = the link u -> col[k];
 * 1 = cut): a message sent on a cut link in a round of [round_from, round_to) is
 * dropped, both ways, so the topology and the mask must be symmetric (GG_EINVAL
 * otherwise). Call after gg_topology (a new topology drops per-edge windows). A
 * per-edge window overrides a group window for the rounds both cover; per-edge
 * windows must not overlap each other. */
int gg_set_partition(gg_engine* e, int64_t round_from, int64_t round_to, const uint64_t* edge_mask_bits);

/* Client broadcast of `message` to `node`, delivered in `round` (>= current
 * round). The first broadcast of a value assigns it the next free lane. */
int gg_broadcast(gg_engine* e, uint32_t node, int64_t message, int64_t round);
/* n client broadcasts at once (same rules, applied in array order). */
int gg_broadcast_many(gg_engine* e, const uint32_t* nodes, const int64_t* messages,
                      const int64_t* rounds, uint64_t n);
int gg_lane_of(const gg_engine* e, int64_t message); /* lane or GG_EINVAL */

/* Run n_rounds lockstep rounds; out[i] (may be NULL) receives round i's stats. */
int gg_step(gg_engine* e, uint32_t n_rounds, gg_round_stats* out);
int64_t gg_current_round(const gg_engine* e);
/* Device time of the last gg_step measured with HIP events on the engine's
 * stream around the whole launch sequence (0 for the CPU oracle). */
int gg_step_device_ms(const gg_engine* e, double* ms);
/* A serving loop of whole episodes without a host round trip between them:
 * called right after gg_reset and the client broadcasts of one episode (current
 * round 0), runs `episodes` episodes of that schedule, each = n_rounds rounds;
 * episode k > 0 first does what gg_reset + the same broadcasts would. The
 * result equals `episodes` x (gg_reset; the same broadcasts; gg_step(n_rounds))
 * — out[k * n_rounds + i] (may be NULL) receives round i of episode k, and the
 * engine is left at the end of the last episode — but the episodes are queued
 * back to back on the engine's stream and the host waits only after the first
 * episode (its trailing quiet rounds tell the later resets which buffers an
 * episode leaves dirty) and at the end.
 * Single engine (not vertex-sharded), 1 <= n_rounds <= 256. gg_step_device_ms
 * then gives the device time per episode of episodes 2..K-1 (episode 1 can hold
 * a graph capture: the hints learned from episode 0 change the batch; with two
 * episodes it is episode 1, with one episode 0). (Host side of a Maelstrom run that
 * replays one broadcast workload many times; the reference has no counterpart.) */
int gg_run_episodes(gg_engine* e, uint32_t n_rounds, uint32_t episodes, gg_round_stats* out);

/* HandleRead: the values node holds, ascending. n_out = count (even if > cap). */
int gg_read(gg_engine* e, uint32_t node, int64_t* out, uint64_t cap, uint64_t* n_out);
/* Raw sets of nodes [lo,hi): (hi-lo) * W/64 words, lane l = bit l%64 of word l/64. */
int gg_read_bits(gg_engine* e, uint32_t node_lo, uint32_t node_hi, uint64_t* out);
/* First round each lane was seen, -1 if never: (hi-lo) * W int32 (GG_TRACK_DELIVERY). */
int gg_delivery_rounds(gg_engine* e, uint32_t node_lo, uint32_t node_hi, int32_t* out, uint64_t cap);

/* Back to round 0 with empty sets, no queued broadcasts, no lanes assigned;
 * topology and partition windows are kept. */
int gg_reset(gg_engine* e);

/* Device memory the engine holds (bytes of its live allocations; 0 for the CPU
 * oracle). sync_part: of which the streamed-sync buffers, which exist only once
 * a round at or after the first possible sync timer (sync_base_ticks) has been
 * enqueued — an episode that ends before the timers never allocates them. */
int gg_device_bytes(const gg_engine* e, uint64_t* total, uint64_t* sync_part);

/* ---- sharded mode (cfg.world > 1): one engine per GPU -------------------------
 * Every rank gives gg_topology the whole graph. The engine orders the nodes for
 * locality (its choice, identical on every rank: the native order or a DFS
 * preorder, whichever cuts fewer edges), splits that order into edge-balanced
 * contiguous ranges, and keeps its range's nodes ("owned") plus read-only copies
 * of the remote nodes adjacent to them ("ghosts"). Results do not depend on the
 * order: claims still go by ascending original sender id. A round is
 *   gg_dist_round_begin -> caller moves the ghost payloads between the ranks of
 *                          its lane group (see gg_exchange)
 *   gg_dist_round_end   -> the engine unpacks the ghosts; per-rank counters are
 *                          summed over ranks by the caller.
 * Only what a peer reads next round crosses: the F rows of owned
 * nodes that learned something this round, and whole sets only where the peer's
 * sync callback or a push reads them next round; sync timers are not exchanged
 * (each engine runs its ghosts' timers). A quiet round moves segment headers only.
 * When `stream` is non-NULL the round's kernels are only enqueued on that HIP
 * stream; the caller enqueues its collective on the same stream and passes
 * out = NULL to gg_dist_round_end, then collects the counters of all pending
 * rounds with gg_dist_flush (no host synchronisation per round). */
typedef struct {
    void* send;                 /* packed payloads: one segment per peer, at send_off[q] */
    void* recv;                 /* the segment from rank p must land at recv_off[p] */
    const uint64_t* send_bytes; /* [world] bytes to send to each rank this round */
    uint64_t* recv_bytes;       /* [world] bytes to receive from each rank (see exact) */
    const uint64_t* send_off;   /* [world] byte offset of the segment for rank q in send */
    const uint64_t* recv_off;   /* [world] byte offset of the segment from rank p in recv */
    uint64_t send_total, recv_total;  /* buffer capacities */
    int32_t on_device;          /* 1: send/recv are device memory of the engine's GPU */
    int32_t exact;              /* 0: static sizes (the segment capacities): send_bytes and recv_bytes
                                   are fixed and the segments are contiguous in rank order, so one
                                   all-to-all-v with them moves the round. 1: send_bytes are this
                                   round's exact sizes (the engine waited for its pack kernel): each
                                   peer must learn the size it receives (e.g. an all-to-all of the
                                   sizes; the caller writes them into recv_bytes) and the bytes must
                                   land at recv_off (e.g. point-to-point receives into views). */
    void* stream;               /* hipStream_t the round was enqueued on (NULL: done on return) */
} gg_exchange;

int gg_dist_round_begin(gg_engine* e, gg_exchange* xch);
/* out != NULL: wait for the round and return its counters; NULL: leave them pending. */
int gg_dist_round_end(gg_engine* e, gg_round_stats* out);
/* Wait for every pending round and return their counters in round order (n_out =
 * count); out = NULL only reports the count (after waiting) and keeps them pending. */
int gg_dist_flush(gg_engine* e, gg_round_stats* out, uint64_t cap, uint64_t* n_out);
/* Owned rows, ghost rows, and owned rows shipped per round (summed over peers). */
int gg_dist_info(const gg_engine* e, uint64_t* n_own, uint64_t* n_ghost, uint64_t* n_send);
/* Original ids of the owned nodes (n_out = count, even if > cap). */
int gg_dist_owned(const gg_engine* e, uint32_t* nodes, uint64_t cap, uint64_t* n_out);

/* Engine-owned exchange over RCCL (GPU engines): the rounds run without a caller
 * collective. The communicator spans the P vertex parts of the engine's lane group
 * (lane groups never exchange anything, so a process may hold engines of several
 * lane groups on one GPU, each with its own communicator): every rank of the lane
 * group passes the same 128-byte id (its part 0 makes it with gg_dist_comm_id and
 * the caller hands it round) and gg_dist_comm_init is collective over the group.
 * gg_dist_step(n) then enqueues n rounds, each gg_dist_round_begin + grouped
 * ncclSend/ncclRecv of the non-empty segments on the engine stream +
 * gg_dist_round_end(NULL); counters stay pending for gg_dist_flush. Replaces the
 * per-round all_to_all_single the caller would issue (the network delivery of every
 * cross-shard message, broadcast.go:55,99,106,120). Directions in exact-size mode
 * (GG_XCHG_MODE, or capacity > 4 MiB) first exchange their 8-byte sizes, and the
 * host waits for them once per round (payload counts are host arguments).
 * gg_dist_comm_available: 0 if the RCCL entry points resolve in this process
 * (why = reason otherwise); the CPU oracle library has no RCCL and returns GG_EIO. */
int gg_dist_comm_available(char* why, uint64_t cap);
/* ABI 6: the id names the lane group it is for — part 0 of EACH lane group makes
 * one with its own engine and hands it to the other parts of that group only;
 * gg_dist_comm_init refuses (GG_EINVAL) an id made for another lane group or part
 * count, instead of joining a wrong communicator (ABI 5 callers passed one id to
 * every rank: with lane_groups > 1 that could hang inside RCCL). */
int gg_dist_comm_id(const gg_engine* e, uint8_t* id_out /* 128 bytes */);
int gg_dist_comm_init(gg_engine* e, const uint8_t* id /* 128 bytes */);
/* The same exchange over the caller's transport instead of RCCL (e.g. a test
 * harness over another backend). gg_dist_step calls group_start, then send/recv of
 * device buffers to/from part indices of the lane group, then group_end, exactly
 * where it would issue the RCCL group. Stream semantics as in RCCL: the operations
 * act in `stream` order (a transport that stages through the host synchronises the
 * stream before reading and has written the receive buffers when group_end
 * returns). Callbacks return 0 on success. */
typedef struct {
    void* user;
    int (*group_start)(void* user);
    int (*send)(void* user, const void* buf, uint64_t bytes, uint32_t part, void* stream);
    int (*recv)(void* user, void* buf, uint64_t bytes, uint32_t part, void* stream);
    int (*group_end)(void* user);
} gg_transport;
int gg_dist_transport_init(gg_engine* e, const gg_transport* t);
/* n sharded rounds with the engine's exchange (RCCL, the transport or IPC; none
 * needed when the engine has no other vertex part). */
int gg_dist_step(gg_engine* e, uint32_t n_rounds);
/* gg_run_episodes for the device-driven sharded round (after gg_dist_ipc_import,
 * or lane groups only): right after gg_reset and the broadcasts, `episodes`
 * episodes of n_rounds gg_dist_step rounds, episode k > 0 first doing what
 * gg_reset + the same broadcasts would; this engine's own per-round stats (not
 * summed over ranks) in out[k * n_rounds + i], one host wait at the end. Every
 * rank of the job calls it with the same sizes. */
int gg_dist_run_episodes(gg_engine* e, uint32_t n_rounds, uint32_t episodes, gg_round_stats* out);

/* Device-driven exchange (no host wait, no collective call per round): every part
 * of a lane group exports one window of uncached device memory (flags and two
 * receive buffers) as a blob of GG_IPC_BLOB_BYTES (gg_dist_ipc_export), the caller
 * hands every part all P blobs of its lane group in part order, and
 * gg_dist_ipc_import maps the peers' windows (hipIpcOpenMemHandle; peers are other
 * processes, on this GPU or another of the node). From then on gg_dist_step packs
 * each peer's segment straight into the peer's receive buffer over xGMI and the
 * kernels hand rounds over with flags in the windows (bounded waits: a peer that
 * never arrives gives GG_EIO at the next flush instead of a hang; the first wait
 * that runs out marks the exchange dead, so every later wait, pack and unpack of
 * this engine returns at once and the job fails after one bound, not one per
 * queued round). A dead exchange stays dead: every later gg_dist_step, flush or
 * gg_dist_run_episodes returns GG_EIO — gg_reset does not revive it; install a
 * new topology and export and import the windows again (collectively). The round is a
 * fixed launch sequence on the engine stream. Every part must run the same number
 * of sharded rounds (they count them); a new topology drops the windows (export
 * and import again). gg_dist_round_begin reports zero bytes to move. */
#define GG_IPC_BLOB_BYTES 1024
int gg_dist_ipc_export(gg_engine* e, uint8_t* blob /* GG_IPC_BLOB_BYTES */);
/* A mapping that does not return within GG_IPC_OPEN_TIMEOUT_S seconds (env, default
 * 30) fails the import with GG_EIO instead of hanging the rank. Windows above 1 GiB are
 * allocated in whole GiB (the size that maps on this ROCm). */
int gg_dist_ipc_import(gg_engine* e, const uint8_t* blobs /* P x GG_IPC_BLOB_BYTES, part order */);
/* Collective teardown, first half: wait for the engine's stream and leave the
 * exchange (the engine no longer touches its peers' windows; it can export and
 * import again). Every part calls it, then the caller barriers, and only then does
 * any part destroy its engine: the engine's window goes back to the process's
 * window pool and is handed, flags zeroed, to a later engine, so no peer may still
 * be writing into it. Windows are never freed and peer mappings never closed while
 * the process lives (a freed-and-reallocated window could take the address range
 * of a mapping just closed, and the runtime then failed its export or blocked the
 * peer's open: DESIGN.md §5.4); a peer window mapped before is mapped again from
 * the process's cache. (The reference's nodes share no memory; this is the
 * device-driven exchange's lifecycle for broadcast.go:50-57's fan-out.) */
int gg_dist_ipc_close(gg_engine* e);

/* gg_read_bits / gg_delivery_rounds for a list of owned nodes (any engine). */
int gg_read_bits_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, uint64_t* out);
int gg_delivery_rounds_nodes(gg_engine* e, const uint32_t* nodes, uint64_t n, int32_t* out);

#ifdef __cplusplus
}
#endif

#endif /* GOSSIP_H_ */
