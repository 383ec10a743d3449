"""O1 — message-level literal restatement of the reference broadcast node.

TEST INFRASTRUCTURE ONLY. This file is the semantic ground truth the checker
uses; nothing in the product imports it (only ``tests/``, ``__graft_entry__.smoke``
and ``bench.py``'s ``cpu_baseline`` leg may).

Parity status: **parity unpinned** — the reference has no tests, fixtures or
golden vectors, its Go toolchain and its pinned maelstrom
dependency (``github.com/jepsen-io/maelstrom/demo/go
v0.0.0-20250806145204-447d18a7c07e``, ``broadcast/go.mod:5``) are absent, and
the shipped ``broadcast/maelstrom-broadcast`` binary is a stale build that is
never run. O1 is anchored on the analytic known-answer tests of SURVEY.md §8c
(tests/test_o1_kat.py) and on a line-by-line restatement of the handlers.

Every node is a ``Node`` holding the reference's state: its ``neighbors`` list
(``Context.neighbors``, ``broadcast/main.go:13``) and its ``received`` set
(``BroadcastContext.receivedMsgs``, ``broadcast/broadcast.go:13-16``). Handlers
follow the Go code statement by statement; the maelstrom library's
Send / Reply / RPC (``broadcast.go:47,55,69,78,106,120,131``) become appends to
an explicit in-memory network. The concurrency of the real system (one
goroutine per inbound message, wall-clock timers) is replaced by the lockstep
contract of SURVEY.md Appendix A / DESIGN.md §2:

* D3: a message sent in round r is delivered in round r+1, unless a partition
  window covering round r separates sender and receiver (then it is dropped).
* D2: inside round r node v handles (1) client broadcasts in call order,
  (2) node broadcasts in ascending sender id (then send order), (3) read_ok
  callbacks in ascending peer id, (4) read requests, answered with the set
  after (1)-(3), (5) its sync timer (``main.go:42-51``).
* broadcast_ok from a node is dispatched to the no-op handler (``main.go:38-40``).

Seeded functions restate include/gossip_spec.h independently.
"""
from __future__ import annotations

from dataclasses import dataclass, field

M64 = (1 << 64) - 1
TAG_SYNC = 0x53594E4353594E43
TAG_PART = 0x5041525450415254
TAG_HASH = 0x4841534848415348


def mix64(x: int) -> int:
    """splitmix64 finaliser (include/gossip_spec.h gg_mix64)."""
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sync_interval(seed: int, v: int, k: int, base: int, jitter: int) -> int:
    """Ticks of ``time.Sleep(2s + rand.Intn(1000)ms)`` (``broadcast/main.go:46-48``)."""
    if jitter == 0:
        return base
    h = mix64(mix64(seed ^ TAG_SYNC) ^ mix64(((v << 20) ^ k) & M64))
    return base + (h % (100 * jitter)) // 100


def part_group(seed: int, epoch_seed: int, v: int) -> int:
    return mix64(mix64(seed ^ TAG_PART ^ epoch_seed) ^ v) & 1


def word_hash(idx: int, word: int) -> int:
    return mix64(mix64(idx ^ TAG_HASH) ^ word)


# --------------------------------------------------------------------------
# wire messages


@dataclass
class Msg:
    src: int  # node id, or -1 - k for client k
    dest: int
    body: dict
    kind: str  # accounting class: fwd | push | ack | read | read_ok | client
    seq: int = 0  # send order at the sender within the round


def is_node(i: int) -> bool:
    return i >= 0


@dataclass
class Counters:
    round: int = 0
    new_bits: int = 0
    fwd_sent: int = 0
    fwd_delivered: int = 0
    pushes: int = 0
    push_delivered: int = 0
    acks: int = 0
    reads: int = 0
    read_oks: int = 0
    dropped: int = 0
    syncs_fired: int = 0
    seen_hash: int = 0

    def as_dict(self):
        return dict(self.__dict__)


# --------------------------------------------------------------------------


@dataclass
class Node:
    """``Context`` (``broadcast/main.go:11-15``) for node ``nid``."""

    nid: int
    neighbors: list = field(default_factory=list)
    received: dict = field(default_factory=dict)  # receivedMsgs map[int]bool
    callbacks: dict = field(default_factory=dict)  # maelstrom RPC callbacks by msg_id
    next_msg_id: int = 1
    sync_k: int = 0
    sync_next: int = 0


class O1Network:
    """Lockstep in-memory network of reference broadcast nodes."""

    def __init__(self, n_nodes: int, n_lanes: int, seed: int = 0, sync_base: int = 20,
                 sync_jitter: int = 10, enable_sync: bool = True):
        self.V = n_nodes
        self.W = n_lanes
        self.seed = seed
        self.sync_base = sync_base
        self.sync_jitter = sync_jitter
        self.enable_sync = enable_sync
        self.nodes = [Node(v) for v in range(n_nodes)]
        for nd in self.nodes:
            nd.sync_k = 0
            nd.sync_next = sync_interval(seed, nd.nid, 0, sync_base, sync_jitter)
        self.round = 0
        self.in_flight: list[Msg] = []  # sent last round, not dropped
        self.client_q: dict[int, list] = {}  # round -> [(node, value)] in call order
        self.lanes: dict[int, int] = {}  # value -> lane (first broadcast call order)
        self.windows: list = []  # (from, to, kind, payload)
        self.first_seen: dict = {}  # (node, value) -> round
        self._ctr: Counters | None = None
        self._seq = 0
        self._hash_total = 0  # seen_hash so far
        self._prev_bits: list[list[int]] = [[0] * (n_lanes // 64) for _ in range(n_nodes)]

    # ---- setup -----------------------------------------------------------

    def topology(self, adj: list[list[int]]):
        """HandleTopology ``broadcast/broadcast.go:36-48`` for every node."""
        for v, nd in enumerate(self.nodes):
            row = adj[v] if v < len(adj) else None
            nd.neighbors = list(row) if row is not None else []  # :41-45

    def partition_seeded(self, r0: int, r1: int, epoch_seed: int):
        self.windows.append((r0, r1, "seeded", epoch_seed))

    def partition_groups(self, r0: int, r1: int, groups):
        self.windows.append((r0, r1, "groups", list(groups)))

    def set_partition(self, r0: int, r1: int, bits):
        """Per-edge window (gg_set_partition): bit k of `bits` (uint64 words) cuts
        adjacency entry k in topology order (row u, then its neighbours); a cut
        link drops messages both ways; it overrides a group window."""
        cut, k = set(), 0
        for nd in self.nodes:
            for n in nd.neighbors:
                if (int(bits[k >> 6]) >> (k & 63)) & 1:
                    cut.add((nd.nid, n))
                    cut.add((n, nd.nid))
                k += 1
        self.windows.append((r0, r1, "edges", frozenset(cut)))

    def broadcast(self, node: int, value: int, rnd: int):
        if value not in self.lanes:
            if len(self.lanes) >= self.W:
                raise ValueError("ENOSPC")
            self.lanes[value] = len(self.lanes)
        self.client_q.setdefault(rnd, []).append((node, value))

    # ---- network ---------------------------------------------------------

    def _group(self, win, v):
        _, _, kind, payload = win
        if kind == "seeded":
            return part_group(self.seed, payload, v)
        return payload[v]

    def masked(self, rnd: int, a: int, b: int) -> bool:
        for win in self.windows:  # a per-edge window overrides a group window
            if win[2] == "edges" and win[0] <= rnd < win[1]:
                return (a, b) in win[3]
        for win in self.windows:
            if win[2] != "edges" and win[0] <= rnd < win[1]:
                return self._group(win, a) != self._group(win, b)
        return False

    def _send(self, src: int, dest: int, body: dict, kind: str):
        c = self._ctr
        self._seq += 1
        msg = Msg(src, dest, body, kind, self._seq)
        if kind == "client":  # replies to clients: not inter-node traffic
            self.last_client_reply = body
            return
        if kind == "fwd":
            c.fwd_sent += 1
        elif kind == "push":
            c.pushes += 1
        elif kind == "ack":
            c.acks += 1
        elif kind == "read":
            c.reads += 1
        elif kind == "read_ok":
            c.read_oks += 1
        if self.masked(self.round, src, dest):
            c.dropped += 1
            return
        if kind == "fwd":
            c.fwd_delivered += 1
        elif kind == "push":
            c.push_delivered += 1
        self._next_flight.append(msg)

    def _reply(self, node: Node, msg: Msg, body: dict):
        """maelstrom Node.Reply: to a node -> inter-node message, to a client -> not counted."""
        body = dict(body)
        body["in_reply_to"] = msg.body.get("msg_id", 0)
        if not is_node(msg.src):
            kind = "client"
        elif body["type"] == "broadcast_ok":
            kind = "ack"
        else:
            kind = "read_ok"
        self._send(node.nid, msg.src, body, kind)

    def _rpc(self, node: Node, dest: int, body: dict, cb):
        body = dict(body)
        body["msg_id"] = node.next_msg_id
        node.callbacks[node.next_msg_id] = cb
        node.next_msg_id += 1
        self._send(node.nid, dest, body, "read")

    # ---- handlers (broadcast/broadcast.go) -------------------------------

    def _add(self, node: Node, m: int):
        if m not in node.received:
            self._ctr.new_bits += 1
            self.first_seen[(node.nid, m)] = self.round
        node.received[m] = True

    def rebroadcast_all_except(self, node: Node, excluded: int, m: int, kind="fwd"):
        """``broadcast.go:50-57``."""
        for n in node.neighbors:
            if n == excluded:  # :52
                continue
            self._send(node.nid, n, {"type": "broadcast", "message": m}, kind)  # :55

    def handle_broadcast(self, node: Node, msg: Msg):
        """``broadcast.go:59-79``."""
        m = msg.body["message"]
        node_from = msg.src  # :62
        if m in node.received:  # :65-67
            return self._reply(node, msg, {"type": "broadcast_ok"})  # :69
        self._add(node, m)  # :72-74
        self.rebroadcast_all_except(node, node_from, m)  # :76
        return self._reply(node, msg, {"type": "broadcast_ok"})  # :78

    def sync_broadcast(self, node: Node):
        """``broadcast.go:81-122``."""

        def sync_msgs(full_msg: Msg):  # :82
            resp = full_msg.body.get("messages") or []  # :83-84 (null -> empty)
            snapshot = {m: True for m, ok in node.received.items() if ok}  # :86-93
            missing = []  # :95
            for m in resp:  # :97
                if not snapshot.get(m, False):  # :98
                    self.rebroadcast_all_except(node, full_msg.src, m)  # :99
                missing.append(m)  # :101 (every m, unconditionally)
            in_resp = set(resp)  # :105 slices.Contains, as a set lookup (same answer)
            for m in sorted(snapshot):  # :104 (map order; all sends land in one round)
                if m not in in_resp:
                    self._send(node.nid, full_msg.src,
                               {"type": "broadcast", "message": m}, "push")  # :106
            for m in missing:  # :110-114
                self._add(node, m)
            return None

        for n in node.neighbors:  # :119
            self._rpc(node, n, {"type": "read"}, sync_msgs)  # :120

    def handle_read(self, node: Node, msg: Msg):
        """``broadcast.go:124-132``: every key; JSON null when empty."""
        messages = sorted(node.received) or None
        return self._reply(node, msg, {"type": "read_ok", "messages": messages})

    # ---- lockstep round ----------------------------------------------------

    def step(self, n_rounds: int = 1):
        out = []
        for _ in range(n_rounds):
            out.append(self._one_round())
        return out

    def _one_round(self) -> dict:
        r = self.round
        self._ctr = Counters(round=r)
        self._next_flight = []
        inbox: dict[int, list] = {}
        for msg in self.in_flight:
            inbox.setdefault(msg.dest, []).append(msg)
        clients = self.client_q.pop(r, [])
        for v, node in enumerate(self.nodes):
            msgs = inbox.get(v, [])
            # (1) client broadcasts, call order
            for k, (dst, val) in enumerate(clients):
                if dst == v:
                    self.handle_broadcast(node, Msg(-1 - k, v, {"type": "broadcast",
                                                               "message": val}, "client"))
            # (2) node broadcasts, ascending sender then send order
            bc = sorted((m for m in msgs if m.body["type"] == "broadcast"),
                        key=lambda m: (m.src, m.seq))
            for m in bc:
                self.handle_broadcast(node, m)
            # (3) read_ok callbacks, ascending peer
            rk = sorted((m for m in msgs if m.body["type"] == "read_ok"),
                        key=lambda m: (m.src, m.seq))
            for m in rk:
                cb = node.callbacks.pop(m.body["in_reply_to"], None)
                if cb is not None:
                    cb(m)
            # broadcast_ok: no-op handler (main.go:38-40)
            # (4) read requests
            rq = sorted((m for m in msgs if m.body["type"] == "read"),
                        key=lambda m: (m.src, m.seq))
            for m in rq:
                self.handle_read(node, m)
            # (5) sync timer (main.go:42-51)
            if self.enable_sync and r == node.sync_next:
                self._ctr.syncs_fired += 1
                self.sync_broadcast(node)
                node.sync_k += 1
                node.sync_next = r + sync_interval(self.seed, v, node.sync_k,
                                                   self.sync_base, self.sync_jitter)
        self.in_flight = self._next_flight
        self._ctr.seen_hash = self.seen_hash()
        self.round += 1
        return self._ctr.as_dict()

    # ---- observation -------------------------------------------------------

    def read(self, v: int) -> list[int]:
        return sorted(self.nodes[v].received)

    def client_read(self, v: int, msg_id: int = 1) -> dict:
        """A client `read` of node v through HandleRead (broadcast.go:124-132):
        the reply body as the handler builds it (messages None = JSON null)."""
        self.last_client_reply = None
        self.handle_read(self.nodes[v], Msg(-1, v, {"type": "read", "msg_id": msg_id}, "client"))
        return self.last_client_reply

    def bits(self, v: int) -> list[int]:
        nw = self.W // 64
        words = [0] * nw
        for m in self.nodes[v].received:
            lane = self.lanes[m]
            words[lane // 64] |= 1 << (lane % 64)
        return words

    def seen_hash(self) -> int:
        """Delivery fingerprint: the sum (mod 2^64), over every
        round so far and every set word that gained bits in it, of
        word_hash(idx, the word's new bits); called once at the end of a round."""
        nw = self.W // 64
        for v in range(self.V):
            prev = self._prev_bits[v]
            for j, w in enumerate(self.bits(v)):
                new = w & ~prev[j]
                if new:
                    self._hash_total = (self._hash_total + word_hash(v * nw + j, new)) & M64
                prev[j] = w
        return self._hash_total

    def delivery_rounds(self, v: int) -> list[int]:
        out = [-1] * self.W
        for m, lane in self.lanes.items():
            out[lane] = self.first_seen.get((v, m), -1)
        return out
