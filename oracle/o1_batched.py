"""O1B — message-level restatement of *batched* gossip.

TEST INFRASTRUCTURE ONLY (like ``o1_literal``): only ``tests/`` import it.

Batched gossip is the engine's opt-in ``gg_config.batch_ticks = B`` mode, the
msgs/op optimisation of the challenge (``/root/reference/README.md:17``), not
the reference's per-value protocol; parity mode (B = 0) is the reference's and
is restated by ``O1Network``. This class keeps O1's network, handlers for
reads and its lockstep order, and changes what a node sends:

* ``broadcast`` messages carry a list of values (``messages``). A receiver
  records each value it did not hold together with its first deliverer
  (``HandleBroadcast`` ``broadcast.go:59-79`` per value, without the
  immediate ``rebroadcastAllExcept`` of ``:76``) and acks the message (``:78``).
* At the end of every round r with (r + 1) % B == 0 a node sends its pending
  values to every neighbour in one message, minus the values that neighbour
  delivered to it first (``rebroadcastAllExcept``'s exclusion ``:52``, per
  value); a message with nothing left is not sent.
* The sync timer (``main.go:42-51``) and the ``read`` RPCs are the reference's
  (``broadcast.go:119-121``, ``:124-132``). The read_ok callback (``:82-117``)
  adds the values it lacked (deliverer: the peer) to the set and the pending
  values (forwarded with the next batch, not at once as ``:99`` does); after a
  round's callbacks the node sends each peer whose read_ok it handled one
  ``broadcast`` carrying every value it holds that the peer's reply lacked
  (``:104-108`` as one message, from the set after all of the round's
  callbacks), if that is not empty.
* Partition windows drop messages exactly as in parity mode (D3).
"""
from __future__ import annotations

from .o1_literal import Counters, Msg, O1Network, is_node, sync_interval


class O1Batched(O1Network):
    def __init__(self, n_nodes: int, n_lanes: int, seed: int = 0, sync_base: int = 20,
                 sync_jitter: int = 10, enable_sync: bool = True, batch_ticks: int = 1):
        super().__init__(n_nodes, n_lanes, seed, sync_base, sync_jitter, enable_sync)
        self.B = batch_ticks
        for nd in self.nodes:
            nd.pending = {}     # value -> first deliverer (node id; None: a client)
            nd.sync_peers = []  # (peer, values of its read_ok) handled this round

    def handle_broadcast(self, node, msg: Msg):
        vals = msg.body["messages"] if "messages" in msg.body else [msg.body["message"]]
        for m in vals:
            if m not in node.received:
                self._add(node, m)
                node.pending[m] = msg.src if is_node(msg.src) else None
        return self._reply(node, msg, {"type": "broadcast_ok"})

    def sync_broadcast(self, node):
        def sync_msgs(full_msg: Msg):
            resp = full_msg.body.get("messages") or []
            for m in resp:
                if m not in node.received:
                    self._add(node, m)
                    node.pending[m] = full_msg.src
            node.sync_peers.append((full_msg.src, set(resp)))

        for n in node.neighbors:
            self._rpc(node, n, {"type": "read"}, sync_msgs)

    def _one_round(self) -> dict:
        """O1Network._one_round plus the pushes after the callbacks and the batch send last."""
        r = self.round
        self._ctr = Counters(round=r)
        self._next_flight = []
        inbox: dict[int, list] = {}
        for msg in self.in_flight:
            inbox.setdefault(msg.dest, []).append(msg)
        clients = self.client_q.pop(r, [])
        tick = (r + 1) % self.B == 0
        for v, node in enumerate(self.nodes):
            msgs = inbox.get(v, [])
            for k, (dst, val) in enumerate(clients):  # (1) client broadcasts
                if dst == v:
                    self.handle_broadcast(node, Msg(-1 - k, v, {"type": "broadcast", "message": val}, "client"))
            for m in sorted((m for m in msgs if m.body["type"] == "broadcast"), key=lambda m: (m.src, m.seq)):
                self.handle_broadcast(node, m)  # (2) node broadcasts (batches, pushes)
            for m in sorted((m for m in msgs if m.body["type"] == "read_ok"), key=lambda m: (m.src, m.seq)):
                cb = node.callbacks.pop(m.body["in_reply_to"], None)  # (3) callbacks, ascending peer
                if cb is not None:
                    cb(m)
            for peer, R in node.sync_peers:  # one push per peer, from the set after every callback
                pay = sorted(x for x in node.received if x not in R)
                if pay:
                    self._send(node.nid, peer, {"type": "broadcast", "messages": pay}, "push")
            node.sync_peers = []
            for m in sorted((m for m in msgs if m.body["type"] == "read"), key=lambda m: (m.src, m.seq)):
                self.handle_read(node, m)  # (4) reads
            if self.enable_sync and r == node.sync_next:  # (5) sync timer
                self._ctr.syncs_fired += 1
                self.sync_broadcast(node)
                node.sync_k += 1
                node.sync_next = r + sync_interval(self.seed, v, node.sync_k, self.sync_base, self.sync_jitter)
            if tick and node.pending:  # (6) the batch
                for n in node.neighbors:
                    pay = sorted(x for x, d in node.pending.items() if d != n)
                    if pay:
                        self._send(node.nid, n, {"type": "broadcast", "messages": pay}, "fwd")
                node.pending = {}
        self.in_flight = self._next_flight
        self._ctr.seen_hash = self.seen_hash()
        self.round += 1
        return self._ctr.as_dict()
