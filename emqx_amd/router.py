"""Host mirror of `emqx_router` routing-schema v2 and the `emqx_router_syncer` stash over
the MI355X engine.

Reference: apps/emqx/src/emqx_router.erl:31-76 (API), :205-212/:511-516 (match_routes_v2),
:483-509 (insert/delete v2), :255-257 (do_batch), :518-578 (lookup/has/cleanup),
:627-635 (topics/stats); apps/emqx/src/emqx_router_syncer.erl:119-138, :297-328,
:381-401 (stash with last-op-wins, priority batches).

A route is `(topic_or_filter, dest)`, dest = node name (str) | (group, node) for a
$share subscription (emqx_shared_sub.erl:450) | ("external", x).  Schema v2 keeps
exact topics in a bag table and wildcard filters in the topic index; here both
live in one engine (exact filters are literal trie paths), so one GPU walk answers
`ets:lookup(emqx_route, T) ++ matches(T)` for a whole batch of topics.
"""
from __future__ import annotations

from collections import OrderedDict

from . import _native as N
from .topic import Share, parse


class Router:
    def __init__(self, device: int = 0, node: str = "emqx@127.0.0.1", engine: N.Engine | None = None, **kw):
        self.eng = engine or N.Engine(device, **kw)
        self.node = node
        self._dest_id: dict = {}
        self._dests: dict = {}  # route id -> dest
        self._groups: dict = {}  # shared group -> [group index, members so far]
        self._routes: dict = {}  # filter bytes -> set(dest)   (lookup_routes / topics)
        self._dirty = False

    def _did(self, dest) -> int:
        """Route id of a dest.  A shared dest {Group, Node} gets TM_SHARED_ID(group, member)
        (include/emqx_tm.h), so the GPU can collapse {Filter, Group} for aggre/1; a node dest
        gets a plain id."""
        u = self._dest_id.get(dest)
        if u is None:
            if isinstance(dest, tuple):
                g = self._groups.setdefault(dest[0], [len(self._groups), 0])
                u = N.shared_id(g[0], g[1])
                g[1] += 1
            else:
                u = len(self._dest_id)
            self._dest_id[dest] = u
            self._dests[u] = dest
        return u

    @staticmethod
    def _t(topic) -> bytes:
        return topic.encode() if isinstance(topic, str) else bytes(topic)

    # ---- writes (do_add_route/2, do_delete_route/2, do_batch/1)
    def do_add_route(self, topic, dest=None):
        t = self._t(topic)
        dest = self.node if dest is None else dest
        s = self._routes.setdefault(t, set())
        if dest not in s:
            s.add(dest)
            self.eng.apply([(N.TM_OP_ADD, t, self._did(dest))])
            self._dirty = True
        return "ok"

    add_route = do_add_route

    def do_delete_route(self, topic, dest=None):
        t = self._t(topic)
        dest = self.node if dest is None else dest
        s = self._routes.get(t)
        if s and dest in s:
            s.discard(dest)
            if not s:
                del self._routes[t]
            self.eng.apply([(N.TM_OP_DEL, t, self._dest_id[dest])])
            self._dirty = True
        return "ok"

    delete_route = do_delete_route

    def do_batch(self, batch: dict) -> dict:
        """batch: {(topic, dest): ('add'|'delete', ...)} -> {} (no errors); one epoch."""
        for (topic, dest), op in batch.items():
            action = op[0] if isinstance(op, tuple) else op
            if action == "add":
                self.do_add_route(topic, dest)
            elif action == "delete":
                self.do_delete_route(topic, dest)
            else:
                raise ValueError(action)
        self.commit()
        return {}

    def subscribe(self, topic_filter, node=None):
        """The route a subscription adds (emqx_topic:parse/1, emqx_topic.erl:324-365):
        `$share/G/F` and `$queue/F` become route (F, {G, Node}) (emqx_shared_sub.erl:450,
        group <<"$queue">> for $queue), anything else (F, Node) (emqx_broker.erl:719)."""
        f, dest = self._sub_route(topic_filter, node)
        return self.do_add_route(f, dest)

    def unsubscribe(self, topic_filter, node=None):
        f, dest = self._sub_route(topic_filter, node)
        return self.do_delete_route(f, dest)

    def _sub_route(self, topic_filter, node):
        node = self.node if node is None else node
        tf, _ = parse(topic_filter)
        if isinstance(tf, Share):
            return tf.topic, (tf.group.decode(), node)
        return tf, node

    def commit(self):
        if self._dirty:
            self.eng.commit()
            self._dirty = False

    def cleanup_routes(self, node):
        """Drop every route whose dest is `node` or (_, node) (emqx_router.erl:535-578)."""
        for t, dests in list(self._routes.items()):
            for d in list(dests):
                dn = d[1] if isinstance(d, tuple) and d[0] != "external" else d
                if dn == node:
                    self.do_delete_route(t, d)
        self.commit()

    # ---- reads
    def match_routes_batch(self, topics) -> list:
        """[[(filter, dest), ...] per topic] — match_routes/1 for a batch."""
        self.commit()
        res = self.eng.match(topics)
        out = []
        for hs in res:
            if hs is None:
                raise ValueError("badarg")
            routes = []
            for h in hs:
                u, fb, _ = self.eng.key_info(h)
                routes.append((fb, self._dests[u]))
            out.append(routes)
        return out

    def match_aggre_batch(self, topics) -> list:
        """[aggre(match_routes(T)) per topic] with the {Filter, Group} collapse done on the GPU
        (TM_MATCH_AGGRE).  emqx_broker:do_route/1 feeds match_routes/1 through aggre/1
        (emqx_broker.erl:361-377) before dispatch; only the final usort ordering is done
        here."""
        self.commit()
        res = self.eng.match(topics, N.TM_MATCH_AGGRE)
        out = []
        for hs in res:
            if hs is None:
                raise ValueError("badarg")
            acc, dedup = [], False
            for h in hs:
                u, fb, _ = self.eng.key_info(h)
                d = self._dests[u]
                if isinstance(d, tuple):
                    dedup = True
                    acc.append((fb, d[0]))
                else:
                    acc.append((fb, d))
            out.append(sorted(acc, key=repr) if dedup else acc)
        return out

    def match_routes(self, topic) -> list:
        return self.match_routes_batch([topic])[0]

    def lookup_routes(self, topic) -> list:
        t = self._t(topic)
        return [(t, d) for d in sorted(self._routes.get(t, ()), key=repr)]

    def has_route(self, topic, dest) -> bool:
        return dest in self._routes.get(self._t(topic), ())

    def has_any_route_batch(self, topics) -> list:
        """emqx_persistent_session_ds_router:has_any_route/1 for a batch (exact lookup or
        emqx_topic_index:match/2 =/= false, emqx_persistent_session_ds_router.erl:115-125):
        only the per-topic counts are needed, so the GPU skips the key copy-out
        (TM_MATCH_COUNT)."""
        self.commit()
        buf, off = N.pack_topics([self._t(t) for t in topics])
        _, cnt, _, st = self.eng.match_packed(buf, off, N.TM_MATCH_COUNT)
        if (st == N.TM_BADARG).any():
            raise ValueError("badarg")
        return [bool(c) for c in cnt]

    def has_any_route(self, topic) -> bool:
        return self.has_any_route_batch([topic])[0]

    def topics(self) -> list:
        return list(self._routes.keys())

    def stats(self, what="n_routes") -> int:
        assert what == "n_routes"
        return self.eng.stats()["n_keys"]


def aggre(routes):
    """emqx_broker:aggre/1 (apps/emqx/src/emqx_broker.erl:361-377): route list ->
    [(filter, node | group)], usorted when any shared dest is present."""
    if not routes:
        return []
    if len(routes) == 1:
        t, d = routes[0]
        return [(t, d[0] if isinstance(d, tuple) else d)]
    acc, dedup = [], False
    for t, d in routes:
        if isinstance(d, tuple):
            dedup = True
            acc.insert(0, (t, d[0]))
        else:
            acc.insert(0, (t, d))
    return sorted(set(acc), key=repr) if dedup else acc


class RouterSyncer:
    """emqx_router_syncer stash: ops coalesce per (topic, dest), last op wins
    (merge_route_op/2, :391-401); batches of at most max_batch ops are taken in
    priority order hi (with reply) > lo (add) > bg (delete) (:154-159, :297-328)."""

    PRIO_HI, PRIO_LO, PRIO_BG = 1, 2, 3

    def __init__(self, router: Router, max_batch: int = 1000):
        self.router = router
        self.max_batch = max_batch
        self.stash: OrderedDict = OrderedDict()

    def push(self, action: str, topic, dest, reply: bool = False):
        prio = self.PRIO_HI if reply else (self.PRIO_LO if action == "add" else self.PRIO_BG)
        key = (bytes(topic) if not isinstance(topic, str) else topic.encode(), dest)
        self.stash[key] = (action, prio)  # latter cancels the former

    def run_batch(self) -> int:
        batch = {}
        for prio in (self.PRIO_HI, self.PRIO_LO, self.PRIO_BG):
            for k, (a, p) in list(self.stash.items()):
                if len(batch) >= self.max_batch:
                    break
                if p == prio:
                    batch[k] = (a,)
                    del self.stash[k]
        if batch:
            self.router.do_batch(batch)
        return len(batch)

    def flush(self):
        while self.stash:
            self.run_batch()
