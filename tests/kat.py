"""Shared runner for the reference's known-answer index cases (tests/golden/kat_*.json).

A case is replayed against any object with the emqx_topic_index-shaped surface
    insert(filter, id) / delete(filter, id) / matches(topic, opts) / match(topic)
returning keys (filter_bytes_or_words_tuple, (id,)) — the GPU mirror
emqx_amd.topic_index.TopicIndex, or OracleIndex below (the CPU restatement).
"""
from __future__ import annotations

import numpy as np

PLUS, HASH = "+", "#"


def dec_word(w):
    if isinstance(w, dict):
        return w["atom"]
    return w.encode()


def dec_filter(f):
    """JSON filter -> bytes (binary form) or list of words (word-list form)."""
    if isinstance(f, list):
        return [dec_word(w) for w in f]
    return f.encode()


def key_topic(key) -> bytes:
    f = key[0]
    if isinstance(f, tuple):
        return b"/".join(w.encode() if isinstance(w, str) else w for w in f)
    return f


class BadArgError(Exception):
    pass


class OracleIndex:
    """emqx_topic_index surface over the C++ restatement (oracle/trie_search.cpp).
    Rebuilt from the live key list at every query (test sizes only)."""

    def __init__(self):
        self.keys = []  # (filter bytes, id, words_form)

    def insert(self, filt, ident, record=b""):
        wf = isinstance(filt, list)
        fb = b"/".join(w.encode() if isinstance(w, str) else w for w in filt) if wf else filt
        if wf and not any(w in (PLUS, HASH) for w in filt):
            k = (fb, ident, 1)
        else:
            k = (fb, ident, 1 if any(w in (b"+", b"#") for w in fb.split(b"/")) else 0)
        if k not in self.keys:
            self.keys.append(k)
        return True

    def delete(self, filt, ident):
        wf = isinstance(filt, list)
        fb = b"/".join(w.encode() if isinstance(w, str) else w for w in filt) if wf else filt
        self.keys = [k for k in self.keys if not (k[0] == fb and k[1] == ident)]
        return True

    def _run(self, topic: bytes, mode: int):
        import oracle
        from emqx_amd.topic import term_key
        ids = sorted({k[1] for k in self.keys}, key=term_key)
        rank = {x: i for i, x in enumerate(ids)}
        if not self.keys:
            fb, off, u, fl = np.zeros(1, np.uint8), np.zeros(1, np.uint64), np.zeros(0, np.uint64), None
        else:
            bs = [k[0] for k in self.keys]
            off = np.zeros(len(bs) + 1, dtype=np.uint64)
            off[1:] = np.cumsum([len(b) for b in bs])
            fb = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
            u = np.array([rank[k[1]] for k in self.keys], dtype=np.uint64)
            fl = np.array([k[2] for k in self.keys], dtype=np.uint32)
        ix = oracle.OrderedIndex(fb, off, u, fl)
        tb = np.frombuffer(topic + b"\0", dtype=np.uint8)
        to = np.array([0, len(topic)], dtype=np.uint32)
        o, got_ids, st, src = ix.match(tb, to, mode=mode, with_src=True)
        if st[0] == 1:
            raise BadArgError(topic)
        out = []
        for s in src.tolist():
            fbk, ident, wf = self.keys[s]
            ws = tuple(HASH if w == b"#" else PLUS if w == b"+" else w for w in fbk.split(b"/"))
            out.append(((ws if wf else fbk), (ident,)))
        return out

    def matches(self, topic: bytes, opts=()):
        from emqx_amd.topic import term_key
        keys = self._run(topic, 0)
        if "unique" in opts:
            best = {}
            for k in keys:  # walk (term) order: last write per id wins
                best[k[1][0]] = k
            return [best[i] for i in sorted(best, key=term_key)]
        return keys

    def match(self, topic: bytes):
        keys = self._run(topic, 2)
        return keys[0] if keys else False


class OracleRouter:
    """emqx_router match_routes/1 over the brute-force emqx_topic:match/2 restatement:
    the route table as a set of (filter, dest)."""

    def __init__(self, node="node"):
        self.node = node
        self.routes = set()

    def add_route(self, t, d):
        self.routes.add((t.encode(), d))

    def delete_route(self, t, d):
        self.routes.discard((t.encode(), d))

    def _sub(self, tf, node):
        from oracle import emqx_topic as et
        p, _ = et.parse(tf.encode())
        return (p.topic, (p.group.decode(), node)) if isinstance(p, et.Share) else (p, node)

    def subscribe(self, tf, node):
        self.routes.add(self._sub(tf, node))

    def unsubscribe(self, tf, node):
        self.routes.discard(self._sub(tf, node))

    def match_routes(self, topic):
        from oracle import emqx_topic as et
        tb = topic.encode()
        return [(f, d) for f, d in self.routes if et.match(tb, f)]

    def topics(self):
        return list({f for f, _ in self.routes})


def run_router_case(case, r):
    """Replay one kat_router.json case against a Router-shaped object (GPU mirror
    emqx_amd.router.Router or OracleRouter).  Steps: add/del/sub/unsub/match/count/topics."""
    def dest(d):
        return tuple(d) if isinstance(d, list) else d

    for step in case["steps"]:
        kind = step[0]
        if kind == "add":
            r.add_route(step[1], dest(step[2]))
        elif kind == "del":
            r.delete_route(step[1], dest(step[2]))
        elif kind == "sub":
            r.subscribe(step[1], step[2])
        elif kind == "unsub":
            r.unsubscribe(step[1], step[2])
        elif kind == "match":
            got = sorted(((bytes(f).decode(), d) for f, d in r.match_routes(step[1])), key=repr)
            exp = sorted(((f, dest(d)) for f, d in step[2]), key=repr)
            assert got == exp, (case["name"], step, got)
        elif kind == "count":
            assert len(r.match_routes(step[1])) == step[2], (case["name"], step)
        elif kind == "topics":
            assert sorted(bytes(t).decode() for t in r.topics()) == sorted(step[1]), (case["name"], step)
        else:
            raise ValueError(kind)


def run_index_case(case, make_index, check):
    """Replay one kat_index.json case; `check(cond, msg)` reports failures."""
    ix = make_index()
    for f, i in case.get("insert", []):
        ix.insert(dec_filter(f), i)
    for f, i in case.get("delete", []):
        ix.delete(dec_filter(f), i)
    for q in case["queries"]:
        kind, topic = q[0], q[1].encode()
        if kind == "badarg":
            try:
                ix.matches(topic, opts=[])
            except Exception as e:  # BadArg / BadArgError
                check("badarg" in type(e).__name__.lower() or "badarg" in str(e).lower(), f"{case['name']}: {e!r}")
                continue
            check(False, f"{case['name']}: {topic!r} should be badarg")
        elif kind == "matches_topics":
            got = sorted(key_topic(k).decode() for k in ix.matches(topic, opts=[]))
            check(got == sorted(q[2]), f"{case['name']} {topic!r}: {got} != {q[2]}")
        elif kind == "matches_ids":
            opts, exp = q[2], q[3]
            got = [k[1][0] for k in ix.matches(topic, opts=opts)]
            if "unique" not in opts:
                got, exp = sorted(got, key=repr), sorted(exp, key=repr)
            check(got == exp, f"{case['name']} {topic!r} {opts}: {got} != {exp}")
        elif kind == "count":
            got = len(ix.matches(topic, opts=[]))
            check(got == q[2], f"{case['name']} {topic!r}: count {got} != {q[2]}")
        elif kind in ("match_id", "match_topic"):
            k = ix.match(topic)
            if q[2] is None:
                check(k is False, f"{case['name']} {topic!r}: {k} should be false")
            else:
                got = k[1][0] if kind == "match_id" and k else (key_topic(k).decode() if k else None)
                check(got == q[2], f"{case['name']} {kind} {topic!r}: {got} != {q[2]}")
        else:
            raise ValueError(kind)
