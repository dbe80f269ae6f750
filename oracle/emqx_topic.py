"""oracle/emqx_topic.py — TEST INFRASTRUCTURE ONLY.

A pure-Python restatement of the reference's topic semantics, used by tests/ to
check the golden vectors transcribed from the reference's suites and to pin the
C++ oracle (oracle/trie_search.cpp).  Nothing under emqx_amd/ imports it.

Follows apps/emqx/src/emqx_topic.erl (line numbers cite that file):
  wildcard/1 :63-75, match/2 :78-102, intersection/2 :111-151, validate/1,2 :177-246,
  levels/1 :268-272, tokens/1 :276-278, words/1 + word/1 :281-291, join/1 :310-322,
  parse/1,2 :324-365, prepend/2 :250-259, feed_var/3 :300-308, systop/1 :294-298.

Erlang atoms are modelled as Python str ('+', '#', ''), binaries as bytes.
"""
from __future__ import annotations

MAX_TOPIC_LEN = 65535  # ?MAX_TOPIC_LEN, apps/emqx/include/emqx_mqtt.hrl:56


class TopicError(Exception):
    """error(Reason) raised by the reference."""

    def __init__(self, reason):
        super().__init__(reason)
        self.reason = reason


class Share:
    """#share{group, topic} (emqx_mqtt.hrl:62)."""

    def __init__(self, group: bytes, topic: bytes):
        self.group, self.topic = group, topic

    def __eq__(self, o):
        return isinstance(o, Share) and (self.group, self.topic) == (o.group, o.topic)

    def __repr__(self):
        return f"Share({self.group!r}, {self.topic!r})"


def tokens(topic: bytes) -> list:
    return topic.split(b"/")


def word(b: bytes):
    if b == b"":
        return ""
    if b == b"+":
        return "+"
    if b == b"#":
        return "#"
    return b


def words(topic) -> list:
    if isinstance(topic, Share):
        topic = topic.topic
    return [word(w) for w in tokens(topic)]


def levels(topic) -> int:
    if isinstance(topic, Share):
        topic = topic.topic
    return len(tokens(topic))


def wildcard(t) -> bool:
    if isinstance(t, Share):
        t = t.topic
    ws = words(t) if isinstance(t, (bytes, bytearray)) else t
    for w in ws:
        if w in ("#", "+"):
            return True
    return False


def trie_filter(topic: bytes):
    """emqx_trie_search:filter/1 + filter_words/1 (emqx_trie_search.erl:136-140,358-366):
    '+'/'#' become atoms, every other level (the empty one included) stays a binary;
    False when no level is a wildcard."""
    ws = ["+" if w == b"+" else "#" if w == b"#" else w for w in tokens(topic)]
    return ws if wildcard(ws) else False


def _match_words(n: list, f: list) -> bool:
    i = 0
    while True:
        if i == len(n) and i == len(f):          # match([], [])
            return True
        if i < len(n) and i < len(f) and n[i] == f[i]:   # match([H|T1], [H|T2])
            i += 1
            continue
        if i < len(n) and i < len(f) and f[i] == "+":    # match([_H|T1], ['+'|T2])
            i += 1
            continue
        if i < len(n) and i < len(f) and n[i] == b"" and f[i] == "":  # match([<<>>|T1], [''|T2])
            i += 1
            continue
        if f[i:] == ["#"]:                       # match(_, ['#'])
            return True
        return False


def match(name, filt) -> bool:
    """emqx_topic:match/2 (emqx_topic.erl:78-102)."""
    if isinstance(name, (bytes, bytearray)) and isinstance(filt, (bytes, bytearray)):
        if name[:1] == b"$" and filt[:1] in (b"+", b"#"):
            return False
        return _match_words(words(name), words(filt))
    if isinstance(name, Share) and isinstance(filt, (bytes, bytearray)):
        return _match_words(words(name.topic), words(filt))
    if isinstance(name, Share) and isinstance(filt, Share):
        return name.group == filt.group and _match_words(words(name.topic), words(filt.topic))
    if isinstance(name, Share):
        return False
    if isinstance(filt, Share):
        return match(name, filt.topic)
    return _match_words(list(name), list(filt))


def match_any(name, filters) -> bool:
    return any(match(name, f) for f in filters)


def _bin(w) -> bytes:
    if w == "":
        return b""
    if w in ("+", "#"):
        return w.encode()
    return w


def join(ws) -> bytes:
    """emqx_topic:join/1 (emqx_topic.erl:310-322)."""
    if not ws:
        return b""
    for i, w in enumerate(ws):
        if w in ("#", b"#") and i != len(ws) - 1:
            raise TopicError("topic_invalid_#")
    return b"/".join(_bin(w) for w in ws)


def prepend(parent, w) -> bytes:
    wb = _bin(w) if not isinstance(w, str) or w in ("", "+", "#") else w.encode()
    if parent is None or parent in (b"", ""):
        return wb
    p = parent.encode() if isinstance(parent, str) else (parent if isinstance(parent, bytes) else _bin(parent))
    return p + wb if p.endswith(b"/") else p + b"/" + wb


def feed_var(var: bytes, val: bytes, topic: bytes) -> bytes:
    return join([val if w == var else w for w in words(topic)])


def systop(name, node: str = "emqx@127.0.0.1") -> bytes:
    n = name.encode() if isinstance(name, str) else name
    return b"$SYS/brokers/" + node.encode() + b"/" + n


def _validate2(ws):
    for i, w in enumerate(ws):
        if w == "#" and i == len(ws) - 1:
            return True
        if w in ("#", b"#") and i != len(ws) - 1:
            raise TopicError("topic_invalid_#")
        if w in ("", "+"):
            continue
        try:
            w.decode("utf-8")
        except UnicodeDecodeError as e:  # <<_/utf8, ...>> fails -> function_clause
            raise TopicError("function_clause") from e
        for ch in w.decode("utf-8"):
            if ch in "#+\0":
                raise TopicError("topic_invalid_char")
    return True


def validate(topic, kind="filter") -> bool:
    """emqx_topic:validate/1,2 (emqx_topic.erl:177-246)."""
    if isinstance(topic, tuple):
        kind, topic = topic
    if topic == b"":
        raise TopicError("empty_topic")
    if len(topic) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    if kind == "filter" and topic.startswith(b"$share/"):
        rest = topic[len(b"$share/"):]
        if rest in (b"", b"/"):
            raise TopicError("share_empty_filter")
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise TopicError("share_empty_filter")  # unreachable in practice
        group, filt = parts
        if group == b"":
            raise TopicError("share_empty_group")
        if filt == b"":
            raise TopicError("share_empty_filter")
        if filt.startswith(b"$share/"):
            raise TopicError("share_recursively")
        if b"+" in group or b"#" in group:
            raise TopicError("share_name_invalid_char")
        return _validate2(words(filt))
    ws = words(topic)
    if kind == "filter":
        return _validate2(ws)
    if _validate2(ws) and not wildcard(ws):
        return True
    raise TopicError("topic_name_error")


def parse(tf, options=None):
    """emqx_topic:parse/1,2 (emqx_topic.erl:324-365)."""
    options = dict(options or {})
    if isinstance(tf, Share):
        if tf.topic.startswith(b"$queue/") or tf.topic.startswith(b"$share/"):
            raise TopicError(("invalid_topic_filter", tf.topic))
        if options.get("nl") == 1:
            raise TopicError(("invalid_subopts_nl", tf))
        return tf, options
    if tf.startswith(b"$queue/"):
        return parse(Share(b"$queue", tf[len(b"$queue/"):]), options)
    if tf.startswith(b"$share/"):
        rest = tf[len(b"$share/"):]
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise TopicError(("invalid_topic_filter", tf))
        group, topic = parts
        if b"+" in group or b"#" in group:
            raise TopicError(("invalid_topic_filter", tf))
        return parse(Share(group, topic), options)
    if tf.startswith(b"$exclusive/"):
        t = tf[len(b"$exclusive/"):]
        if t == b"":
            raise TopicError(("invalid_topic_filter", tf))
        options["is_exclusive"] = True
        return t, options
    return tf, options


def _is_wild(w) -> bool:
    return w in ("+", "#")


def intersection(t1: bytes, t2: bytes):
    """emqx_topic:intersection/2 (emqx_topic.erl:111-151)."""
    w1, w2 = words(t1), words(t2)
    if w1 and w2:
        if isinstance(w1[0], bytes) and w1[0].startswith(b"$") and _is_wild(w2[0]):
            return False
        if isinstance(w2[0], bytes) and w2[0].startswith(b"$") and _is_wild(w1[0]):
            return False
    r = _intersect(w1, w2)
    return False if r is False else join(r)


def _intersect(a, b):
    if b == ["#"]:
        return a
    if a == ["#"]:
        return b
    if len(a) == 1 and b == ["+"]:
        return [a[0]]
    if a == ["+"] and len(b) == 1:
        return [b[0]]
    if a and b:
        x, y = a[0], b[0]
        if _is_wild(x) and _is_wild(y):
            rest = _intersect(a[1:], b[1:])
            return False if rest is False else [x if x == y else "+"] + rest
        if x == y:
            rest = _intersect(a[1:], b[1:])
            return False if rest is False else [x] + rest
        if _is_wild(x):
            rest = _intersect(a[1:], b[1:])
            return False if rest is False else [y] + rest
        if _is_wild(y):
            rest = _intersect(a[1:], b[1:])
            return False if rest is False else [x] + rest
    if not a and not b:
        return []
    return False


def brute_matches(topic: bytes, keys) -> list:
    """All (filter, id) keys whose filter matches `topic` under match/2 — the
    brute-force side of t_prop_matches (emqx_topic_index_SUITE.erl:318-329)."""
    return [k for k in keys if match(topic, k[0])]
