"""Product-side topic helpers the boundary needs (not the match itself).

Mirrors the parts of emqx_topic (apps/emqx/src/emqx_topic.erl) that callers of the
index use before/after a match: tokenising, the word-list form of a filter, join,
wildcard detection and the $share/$queue/$exclusive parse that decides which
(filter, dest) route key a subscription becomes (emqx_shared_sub.erl:444-456).
Matching itself is done only by the HIP engine.
"""
from __future__ import annotations

from dataclasses import dataclass

PLUS = "+"   # the atom '+' of a filter word list
HASH = "#"   # the atom '#'
SHARE = b"$share"
QUEUE = b"$queue"


def _b(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def tokens(topic) -> list[bytes]:
    """emqx_topic:tokens/1 (emqx_topic.erl:276-278): binary:split(T, "/", [global])."""
    return _b(topic).split(b"/")


def filter_words(topic) -> list:
    """emqx_trie_search:filter_words/1 (emqx_trie_search.erl:358-366): '+'/'#' become
    atoms, everything else (including the empty level) stays a binary."""
    if isinstance(topic, list):
        return topic
    out = []
    for w in tokens(topic):
        out.append(PLUS if w == b"+" else HASH if w == b"#" else w)
    return out


def wildcard(words_or_topic) -> bool:
    """emqx_topic:wildcard/1 (emqx_topic.erl:63-75)."""
    ws = filter_words(words_or_topic) if not isinstance(words_or_topic, list) else words_or_topic
    return any(w in (PLUS, HASH) for w in ws)


def filter(topic):  # noqa: A001 - the reference's name
    """emqx_trie_search:filter/1 (emqx_trie_search.erl:136-140): the word list of a
    wildcard filter, False for a filter without '+'/'#' (make_key/2 keeps those binary)."""
    ws = filter_words(topic)
    return ws if wildcard(ws) else False


def join(words) -> bytes:
    """emqx_topic:join/1 (emqx_topic.erl:310-322) for word lists."""
    parts = []
    for i, w in enumerate(words):
        if w == HASH and i != len(words) - 1:
            raise ValueError("topic_invalid_#")
        parts.append(b"+" if w == PLUS else b"#" if w == HASH else b"" if w == "" else _b(w))
    return b"/".join(parts)


@dataclass(frozen=True)
class Share:
    """#share{group, topic} (emqx_mqtt.hrl:62)."""
    group: bytes
    topic: bytes


def parse(topic_filter):
    """emqx_topic:parse/1 (emqx_topic.erl:324-365) without the subopts checks:
    returns (filter_or_Share, opts)."""
    tf = _b(topic_filter)
    if tf.startswith(QUEUE + b"/"):
        real = tf[len(QUEUE) + 1:]
        if real.startswith(QUEUE + b"/") or real.startswith(SHARE + b"/"):
            raise ValueError(("invalid_topic_filter", real))
        return Share(QUEUE, real), {}
    if tf.startswith(SHARE + b"/"):
        rest = tf[len(SHARE) + 1:]
        if b"/" not in rest:
            raise ValueError(("invalid_topic_filter", tf))
        group, real = rest.split(b"/", 1)
        if b"+" in group or b"#" in group:
            raise ValueError(("invalid_topic_filter", tf))
        if real.startswith(QUEUE + b"/") or real.startswith(SHARE + b"/"):
            raise ValueError(("invalid_topic_filter", real))
        return Share(group, real), {}
    if tf.startswith(b"$exclusive/"):
        real = tf[len(b"$exclusive/"):]
        if not real:
            raise ValueError(("invalid_topic_filter", tf))
        return real, {"is_exclusive": True}
    return tf, {}


# --- Erlang term order, used to reproduce the ordered walk's return_first / unique
# choices on top of an unordered match set (emqx_trie_search.erl:171-178, :350-356).
# number < atom < tuple < list < binary; atoms compare by name ('#' < '+').

def term_key(x):
    if isinstance(x, bool):
        return (1, str(x).lower())
    if isinstance(x, (int, float)):
        return (0, x)
    if isinstance(x, str):  # atoms
        return (1, x)
    if isinstance(x, tuple):
        return (2, len(x), tuple(term_key(e) for e in x))
    if isinstance(x, list):
        return (3, tuple(term_key(e) for e in x))
    if isinstance(x, (bytes, bytearray)):
        return (4, bytes(x))
    raise TypeError(f"no Erlang term order for {type(x)}")
