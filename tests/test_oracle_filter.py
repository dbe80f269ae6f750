"""CPU: the oracle's matches_filter/3 restatement (oracle/trie_search.cpp, ALGO_FILTER)
against a second, literal restatement written here: the recursive compare/3 with the
reference's clause order (apps/emqx/src/emqx_trie_search.erl:260-348, incl. the two
"Filter search" clauses :291-300) over a Python sorted list standing in for the ETS
ordered_set, `next` = the smallest key greater than the argument (:230-258).

The reference has no test of matches_filter/3 (no caller either), so there is no golden
vector to pin it to: parity for this row is pinned by the two restatements agreeing and by
the hand-derived cases below, each worked through the clauses in its comment."""
import bisect
import random

import numpy as np
import pytest

import oracle

END = object()


def _ord(w):
    # Erlang term order of a word: atoms '#' < '+' < every binary; binaries bytewise
    return (0,) if w == "#" else (1,) if w == "+" else (2, w)


def _words(f: bytes):
    # filter_words/1 (:356-366): tokens, "+" / "#" -> the atoms, everything else binary
    f = f.encode() if isinstance(f, str) else f
    return ["#" if t == b"#" else "+" if t == b"+" else t for t in f.split(b"/")]


def _wild(ws):
    return any(w in ("#", "+") for w in ws)


class RefIndex:
    """ETS ordered_set of keys {Words, {ID}} (list) or {Binary, {ID}} (make_key/2, :115-128)."""

    def __init__(self, filters, ids, word_form):
        self.keys = []
        for f, i, wf in zip(filters, ids, word_form):
            ws = _words(f)
            if _wild(ws) or wf:
                self.keys.append((0, tuple(_ord(w) for w in ws), (i,), ("L", tuple(ws), i)))
            else:
                self.keys.append((1, f, (i,), ("B", f, i)))
        self.keys.sort(key=lambda k: k[:3])
        self.sort_keys = [k[:3] for k in self.keys]

    def next(self, probe):
        j = bisect.bisect_right(self.sort_keys, probe)
        return END if j == len(self.keys) else self.keys[j]

    def base(self, prefix):  # {Prefix, {}}: () sorts before every (ID,)
        return (0, tuple(_ord(w) for w in prefix), ())


def compare(F, W, pos):
    """compare/3, one Erlang clause per branch, in source order."""
    if F is None:  # compare(NotFilter, _, _) when is_binary(NotFilter)
        return "lower"
    if not F and not W:
        return "full"
    if not F:
        return "prefix"
    if F == ["#"]:
        return "full"
    if W == ["#"]:  # filter search
        return "full"
    if W and W[0] == "+":  # compare([_ | TF], ['+' | TW], Pos): filter search
        return compare(F[1:], W[1:], pos + 1)
    if F[0] == "+" and W:
        r = compare(F[1:], W[1:], pos + 1)
        return ("seek", pos, W[0]) if r == "lower" else r
    if W and F[0] == W[0]:
        return compare(F[1:], W[1:], pos + 1)
    if W and _ord(F[0]) > _ord(W[0]):
        return "lower"
    if not W:
        return "lower"
    return ("seek", pos, W[0])


def ref_matches_filter(ix: RefIndex, q: bytes):
    """search/3 with topic_filter set (:192-228): returns the accumulator as the reference
    would, i.e. the matched keys in REVERSE walk order."""
    W = list(q) if isinstance(q, (list, tuple)) else _words(q)  # a word list is taken as is (:359-360)
    w0 = W[0] if W else None
    base = [w0] if isinstance(w0, bytes) and w0.startswith(b"$") else []  # base_init/1 :160-163
    cur = ix.next(ix.base(base))
    acc = []
    while cur is not END:
        kind, _, _, (form, ws, i) = cur
        r = compare(list(ws) if form == "L" else None, W, 0)
        if r == "full":
            acc.insert(0, (ws, i))
            cur = ix.next(cur[:3])
        elif r == "prefix":
            cur = ix.next(cur[:3])
        elif r == "lower":
            break
        else:
            _, pos, sw = r
            cur = ix.next(ix.base(list(ws[:pos]) + [sw]))
    return acc


def oracle_matches_filter(filters, ids, word_form, queries, mode=oracle.MODE_ALL):
    ix = oracle.OrderedIndex.from_filters(filters, ids, word_form)
    qb = b"".join(queries)
    qo = np.zeros(len(queries) + 1, dtype=np.uint32)
    qo[1:] = np.cumsum([len(q) for q in queries])
    buf = np.frombuffer(qb + b"\0", dtype=np.uint8)
    off, got_ids, st, src = ix.match(buf, qo, algo=oracle.ALGO_FILTER, mode=mode, with_src=True)
    assert not st.any()  # valid filters only: no badarg status
    out, k = [], 0
    for t in range(len(queries)):
        c = int(off[t + 1] - off[t])
        out.append([(tuple(_words(filters[s])), int(ids[s])) for s in src[k:k + c]])
        k += c
    return out


def _rand_filter(rng, vocab, query=False):
    n = rng.randint(1, 5)
    ws = []
    for i in range(n):
        r = rng.random()
        if r < 0.2:
            ws.append("+")
        elif r < 0.3 and (not query or i == n - 1):
            # keys: also mid-filter (a dead key, still a word-list key in the set); queries:
            # last level only (see test_filter_search_mid_hash_is_badarg)
            ws.append("#")
        else:
            ws.append(rng.choice(vocab))
    return "/".join(ws).encode()


def _rand_set(rng, nkeys, vocab):
    seen, filters, ids, wf = set(), [], [], []
    while len(filters) < nkeys:
        f = _rand_filter(rng, vocab)
        i = rng.randint(0, 9)
        w = int(rng.random() < 0.15)
        key = (tuple(_words(f)), i) if (_wild(_words(f)) or w) else (f, i)
        if key in seen:
            continue
        seen.add(key)
        filters.append(f)
        ids.append(i)
        wf.append(w)
    return filters, ids, wf


@pytest.mark.parametrize("seed", range(12))
def test_filter_search_two_restatements_agree(seed):
    rng = random.Random(0xF117E4 + seed)
    vocab = ["a", "b", "c", "", "$SYS", "$x", "zz"]
    filters, ids, wf = _rand_set(rng, rng.randint(1, 60), vocab)
    queries = [_rand_filter(rng, vocab + ["q"], query=True) for _ in range(200)]
    got = oracle_matches_filter(filters, ids, wf, queries)
    rix = RefIndex(filters, ids, wf)
    for q, g in zip(queries, got):
        exp = ref_matches_filter(rix, q)
        assert g == exp[::-1], (q, g, exp)


def _wl(s):
    return tuple(_words(s.encode()))


def test_filter_search_hand_cases():
    # keys (all word lists): a/+ , a/b/# , # , +/b , a/#/c (dead), $SYS/#
    fs = ["a/+", "a/b/#", "#", "+/b", "a/#/c", "$SYS/#"]
    ids = [1, 2, 3, 4, 5, 6]
    got = dict(zip(["a/#", "+/b", "$SYS/x", "a/b", "x/y/z"],
                   oracle_matches_filter(fs, ids, [0] * 6, [b"a/#", b"+/b", b"$SYS/x", b"a/b", b"x/y/z"])))
    # term order: [#] < [+, b] < [$SYS, #] < [a, #, c] < [a, +] < [a, b, #]   ('$' < 'a')
    # "a/#": [#] full (compare(['#'], _)); [+, b]: '+' takes a, then W == ['#'] -> full;
    #        [$SYS, #]: $SYS < a -> seek {0, a}; [a, #, c]: a = a, W == ['#'] -> full;
    #        [a, +] full; [a, b, #] full; end of table
    assert got["a/#"] == [(_wl("#"), 3), (_wl("+/b"), 4), (_wl("a/#/c"), 5), (_wl("a/+"), 1), (_wl("a/b/#"), 2)]
    # "+/b": [#] full; [+, b]: query '+' passes through, b = b -> full; [$SYS, #]: '+', then
    #        F == ['#'] -> full; [a, #, c]: '+', then '#' < b -> {1, b} (no backtrack point: a
    #        query '+' is not one) -> next({[a, b], {}}) = [a, b, #]: full.  [a, +] is skipped.
    assert got["+/b"] == [(_wl("#"), 3), (_wl("+/b"), 4), (_wl("$SYS/#"), 6), (_wl("a/b/#"), 2)]
    # "$SYS/x": base_init starts at [$SYS]: [$SYS, #] full; [a, #, c]: a > $SYS -> lower
    assert got["$SYS/x"] == [(_wl("$SYS/#"), 6)]
    # "a/b": [#] full; [+, b]: filter '+' then b = b -> full; [$SYS, #] -> {0, a};
    #        [a, #, c]: '#' < b -> {1, b} -> [a, b, #] full.  [a, +] is skipped by the seek.
    assert got["a/b"] == [(_wl("#"), 3), (_wl("+/b"), 4), (_wl("a/b/#"), 2)]
    # "x/y/z": [#] full; [+, b]: b < y -> {1, y}, passed through the '+' -> [$SYS, #]:
    #        $SYS < x -> {0, x} -> no key >= [x]: end of table
    assert got["x/y/z"] == [(_wl("#"), 3)]


def test_filter_search_modes():
    fs = ["a/+", "a/#", "+/+", "a/+"]
    ids = [7, 7, 8, 9]
    ix = oracle.OrderedIndex.from_filters(fs, ids)
    q = np.frombuffer(b"a/b\0", dtype=np.uint8)
    qo = np.array([0, 3], dtype=np.uint32)
    off, got, st, src = ix.match(q, qo, algo=oracle.ALGO_FILTER, mode=oracle.MODE_FIRST, with_src=True)
    assert len(src) == 1 and (fs[src[0]], ids[src[0]]) == ("+/+", 8)  # the least key in term order
    off, got, st = ix.match(q, qo, algo=oracle.ALGO_FILTER, mode=oracle.MODE_UNIQUE)
    assert list(got) == [7, 8, 9]


def test_filter_search_mid_hash_is_badarg():
    # query "#/y" over [+, z]: compare([z], [y]) is lower, the '+' turns it into {0, '#'},
    # and next({['#'], {}}) is [+, z] again -- the reference's walk never ends.  The
    # restatement (and the engine) refuse such a query with the badarg status.
    ix = oracle.OrderedIndex.from_filters(["+/z"], [1])
    q = np.frombuffer(b"#/y\0", dtype=np.uint8)
    off, got, st = ix.match(q, np.array([0, 3], dtype=np.uint32), algo=oracle.ALGO_FILTER)
    assert list(st) == [1] and off[-1] == 0


@pytest.mark.parametrize("seed", range(4))
def test_word_list_topics_map_to_filter_search(seed):
    """matches/3 of a pre-split topic (emqx_trie_search.erl:182,369-370): the literal
    restatement walks the word list as given (no badarg; '+'/'#' atoms are wildcards of the
    topic); the mirror hands the engine words_topic_bytes(...) through matches_filter, which
    the oracle's filter walk answers here.  Both must agree key by key.  Words with no byte
    form (<<"+">>, <<"#">>, words with '/') are refused."""
    from emqx_amd.topic_index import words_topic_bytes
    rng = random.Random(100 + seed)
    svocab = ["a", "b", "c", "$SYS", ""]
    vocab = [v.encode() for v in svocab]
    filters, ids, wf = _rand_set(rng, 300, svocab)
    rix = RefIndex(filters, ids, wf)
    odd = [b"zz", b"$x", b"\xff"]
    for w in (b"+", b"#", b"a/b"):
        with pytest.raises(ValueError):
            words_topic_bytes([b"a", w])
    topics = []
    for _ in range(300):
        n = rng.randint(1, 5)
        ws = []
        for k in range(n):
            r = rng.random()
            if r < 0.1:
                ws.append("+")
            elif r < 0.15 and k == n - 1:
                ws.append("#")
            elif r < 0.35:
                ws.append(rng.choice(odd))
            else:
                ws.append(rng.choice(vocab))
        topics.append(ws)
    qs = [words_topic_bytes(t) for t in topics]
    got = oracle_matches_filter(filters, ids, wf, qs)
    for t, q, g in zip(topics, qs, got):
        exp = [(tuple(ws), i) for ws, i in ref_matches_filter(rix, t)]
        assert g == exp[::-1], (t, q)
