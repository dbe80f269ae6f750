"""GPU parity of matches_filter/3 (tm_match_filter_batch, filter_kernels.hip k_filter_walk)
against the oracle's restatement of the reference's filter search (ALGO_FILTER), which
tests/test_oracle_filter.py checks against a literal recursive restatement and hand-worked
cases.  The walk order itself is compared (key by key), not just the sets: integer work,
bit-exact, no tolerance."""
import random

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads
from tests.test_oracle_filter import RefIndex, _rand_filter, _rand_set, _words, ref_matches_filter

pytestmark = pytest.mark.gpu


def _pack(qs):
    off = np.zeros(len(qs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(q) for q in qs])
    return np.frombuffer(b"".join(qs) + b"\0", dtype=np.uint8), off


def _oracle_walks(filters, ids, wf, queries, mode=oracle.MODE_ALL):
    ix = oracle.OrderedIndex.from_filters(filters, ids, wf)
    buf, off = _pack(queries)
    o, got_ids, st, src = ix.match(buf, off, algo=oracle.ALGO_FILTER, mode=mode, with_src=True)
    walks, k = [], 0
    for t in range(len(queries)):
        c = int(o[t + 1] - o[t]) if mode != oracle.MODE_UNIQUE else None
        if mode == oracle.MODE_UNIQUE:
            walks.append(sorted(int(x) for x in got_ids[o[t]:o[t + 1]]))
            continue
        walks.append([(tuple(_words(filters[s])), int(ids[s])) for s in src[k:k + c]])
        k += c
    return walks, st


def _engine_walks(eng, queries, mode=N.TM_MATCH_ALL):
    res = eng.match_filter(queries, mode)
    out = []
    for hs in res:
        if hs is None:
            out.append(None)
            continue
        keys = []
        for h in hs:
            u, fb, flags = eng.key_info(h)
            keys.append((tuple(_words(fb)), int(u)))
        out.append(keys)
    return out


def _load(eng, filters, ids, wf):
    eng.apply([(N.TM_OP_ADD, f, i, N.TM_KEY_WORDS if w else 0) for f, i, w in zip(filters, ids, wf)])
    eng.commit()


@pytest.mark.parametrize("seed", range(8))
def test_filter_walk_matches_oracle(seed):
    rng = random.Random(0xF1170 + seed)
    vocab = ["a", "b", "c", "", "$SYS", "$x", "zz", "longer-word-than-8"]
    filters, ids, wf = _rand_set(rng, rng.randint(1, 120), vocab)
    queries = [_rand_filter(rng, vocab + ["q"], query=True) for _ in range(400)]
    queries += [b"#/a", b"a/#/+", b"$SYS/#", b"+", b"#", b"", b"/", b"$"]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    got = _engine_walks(eng, queries)
    exp, st = _oracle_walks(filters, ids, wf, queries)
    for q, g, e, s in zip(queries, got, exp, st):
        if s:
            assert g is None, q
        else:
            assert g == e, (q, g, e)
    # and against the literal recursive restatement (the reference's list is the walk reversed)
    rix = RefIndex(filters, ids, wf)
    for q, g, s in zip(queries, got, st):
        if not s:
            assert g == ref_matches_filter(rix, q)[::-1], q


@pytest.mark.parametrize("seed", range(3))
def test_filter_modes_match_oracle(seed):
    rng = random.Random(0xF1F0 + seed)
    vocab = ["a", "b", "c", "$SYS"]
    filters, ids, wf = _rand_set(rng, 80, vocab)
    queries = [_rand_filter(rng, vocab, query=True) for _ in range(300)]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    first = _engine_walks(eng, queries, N.TM_MATCH_FIRST)
    exp_first, _ = _oracle_walks(filters, ids, wf, queries, oracle.MODE_FIRST)
    assert first == exp_first
    uniq = eng.match_filter(queries, N.TM_MATCH_UNIQUE)
    exp_uniq, _ = _oracle_walks(filters, ids, wf, queries, oracle.MODE_UNIQUE)
    for q, hs, e in zip(queries, uniq, exp_uniq):
        got_ids = [int(i) for i in eng.key_ids(np.array(hs, dtype=np.uint32))] if hs else []
        assert got_ids == e, q  # one key per id, listed by id


def test_filter_index_follows_epochs():
    rng = random.Random(0xEE)
    vocab = ["a", "b", "c", "d"]
    filters, ids, wf = _rand_set(rng, 100, vocab)
    queries = [_rand_filter(rng, vocab, query=True) for _ in range(300)]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    assert _engine_walks(eng, queries) == _oracle_walks(filters, ids, wf, queries)[0]
    # delete half, add new keys (same filters with other ids, new filters), commit
    keep = [i for i in range(len(filters)) if i % 2]
    eng.apply([(N.TM_OP_DEL, filters[i], ids[i], N.TM_KEY_WORDS if wf[i] else 0)
               for i in range(len(filters)) if not i % 2])
    f2, i2, w2 = [filters[i] for i in keep], [ids[i] for i in keep], [wf[i] for i in keep]
    seen = {(tuple(_words(f)), i) for f, i in zip(f2, i2)}
    add = []
    while len(add) < 60:
        f = _rand_filter(rng, vocab + ["e"])
        i = rng.randint(10, 20)
        if (tuple(_words(f)), i) in seen:
            continue
        seen.add((tuple(_words(f)), i))
        add.append((f, i))
    eng.apply([(N.TM_OP_ADD, f, i, 0) for f, i in add])
    eng.commit()
    # a wildcard-free filter added in binary form is a {Binary, {ID}} key: drop it from the
    # oracle's set the same way (the oracle decides word-list vs binary from the flags)
    f2 += [f for f, _ in add]
    i2 += [i for _, i in add]
    w2 += [0] * len(add)
    assert _engine_walks(eng, queries) == _oracle_walks(f2, i2, w2, queries)[0]


def test_filter_empty_index_and_empty_batch():
    eng = N.Engine(0)
    assert eng.match_filter([b"a/#", b"+"]) == [[], []]
    assert eng.match_filter([]) == []
    _load(eng, ["a/b"], [1], [0])  # a binary key only: the walk never meets it
    assert eng.match_filter([b"a/b", b"#", b"a/+"]) == [[], [], []]


def test_filter_walk_config_a():
    """Config A's 10 K route keys; queries are its own filters, generalised ('+' for a
    level, '#' for a tail) -- long walks with many seeks."""
    w = workloads.generate("A", n_topics=1000)
    filters = w.filters()
    ids = [int(x) for x in w.f_id]
    rng = random.Random(0xA11)
    queries = []
    for f in rng.sample(filters, 1500):
        ws = f.split(b"/")
        r = rng.random()
        if r < 0.3:
            ws[rng.randrange(len(ws))] = b"+"
        elif r < 0.6:
            ws = ws[:rng.randint(0, len(ws) - 1)] + [b"#"]
        queries.append(b"/".join(ws))
    queries += [b"#", b"+/#", b"+/+/+/+", b"$SYS/#"]
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    got = _engine_walks(eng, queries)
    exp, st = _oracle_walks(filters, ids, [0] * len(filters), queries)
    assert not st.any()
    bad = [q for q, g, e in zip(queries, got, exp) if g != e]
    assert not bad, bad[:5]
    assert sum(len(g) for g in got) > 1000  # the walks did find keys


def test_topic_index_matches_filter_order():
    from emqx_amd.topic_index import TopicIndex
    tab = TopicIndex(0)
    fs = ["a/+", "a/b/#", "#", "+/b", "a/#/c", "$SYS/#"]
    for i, f in enumerate(fs, 1):
        tab.insert(f.encode(), i)
    rix = RefIndex([f.encode() for f in fs], list(range(1, 7)), [0] * 6)
    for q in [b"a/#", b"+/b", b"$SYS/x", b"a/b", b"x/y/z"]:
        got = [(k[0], k[1][0]) for k in tab.matches_filter(q)]
        exp = [(tuple(ws), i) for ws, i in ref_matches_filter(rix, q)]
        assert got == exp, q
    with pytest.raises(ValueError):
        tab.matches_filter(b"#/a")


def test_filter_walk_config_e_scaled():
    """Config E (scaled): $SYS topics, root '#', '+/...' and $share duplicates (same filter,
    several dests); queries include '$SYS/...' ones (base_init starts at [W0])."""
    w = workloads.generate("E", scale=0.2, n_topics=2000)
    filters = w.filters()
    ids = [int(x) for x in w.f_id]
    rng = random.Random(0xE5)
    queries = []
    for f in rng.sample(filters, 1500):
        ws = f.split(b"/")
        r = rng.random()
        if r < 0.3:
            ws[rng.randrange(len(ws))] = b"+"
        elif r < 0.6:
            if ws[-1] == b"#":
                ws = ws[:-1] or [b"x"]
            ws = ws[:rng.randint(1, len(ws))] + [b"#"]
        queries.append(b"/".join(ws))
    queries += [t for t in w.topics()[:500] if t.startswith(b"$SYS")][:100]
    queries += [b"$SYS/#", b"$SYS/+/+/#", b"#", b"+/#"]
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    got = _engine_walks(eng, queries)
    exp, st = _oracle_walks(filters, ids, [0] * len(filters), queries)
    assert not st.any()
    bad = [q for q, g, e in zip(queries, got, exp) if g != e]
    assert not bad, bad[:5]


def test_filter_walk_one_pass_and_two_pass_agree():
    """The one-pass walk (keys chunked on the device, one output reservation per query) and
    the count + emit passes give the same walks.  The first batch of a fresh engine is sized
    for 64 Ki keys: a batch returning more takes the two-pass path, which sizes the next
    batch for the one pass."""
    w = workloads.generate("E", scale=0.2, n_topics=100)
    filters = w.filters()
    ids = [int(x) for x in w.f_id]
    rng = random.Random(0x1F)
    queries = [b"#", b"+/#"] + [b"/".join(f.split(b"/")[:2]) + b"/#" for f in rng.sample(filters, 600)]
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    exp, st = _oracle_walks(filters, ids, [0] * len(filters), queries)
    assert sum(len(e) for e in exp) > 1 << 16
    got1 = _engine_walks(eng, queries)
    s1 = eng.stats()
    got2 = _engine_walks(eng, queries)
    s2 = eng.stats()
    assert s1["n_filter_twopass"] == 1 and s2["n_filter_onepass"] == s1["n_filter_onepass"] + 1
    assert got1 == exp and got2 == exp
    # a small batch after it: one pass
    small = queries[2:50]
    assert _engine_walks(eng, small) == exp[2:50]


def test_topic_index_word_list_topics():
    """matches/3 with a pre-split topic (emqx_trie_search.erl:182,369-370) through the
    mirror: the engine's filter walk of the joined words, against the literal restatement
    walking the list itself; [] reaches only the root '#' keys (compare/3 :282-290, :333-340)."""
    from emqx_amd.topic_index import TopicIndex
    tab = TopicIndex(0)
    fs = ["a/+", "a/b/#", "#", "+/b", "a/b", "$SYS/#", "+", "+/+/c"]
    for i, f in enumerate(fs, 1):
        tab.insert(f.encode(), i)
    tab.insert([b"a", b"b"], 20)  # a word-list key without wildcards
    rix = RefIndex([f.encode() for f in fs] + [b"a/b"], list(range(1, 9)) + [20], [0] * 8 + [1])
    for ws in ([b"a", b"b"], [b"a", "+"], ["+", b"b"], [b"$SYS", b"x"], [b"x", b"y", b"c"], [b"a", "#"], []):
        got = [(k[0] if isinstance(k[0], tuple) else k[0], k[1][0]) for k in tab.matches(ws)]
        exp = [(tuple(w), i) for w, i in ref_matches_filter(rix, ws)]
        assert sorted(got, key=repr) == sorted(exp, key=repr), ws
    # a binary exact key never matches a word-list topic (match_topics/4, :381-389) ...
    assert (b"a/b", (5,)) not in tab.matches([b"a", b"b"])
    # ... but does match the same topic as a binary
    assert (b"a/b", (5,)) in tab.matches(b"a/b")


def test_filter_walk_long_full_steps_and_bulk_ranges():
    """Steps where all 64 keys are match_full without a query '#' (70,000 copies of one
    word-list filter under different ids: the one-pass chain stores them as 64-key ranges), and
    '#'-query runs longer than FW_BULK keys (copied by k_filter_bulk), through both the
    two-pass path (the first batch: more than the 64 Ki keys a fresh engine sizes for) and
    the one-pass path (the second), walk order against the oracle."""
    filters = [b"d/e"] * 70000 + [b"d/f"] * 5000 + [b"d/+"] * 300 + [b"d/e/g"] * 9000 + [b"x/#"] * 10
    ids = list(range(1, len(filters) + 1))
    wf = [1] * len(filters)  # word-list keys: {Binary, {ID}} keys end a filter search
    queries = [b"d/e", b"d/+", b"+/e", b"d/#", b"#", b"+/+", b"d/e/#", b"x/y", b"d/+/g"]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    exp, st = _oracle_walks(filters, ids, wf, queries)
    assert not st.any() and sum(len(e) for e in exp) > 1 << 16
    got1 = _engine_walks(eng, queries)
    got2 = _engine_walks(eng, queries)
    s = eng.stats()
    assert s["n_filter_twopass"] >= 1 and s["n_filter_onepass"] >= 1
    for q, g1, g2, e in zip(queries, got1, got2, exp):
        assert g1 == e, q
        assert g2 == e, q
    first = _engine_walks(eng, queries, N.TM_MATCH_FIRST)
    exp_first, _ = _oracle_walks(filters, ids, wf, queries, oracle.MODE_FIRST)
    assert first == exp_first
