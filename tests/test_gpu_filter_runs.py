"""matches_filter/3 in runs form (tm_match_filter_batch_runs): the walk's ranges of the
term-ordered keys cross PCIe instead of its keys, and the host turns them into spans of the
sorted key ids.  Per query, the ids must be the oracle's walk (ALGO_FILTER) id for id, in
walk order, and equal the keys form's ids; bit-exact, no tolerance."""
import random

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads
from tests.test_gpu_filter import _load, _oracle_walks, _pack
from tests.test_oracle_filter import _rand_filter, _rand_set

pytestmark = pytest.mark.gpu


def _check(eng, filters, ids, wf, queries, mode=N.TM_MATCH_ALL):
    buf, off = _pack(queries)
    ro, rids, kcnt, rst = eng.match_filter_runs(buf, off, mode)
    o, c, k, st = eng.match_filter_packed(buf, off, mode)
    assert np.array_equal(rst, st)
    assert np.array_equal(kcnt, c)
    kids = eng.key_ids(k) if len(k) else np.zeros(0, np.uint64)
    omode = oracle.MODE_FIRST if mode == N.TM_MATCH_FIRST else oracle.MODE_ALL
    exp, est = _oracle_walks(filters, ids, wf, queries, omode)
    assert np.array_equal(st, est)
    for i, q in enumerate(queries):
        got = rids[ro[i]:ro[i + 1]]
        assert np.array_equal(got, kids[o[i]:o[i] + c[i]]), q
        if not st[i]:
            assert got.tolist() == [e[1] for e in exp[i]], q
    return int(ro[-1])


@pytest.mark.parametrize("seed", range(4))
def test_filter_runs_random_sets(seed):
    rng = random.Random(0xF1A0 + seed)
    vocab = ["a", "b", "c", "", "$SYS", "zz", "longer-word-than-8"]
    filters, ids, wf = _rand_set(rng, rng.randint(1, 150), vocab)
    queries = [_rand_filter(rng, vocab + ["q"], query=True) for _ in range(400)]
    queries += [b"#/a", b"a/#/+", b"$SYS/#", b"+", b"#", b"", b"/"]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    _check(eng, filters, ids, wf, queries)
    _check(eng, filters, ids, wf, queries, N.TM_MATCH_FIRST)
    with pytest.raises(N.TMError):  # UNIQUE is the keys form's (a map over the whole walk)
        buf, off = _pack(queries)
        eng.match_filter_runs(buf, off, N.TM_MATCH_UNIQUE)


def test_filter_runs_config_e_scaled_and_long_ranges():
    """Config E (scaled) with '+' and '#' variants of its filters, then a set whose '#' runs and
    64-key steps give ranges of thousands of keys; the first batch outgrows the fresh engine's
    range output and is run again."""
    w = workloads.generate("E", scale=0.2, n_topics=100)
    filters = w.filters()
    ids = [int(x) for x in w.f_id]
    rng = random.Random(0xE6)
    queries = [b"#", b"+/#", b"$SYS/#"]
    for f in rng.sample(filters, 3000):
        ws = f.split(b"/")
        r = rng.random()
        if r < 0.4:
            ws[rng.randrange(len(ws))] = b"+"
        elif r < 0.8:
            if ws[-1] == b"#":
                ws = ws[:-1] or [b"x"]
            ws = ws[:rng.randint(1, len(ws))] + [b"#"]
        queries.append(b"/".join(ws))
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    total = _check(eng, filters, ids, [0] * len(filters), queries)
    assert total > 1 << 16
    _check(eng, filters, ids, [0] * len(filters), queries)  # sized now: one run
    # long ranges: 70,000 copies of one word-list filter, '#' runs past FW_BULK keys
    f2 = [b"d/e"] * 70000 + [b"d/f"] * 5000 + [b"d/+"] * 300 + [b"d/e/g"] * 9000
    i2 = list(range(1, len(f2) + 1))
    eng2 = N.Engine(0)
    _load(eng2, f2, i2, [1] * len(f2))
    _check(eng2, f2, i2, [1] * len(f2), [b"d/e", b"d/+", b"+/e", b"d/#", b"#", b"+/+", b"d/e/#", b"d/+/g"])


def test_filter_runs_outlive_a_commit():
    """A runs result stays readable after a commit and another thread-local call rebuilt the
    index: its spans point into the ids the call was made against."""
    rng = random.Random(0xC0)
    vocab = ["a", "b", "c"]
    filters, ids, wf = _rand_set(rng, 100, vocab)
    queries = [_rand_filter(rng, vocab, query=True) for _ in range(200)]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    buf, off = _pack(queries)
    exp = eng.match_filter_runs(buf, off)
    res = eng.match_filter_runs_view(buf, off)
    eng.apply([(N.TM_OP_DEL, f, i, N.TM_KEY_WORDS if w_ else 0) for f, i, w_ in zip(filters, ids, wf)])
    eng.commit()
    assert all(x == [] for x in eng.match_filter(queries))  # the keys form rebuilt the index
    got = eng._expand_runs(res, len(queries))
    for a, b in zip(got, exp):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("split", ["1:1", "64:16", "512:128"])
def test_filter_runs_split_parts(monkeypatch, split):
    """Long one-'+' queries walked as parts, one wave each, cut at child-group starts of the
    '+' level (plan_filter_parts): the query's ids are its parts' in order up to the first part
    that stopped, id for id the oracle's walk (ALL and FIRST)."""
    monkeypatch.setenv("EMQX_TM_FILTER_SPLIT", split)
    rng = random.Random(0x5917)
    filters = []
    for i in range(20000):
        g = rng.randrange(3000)
        tail = rng.choice([b"x", b"y", b"x/z", b"#", b"+", b"x/#", b""])
        filters.append(b"a/b/g%d" % g + (b"/" + tail if tail else b""))
    filters += [b"a/b", b"a/b", b"a", b"a/c/g1/x", b"a/b/#", b"a/+/g7/x", b"$SYS/a/b/x"] * 3
    # the regions of keys that cover the query's literal levels with '+' (R(a, +), R(+, b),
    # R(+, +)) are split as well: many child groups there too
    for i in range(6000):
        g = rng.randrange(2500)
        head = rng.choice([b"a/+", b"+/b", b"+/+"])
        filters.append(head + b"/g%d" % g + rng.choice([b"/x", b"/#", b"", b"/+", b"/x/z", b"/y"]))
    ids = list(range(1, len(filters) + 1))
    wf = [i % 2 for i in range(len(filters))]
    queries = [b"a/b/+/x", b"a/b/+", b"a/b/+/#", b"a/b/+/x/z", b"a/b/+/+", b"a/b/+/y/#", b"a/+/+/x",
               b"+/b/+/x", b"a/b/+/nope", b"a/b/+/x/+", b"$SYS/a/+/x", b"a/b/g7/x", b"a/b/+/+/z"]
    queries += [b"a/b/+/" + rng.choice([b"x", b"y", b"#", b"+", b"x/z", b"q"]) for _ in range(40)]
    eng = N.Engine(0)
    _load(eng, filters, ids, wf)
    _check(eng, filters, ids, wf, queries)
    _check(eng, filters, ids, wf, queries, N.TM_MATCH_FIRST)
