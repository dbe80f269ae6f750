"""GPU parity: the HIP engine (through the C-ABI) against the CPU restatement of the
reference (oracle/) and the reference's own known-answer cases.  Bit-exact sorted
matched-id sets; integer work, no tolerance."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads
from oracle import emqx_topic as et
from tests.kat import run_index_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[False, True], ids=["fast", "spill"])
def mode(request):
    return request.param


def _engine(force_slow=False, **kw):
    return N.Engine(0, force_slow=force_slow, **kw)


def _engine_sets(eng, t_bytes, t_off, mode=N.TM_MATCH_ALL):
    off, cnt, keys, st = eng.match_packed(t_bytes, t_off, mode)
    ids = eng.key_ids(keys)
    return off, cnt, ids, st


def _assert_same(eng_res, orc_res, what=""):
    off, cnt, ids, st = eng_res
    eo, eids, est = orc_res
    assert np.array_equal(st, est), what
    assert np.array_equal(cnt.astype(np.int64), np.diff(eo).astype(np.int64)), what
    bad = []
    for i in range(len(cnt)):
        got = np.sort(ids[off[i]:off[i] + cnt[i]])
        if not np.array_equal(got, eids[eo[i]:eo[i + 1]]):
            bad.append(i)
            if len(bad) > 5:
                break
    assert not bad, f"{what}: topics {bad} differ"


def _load(eng, w):
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()


# ------------------------------------------------------------------ reference KATs
def test_index_kats_gpu(golden, mode):
    from emqx_amd.topic_index import TopicIndex
    errs = []
    for case in golden("kat_index.json"):
        run_index_case(case, lambda: TopicIndex(0, force_slow=mode), lambda c, m: c or errs.append(m))
    assert not errs, "\n".join(errs)


def test_router_kats_gpu(golden):
    from emqx_amd.router import Router
    from tests.kat import run_router_case
    for case in golden("kat_router.json"):
        run_router_case(case, Router(0, node="node"))


def test_filter_kats_key_form_gpu(golden):
    """emqx_trie_search_tests:filter_test_ :23-33 through the engine: a wildcard filter's
    key comes back as its word list (the empty level a binary), a filter without
    wildcards as its binary (make_key/2, emqx_trie_search.erl:115-128)."""
    from emqx_amd.topic_index import TopicIndex
    ix = TopicIndex(0)
    cases = golden("kat_topic.json")["filter"]
    for n, (t, _) in enumerate(cases):
        ix.insert(t.encode(), n)
    for n, (t, exp) in enumerate(cases):
        topic = t.replace("+", "x").replace("#", "y").encode()
        keys = [k for k in ix.matches(topic, None, []) if k[1] == (n,)]
        want = tuple(w["atom"] if isinstance(w, dict) else w.encode() for w in exp) if exp else t.encode()
        assert keys == [(want, (n,))], (t, keys)


def test_config_a_golden_sample_gpu(golden, mode):
    g = golden("config_a_sample.json")
    eng = _engine(mode)
    eng.apply([(N.TM_OP_ADD, f, i) for f, i in zip(g["filters"], g["ids"])])
    eng.commit()
    res = eng.match(g["topics"])
    for i, exp in enumerate(g["expected"]):
        assert sorted(eng.key_ids(np.array(res[i], dtype=np.uint32)).tolist()) == exp, g["topics"][i]


# ------------------------------------------------------------- seeded configs
@pytest.mark.parametrize("name,scale,nt", [("A", 1.0, 100_000), ("B", 0.2, 50_000), ("C", 0.02, 50_000),
                                           ("E", 0.1, 50_000)])
def test_config_parity(name, scale, nt, mode):
    w = workloads.generate(name, scale=scale, n_topics=nt)
    eng = _engine(mode)
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    exp = ix.match(w.t_bytes, w.t_off, threads=8)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, name)
    if not mode:
        # pools are sized from the first batch's demand: a repeat batch never spills
        _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, name + " (repeat)")
        assert eng.stats()["n_slow_topics"] == 0


def test_host_batch_pipelined_vs_oracle(mode):
    """tm_match_batch at >= 2 x 262,144 topics runs as sub-batches on two streams (each
    sub-batch's walk overlaps the previous one's D2H, engine.cpp match_batch_pipelined):
    the joined result is the oracle's.  The first call starts with key halves far too small
    (no estimate yet), so it also takes the grow-and-rewalk path; the repeat uses the
    estimate.  Afterwards the device holds no single batch: tm_result_ids_device refuses."""
    w = workloads.generate("C", scale=0.02, n_topics=800_000)
    eng = _engine(mode)
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    exp = ix.match(w.t_bytes, w.t_off, threads=8)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, "pipelined")
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, "pipelined (repeat)")
    import torch
    ids = torch.zeros(16, dtype=torch.int64, device="cuda:0")
    lo = torch.zeros(16, dtype=torch.int32, device="cuda:0")
    with pytest.raises(N.TMError):
        eng.result_ids_device(ids.data_ptr(), 16, lo.data_ptr())


@pytest.mark.parametrize("tpw", [4, 16, 64])
@pytest.mark.parametrize("name,scale,nt", [("A", 1.0, 50_000), ("C", 0.02, 50_000), ("E", 0.1, 50_000)])
def test_config_parity_topics_per_wave(name, scale, nt, tpw):
    """Every wave width (tm_config.topics_per_wave) gives the same sets; test-sized batches
    otherwise run at the narrow width the batch size picks."""
    w = workloads.generate(name, scale=scale, n_topics=nt)
    eng = _engine(topics_per_wave=tpw)
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), ix.match(w.t_bytes, w.t_off, threads=8), f"{name} tpw={tpw}")


def test_modes_unique_first_vs_oracle():
    w = workloads.generate("E", scale=0.02, n_topics=4000)
    eng = _engine()
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off, N.TM_MATCH_UNIQUE),
                 ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_UNIQUE), "unique")
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off, N.TM_MATCH_FIRST),
                 ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_FIRST), "first")


@pytest.mark.parametrize("name,scale,nt", [("A", 1.0, 20_000), ("B", 0.05, 20_000), ("C", 0.01, 20_000),
                                           ("E", 0.05, 20_000)])
def test_device_first_and_count_modes(name, scale, nt):
    """TM_MATCH_FIRST runs k_match_first (return_first, emqx_trie_search.erl:171-178) and
    TM_MATCH_COUNT skips the key copy-out (has_any_route/1 is cnt > 0)."""
    w = workloads.generate(name, scale=scale, n_topics=nt)
    eng = _engine()
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off, N.TM_MATCH_FIRST),
                 ix.match(w.t_bytes, w.t_off, mode=oracle.MODE_FIRST, threads=8), f"first {name}")
    o_all, c_all, _, s_all = eng.match_packed(w.t_bytes, w.t_off)
    _, c_cnt, k_cnt, s_cnt = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_COUNT)
    assert np.array_equal(c_all, c_cnt) and np.array_equal(s_all, s_cnt) and len(k_cnt) == 0


def test_device_first_mode_through_device_api():
    import torch
    w = workloads.generate("E", scale=0.05, n_topics=10_000)
    eng = _engine()
    _load(eng, w)
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), w.n_topics, int(w.t_off[-1]), N.TM_MATCH_FIRST)
    eng.device_sync()
    import ctypes as C
    n = w.n_topics
    cnt_t = torch.empty(n, dtype=torch.int32, device=dev)
    keys_t = torch.empty(n, dtype=torch.int32, device=dev)
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert lib.hipMemcpy(C.c_void_p(cnt_t.data_ptr()), C.c_void_p(r.d_cnt), 4 * n, 3) == 0
    assert lib.hipMemcpy(C.c_void_p(keys_t.data_ptr()), C.c_void_p(r.d_keys), 4 * n, 3) == 0
    cnt = cnt_t.cpu().numpy().view(np.uint32)
    keys = keys_t.cpu().numpy().view(np.uint32)
    off, hcnt, hkeys, _ = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_FIRST)
    assert np.array_equal(cnt, hcnt)
    assert np.array_equal(keys[cnt == 1], hkeys)


def test_first_mode_term_order_kats():
    """Term order of matching keys (Erlang: lists < binaries; '#' < '+' < binary words; a
    shorter list first; then {ID}): KATs for the device FIRST walk."""
    eng = _engine()
    ops = [(N.TM_OP_ADD, b"a/b", 1), (N.TM_OP_ADD, b"a/b", 2, N.TM_KEY_WORDS), (N.TM_OP_ADD, b"a/+", 5),
           (N.TM_OP_ADD, b"a/#", 9), (N.TM_OP_ADD, b"a/#", 7), (N.TM_OP_ADD, b"+/b", 3), (N.TM_OP_ADD, b"#", 8),
           (N.TM_OP_ADD, b"x/y", 4), (N.TM_OP_ADD, b"x/y", 6), (N.TM_OP_ADD, b"$s/+", 10), (N.TM_OP_ADD, b"$s/q", 11)]
    eng.apply(ops)
    eng.commit()
    first = lambda t: [eng.key_info(k)[0] for k in eng.match([t], N.TM_MATCH_FIRST)[0]]  # noqa: E731
    assert first(b"a/b") == [8]       # ['#'] is the smallest list
    assert first(b"x/y") == [8]
    assert first(b"$s/q") == [10]     # no root '#' for '$' topics; ['$s','+'] < <<"$s/q">>
    eng.apply([(N.TM_OP_DEL, b"#", 8)])
    eng.commit()
    assert first(b"a/b") == [3]       # ['+', b] < ['a', ...]
    assert first(b"x/y") == [4]       # only binaries: smallest id
    eng.apply([(N.TM_OP_DEL, b"+/b", 3)])
    eng.commit()
    assert first(b"a/b") == [7]       # ['a','#'] (ids 7, 9) < ['a','+'] < ['a','b'] < <<"a/b">>
    eng.apply([(N.TM_OP_DEL, b"a/#", 7), (N.TM_OP_DEL, b"a/#", 9)])
    eng.commit()
    assert first(b"a/b") == [5]
    eng.apply([(N.TM_OP_DEL, b"a/+", 5)])
    eng.commit()
    assert first(b"a/b") == [2]       # the word-list key sorts before the binary one
    assert first(b"q") == []


def _random_shape_index(seed, n_filters=4000, n_topics=6000, levels=9, vocab=6):
    """Filters over a tiny vocabulary with '+' and '#' at every depth (many matching keys of
    every shape per topic: the FIRST walk's pruning decides between them), word-list and
    binary exact keys, $-topics; topics of 1..levels levels."""
    rng = np.random.default_rng(seed)
    words = [b"w%d" % i for i in range(vocab)] + [b"", b"$s"]
    ops = []
    for i in range(n_filters):
        nl = int(rng.integers(1, levels + 1))
        ws = [words[int(rng.integers(0, vocab))] for _ in range(nl)]
        for j in range(nl):
            if rng.random() < 0.25:
                ws[j] = b"+"
        if rng.random() < 0.3:
            ws = ws[:int(rng.integers(0, nl + 1))] + [b"#"]
        f = b"/".join(ws)
        fl = N.TM_KEY_WORDS if (b"+" not in ws and b"#" not in ws and rng.random() < 0.5) else 0
        ops.append((N.TM_OP_ADD, f, int(rng.integers(0, 50)), fl))
    topics = []
    for _ in range(n_topics):
        nl = int(rng.integers(1, levels + 1))
        ts = [words[int(rng.integers(0, len(words)))] for _ in range(nl)]
        topics.append(b"/".join(ts))
    return ops, topics


def _oracle_first(ops, topics):
    keys = {}
    for op, f, i, fl in ops:
        keys[(f, i, fl)] = True
    ks = sorted(keys)
    ix = oracle.OrderedIndex.from_filters([k[0] for k in ks], [k[1] for k in ks], [k[2] for k in ks])
    buf, off = N.pack_topics(topics)
    return ix.match(buf, off, mode=oracle.MODE_FIRST, threads=8), (buf, off)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("variant", ["wave", "tpw4", "spill", "pool1"])
def test_first_wave_vs_oracle_random_shapes(seed, variant):
    """k_match_first_wave (term-order codes, pruning) == the oracle's return_first walk,
    key for key, on indexes dense in '+' / '#' shapes; also at 4 topics per wave, with every
    topic forced through the DFS spill kernel, and with the frontier pool exhausted (topics
    hand off to k_first_slow mid-walk)."""
    ops, topics = _random_shape_index(seed)
    kw = {"wave": {}, "tpw4": {"topics_per_wave": 4}, "spill": {"force_slow": True},
          "pool1": {"seg_chunks": 1, "topics_per_wave": 64}}[variant]
    eng = _engine(**kw)
    eng.apply(ops)
    eng.commit()
    assert eng.stats()["n_deep_keys"] == 0
    exp, (buf, off) = _oracle_first(ops, topics)
    _assert_same(_engine_sets(eng, buf, off, N.TM_MATCH_FIRST), exp, f"first {variant} seed {seed}")
    eng.close()


def test_first_deep_binary_and_deep_word_keys():
    """Keys past the 31-level order code: a {Binary, {ID}} key 40 levels deep is found by the
    wave walk (it follows the all-literal path past depth 30); a 35-level word-list key
    switches the engine to the lane-per-topic DFS (n_deep > 0); both agree with the oracle."""
    deep = b"/".join(b"L%d" % i for i in range(40))
    base = [(N.TM_OP_ADD, deep, 1, 0), (N.TM_OP_ADD, b"L0/+/L2/#", 2, 0), (N.TM_OP_ADD, b"L0/L1/L2", 5, 0)]
    extra = [(N.TM_OP_ADD, deep, 3, N.TM_KEY_WORDS), (N.TM_OP_ADD, b"/".join([b"+"] * 35), 4, 0)]
    topics = [deep, b"L0/x/L2", b"/".join(b"L%d" % i for i in range(35)), b"L0/L1/L2/q", b"L0/L1/L2"]
    for ops in (base, base + extra):
        eng = _engine()
        eng.apply(ops)
        eng.commit()
        assert (eng.stats()["n_deep_keys"] > 0) == (ops is not base)
        exp, (buf, off) = _oracle_first(ops, topics)
        _assert_same(_engine_sets(eng, buf, off, N.TM_MATCH_FIRST), exp, f"deep {len(ops)} keys")
        eng.close()


def test_first_edge_cases_vs_oracle(mode):
    shallow = [f for f in EDGE_FILTERS if len(f.split(b"/")) <= 30]
    for filters in (shallow, EDGE_FILTERS):
        ops = [(N.TM_OP_ADD, f, i, 0) for i, f in enumerate(filters)]
        eng = _engine(mode)
        eng.apply(ops)
        eng.commit()
        exp, (buf, off) = _oracle_first(ops, EDGE_TOPICS)
        _assert_same(_engine_sets(eng, buf, off, N.TM_MATCH_FIRST), exp, "first edge")
        eng.close()


# ------------------------------------------------------------- edge cases
EDGE_FILTERS = [b"#", b"+", b"+/+", b"/#", b"/+", b"//", b"", b"a", b"a/#", b"a/+", b"a//b", b"a/+/+", b"+/#",
                b"$SYS/#", b"$SYS/+", b"$SYS/brokers/+/clients/#", b"+/brokers/#", b"a/#/b", b"a/b#", b"a/b+",
                b"sport/", b"sport/+", b"$share", b"$queue/x", b"\xc3\xa9t\xc3\xa9/+", b"x" * 300 + b"/#",
                b"/".join([b"+"] * 26) + b"/#", b"/".join([b"+"] * 40), b"/".join(b"L%d" % i for i in range(30)),
                b"abcdefgh/+", b"abcdefghi/#", b"abcdefgh", b"abcdefghi", b"abcdefghij/x", b"\x00a/+", b"a\x00"]
EDGE_TOPICS = [b"", b"/", b"//", b"a", b"a/", b"a/b", b"a//b", b"a/b/c", b"$SYS", b"$SYS/brokers/n1/clients/c",
               b"$", b"$x/y", b"sport/", b"sport", b"a/b#", b"a/b+", b"\xc3\xa9t\xc3\xa9/x", b"x" * 300 + b"/y",
               b"/".join(b"L%d" % i for i in range(30)), b"/".join([b"q"] * 40), b"/".join([b"q"] * 26),
               b"/" * 200, b"+", b"#", b"a/+/b", b"a/b/#", b"b" * 65535, b"/".join([b"z"] * 3000),
               b"abcdefgh", b"abcdefgh/1", b"abcdefghi", b"abcdefghi/2", b"abcdefghij/x", b"abcdefghiJ/x",
               b"\x00a/q", b"a\x00", b"a", b"abcdefg"]


def test_edge_cases_vs_python_semantics(mode):
    eng = _engine(mode)
    eng.apply([(N.TM_OP_ADD, f, i) for i, f in enumerate(EDGE_FILTERS)])
    eng.commit()
    res = eng.match(EDGE_TOPICS)
    for t, r in zip(EDGE_TOPICS, res):
        levels = t.split(b"/")
        if b"+" in levels or b"#" in levels:
            assert r is None, t  # badarg
            continue
        exp = sorted(i for i, f in enumerate(EDGE_FILTERS) if et.match(t, f))
        got = sorted(eng.key_ids(np.array(r, dtype=np.uint32)).tolist())
        assert got == exp, (t[:60], got, exp)


def test_empty_index_and_empty_batch():
    eng = _engine()
    assert eng.match([]) == []
    assert eng.match([b"a/b", b"", b"$SYS/x"]) == [[], [], []]
    eng.commit()  # empty epoch
    assert eng.match([b"a"]) == [[]]


def test_output_arena_overflow_rerun():
    w = workloads.generate("C", scale=0.005, n_topics=3000)
    eng = _engine(reserve_matches=16)
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), ix.match(w.t_bytes, w.t_off), "overflow")


def _pool_workload(n_topics=2048, levels=10):
    """Half the topics match one '#' key at each of their prefixes and at every copy of
    a prefix with one level replaced by '+': dozens of key segments and a frontier
    about as wide as the depth per topic, so waves overflow their LDS segment and
    frontier buffers into the global chunk pools."""
    rng = np.random.default_rng(7)
    topics = [b"/".join(b"w%d" % rng.integers(0, 50) for _ in range(levels)) for _ in range(n_topics)]
    filters = set()
    for t in topics[: n_topics // 2]:
        ws = t.split(b"/")
        for d in range(1, levels):
            filters.add(b"/".join(ws[:d]) + b"/#")
            for j in range(d):  # '+' at every single position: frontier ~ depth wide
                pw = list(ws[:d])
                pw[j] = b"+"
                filters.add(b"/".join(pw) + b"/#")
    filters = sorted(filters)
    return filters, topics


def test_segment_and_frontier_chunks_and_pool_exhaustion():
    filters, topics = _pool_workload()
    ix = oracle.OrderedIndex.from_filters(filters)
    buf, off = N.pack_topics(topics)
    exp = ix.match(buf, off, threads=8)
    for chunks in (0, 1):
        eng = _engine(seg_chunks=chunks, topics_per_wave=64)  # wide waves: frontiers overflow LDS
        eng.apply([(N.TM_OP_ADD, f, i) for i, f in enumerate(filters)])
        eng.commit()
        eng.debug_stats(True, read=False)
        res = _engine_sets(eng, buf, off)
        st = dict(zip(N.Engine.STAT_NAMES, eng.debug_stats(False)))
        _assert_same(res, exp, f"seg_chunks={chunks}")
        assert st["chunk_flushes"] > 0 and st["frontier_chunks"] > 0, st
        if chunks == 1:
            assert st["spilled_topics"] > 0, st
        else:
            assert st["spilled_topics"] == 0, st
        eng.close()


# ------------------------------------------------------------- delta epochs (config E)
def test_churn_epochs_vs_oracle():
    rng = np.random.default_rng(0xE11A0005)
    w = workloads.generate("E", scale=0.02, n_topics=5000)
    filters = w.filters()
    ids = w.f_id.tolist()
    eng = _engine()
    live = set(range(len(ids)))
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    next_id = max(ids) + 1
    extra = {}
    for epoch in range(4):
        dels = rng.choice(sorted(live), size=max(1, len(live) // 100), replace=False)
        ops = [(N.TM_OP_DEL, filters[k] if k < len(filters) else extra[k][0], ids[k] if k < len(ids) else extra[k][1])
               for k in dels]
        for k in dels:
            live.discard(int(k))
        adds = []
        for _ in range(max(1, len(live) // 100)):
            src = int(rng.integers(len(filters)))
            f = filters[src] if rng.random() < 0.5 else b"$share-like/" + filters[src]
            extra[next_id] = (f, next_id)
            adds.append((N.TM_OP_ADD, f, next_id))
            live.add(next_id)
            next_id += 1
        # re-adding and re-deleting inside one epoch: last op wins
        ops += adds + [(N.TM_OP_DEL, adds[0][1], adds[0][2]), (N.TM_OP_ADD, adds[0][1], adds[0][2])]
        eng.apply(ops)
        eng.commit()
        lf = [filters[k] if k < len(filters) else extra[k][0] for k in sorted(live)]
        li = [ids[k] if k < len(ids) else extra[k][1] for k in sorted(live)]
        ix = oracle.OrderedIndex.from_filters(lf, li)
        _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), ix.match(w.t_bytes, w.t_off), f"epoch {epoch}")
    s = eng.stats()
    assert s["n_delta_commits"] >= 4 and s["n_keys"] == len(live)


def test_large_epochs_resolve_prefixes_in_parallel():
    """Epochs of >= 4096 ops on a populated trie take the parallel prefix resolution
    (engine.cpp apply_staged): paths resolved against the trie as it stood, then applied in
    order.  Covers ops whose path appears only during the epoch (add, then delete or re-add
    of the same key), deletes of keys that never existed, filters with '#' before the end
    (kept on the host), word-list keys, and filters deeper than the device order code
    (n_deep_keys), each epoch bit-exact vs the oracle."""
    rng = np.random.default_rng(0xE11A0006)
    w = workloads.generate("E", scale=0.05, n_topics=6000)
    filters = w.filters()
    base = [(f, int(i), 0) for f, i in zip(filters, w.f_id.tolist())]
    eng = _engine()
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    live = set(base)
    next_id = int(w.f_id.max()) + 1
    deep = b"/".join([b"d"] * 34)
    for epoch in range(3):
        ops, dead = [], []
        order = sorted(live)
        for j in rng.choice(len(order), size=2500, replace=False):
            k = order[int(j)]
            ops.append((N.TM_OP_DEL, k[0], k[1], N.TM_KEY_WORDS if k[2] else 0))
            live.discard(k)
        for _ in range(2500):
            src = filters[int(rng.integers(len(filters)))]
            r = rng.random()
            if r < 0.3:
                f = src + b"/new%d" % int(rng.integers(50))      # a new level under an old path
            elif r < 0.4:
                f = b"fresh%d/" % int(rng.integers(30)) + src     # a new path from the root
            elif r < 0.45:
                f = deep + (b"/+" if rng.random() < 0.5 else b"/#")  # deeper than the order code
            elif r < 0.5:
                f = src + b"/#"
            else:
                f = src
            wf = 1 if (r > 0.9 and b"+" not in f and b"#" not in f) else 0
            k = (f, next_id, wf)
            next_id += 1
            ops.append((N.TM_OP_ADD, f, k[1], N.TM_KEY_WORDS if wf else 0))
            live.add(k)
        # same-epoch sequences: add then delete, delete then re-add, deletes of nothing
        for t in range(200):
            f = b"tmp%d/x/%d" % (epoch, t)
            ops += [(N.TM_OP_ADD, f, 7), (N.TM_OP_DEL, f, 7)]
            g = order[t]
            if g in live:
                ops += [(N.TM_OP_DEL, g[0], g[1], N.TM_KEY_WORDS if g[2] else 0),
                        (N.TM_OP_ADD, g[0], g[1], N.TM_KEY_WORDS if g[2] else 0)]
            ops.append((N.TM_OP_DEL, b"never/there/%d" % t, 1))
        for t in range(20):  # '#' before the last level: stored, never matched
            dead.append((b"z%d/#/y" % t, 5))
            ops.append((N.TM_OP_ADD, b"z%d/#/y" % t, 5))
        eng.apply(ops)
        eng.commit()
        keys = sorted(live)
        ix = oracle.OrderedIndex.from_filters([k[0] for k in keys], ids=[k[1] for k in keys],
                                              word_form=[k[2] for k in keys])
        _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), ix.match(w.t_bytes, w.t_off), f"epoch {epoch}")
        deep_live = sum(1 for k in keys if k[0].startswith(deep))
        st_ = eng.stats()
        assert st_["n_deep_keys"] == deep_live, (st_["n_deep_keys"], deep_live)
        assert st_["n_keys"] == len(live) + 20
        eng.apply([(N.TM_OP_DEL, f, i) for f, i in dead])  # the dead keys go again
        eng.commit()


# ------------------------------------------------------------- property
_lvl = st.sampled_from([b"a", b"b", b"c", b"", b"foo", b"$x", b"0F"])
_topic = st.lists(_lvl, min_size=1, max_size=7).map(lambda l: b"/".join(l))
_flvl = st.sampled_from([b"a", b"b", b"", b"+", b"+", b"#", b"$x", b"foo"])
_filter = st.lists(_flvl, min_size=1, max_size=7).map(lambda l: b"/".join(l))


@settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck))
@given(filters=st.lists(_filter, min_size=1, max_size=40), topics=st.lists(_topic, min_size=1, max_size=40),
       slow=st.booleans())
def test_property_engine_vs_match2(filters, topics, slow):
    eng = _engine(slow)
    eng.apply([(N.TM_OP_ADD, f, i) for i, f in enumerate(filters)])
    eng.commit()
    for t, r in zip(topics, eng.match(topics)):
        exp = sorted({i for i, f in enumerate(filters) if et.match(t, f)})
        assert sorted(eng.key_ids(np.array(r, dtype=np.uint32)).tolist()) == exp, (t, filters)
    eng.close()


def test_counter_blocks_across_empty_batches_and_modes():
    """A launch's counters (output cursor, spill count, pool cursors) are zeroed by the
    launch before it (two alternating blocks, no memsets): every sequence of empty
    batches, FIRST / COUNT / ALL launches and spill-forcing launches must still start each
    batch from zero — checked through the device total and the host results."""
    import torch
    w = workloads.generate("C", scale=0.005, n_topics=4000)
    eng = _engine()
    _load(eng, w)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    exp = ix.match(w.t_bytes, w.t_off)
    want_total = int(exp[0][-1])
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    tb = int(w.t_off[-1])

    def dev_total(mode):
        r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), w.n_topics, tb, mode)
        eng.device_sync()
        t = torch.empty(1, dtype=torch.int64, device=dev)
        import ctypes as C
        lib = C.CDLL("libamdhip64.so")
        lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        assert lib.hipMemcpy(C.c_void_p(t.data_ptr()), C.c_void_p(r.d_total), 8, 3) == 0
        return int(t.cpu().item())

    seq = [N.TM_MATCH_ALL, None, N.TM_MATCH_ALL, N.TM_MATCH_FIRST, N.TM_MATCH_ALL, N.TM_MATCH_COUNT, None, None,
           N.TM_MATCH_ALL, N.TM_MATCH_UNIQUE, N.TM_MATCH_ALL, N.TM_MATCH_FIRST, N.TM_MATCH_FIRST, N.TM_MATCH_ALL]
    for k, mode in enumerate(seq):
        if mode is None:  # an empty batch launches no kernel
            r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), 0, 0, N.TM_MATCH_ALL)
            eng.device_sync()
            continue
        tot = dev_total(mode)
        if mode == N.TM_MATCH_FIRST:
            assert tot == 0, (k, tot)  # k_match_first writes keys[t] directly, never the cursor
        else:
            assert tot == want_total, (k, mode, tot, want_total)
    # the host path interleaved with the device path, then full parity
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, "after device sequence")
    assert eng.match([]) == []
    _assert_same(_engine_sets(eng, w.t_bytes, w.t_off), exp, "after empty host batch")
    # spilled topics count from zero in every batch too
    slow = _engine(force_slow=True)
    _load(slow, w)
    for _ in range(3):
        _assert_same(_engine_sets(slow, w.t_bytes, w.t_off), exp, "forced spill, repeated")
        assert slow.stats()["n_slow_topics"] == w.n_topics
