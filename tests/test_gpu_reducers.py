"""GPU parity of the per-topic reducers (result_kernels.hip k_dedupe) through the C-ABI:

  * TM_MATCH_UNIQUE — matches/3 with [unique]: per id the key the ordered walk writes
    LAST survives (match_add/2, apps/emqx/src/emqx_trie_search.erl:349-351).  The check is
    on the winning KEY, not only the id: the oracle's walk (oracle/trie_search.cpp, with
    the matched keys in ETS term order) names the winner.
  * TM_MATCH_AGGRE — emqx_broker:aggre/1 (apps/emqx/src/emqx_broker.erl:361-377): shared
    dests collapse per {Filter, Group}; plain node dests stay.

Integer work: exact equality, no tolerance."""
import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads

pytestmark = pytest.mark.gpu


def _canon_keys(filters, ids, word_form):
    """Deduplicate (filter, id, form) keys; the word form only makes a different key for
    a filter without wildcards (emqx_trie_search.erl:115-128)."""
    seen, out = set(), []
    for f, i, wf in zip(filters, ids, word_form):
        wild = any(l in (b"+", b"#") for l in f.split(b"/"))
        k = (f, int(i), 0 if wild else int(wf))
        if k not in seen:
            seen.add(k)
            out.append(k)
    return out


def _load(keys, **kw):
    eng = N.Engine(0, **kw)
    by_flag = {}
    for f, i, wf in keys:
        by_flag.setdefault(wf, []).append((f, i))
    for wf, ks in by_flag.items():
        eng.apply([(N.TM_OP_ADD, f, i, N.TM_KEY_WORDS if wf else 0) for f, i in ks])
    eng.commit()
    ix = oracle.OrderedIndex.from_filters([k[0] for k in keys], ids=[k[1] for k in keys],
                                          word_form=[k[2] for k in keys])
    return eng, ix


def _engine_key_index(eng, keys):
    """key handle -> index into `keys` (by filter bytes, id and form)."""
    at = {k: j for j, k in enumerate(keys)}

    def look(h):
        i, fb, fl = eng.key_info(int(h))
        wild = any(l in (b"+", b"#") for l in fb.split(b"/"))
        return at[(fb, i, 0 if wild else (1 if fl & N.TM_KEY_WORDS else 0))]
    return look


def _walks(ix, t_bytes, t_off):
    """Per topic, the matched key indices in the oracle's walk (ascending term) order."""
    off, _, st, src = ix.match(t_bytes, t_off, with_src=True, threads=8)
    return [src[off[t]:off[t + 1]] for t in range(len(off) - 1)], st


def _unique_reference(walk, ids):
    last = {}
    for j in walk:  # ascending walk order: Acc#{ID => K}, the last write wins
        last[ids[j]] = j
    return sorted(last.values())


def _unique_case(keys, t_bytes, t_off):
    eng, ix = _load(keys)
    walks, st = _walks(ix, t_bytes, t_off)
    ids = [k[1] for k in keys]
    look = _engine_key_index(eng, keys)
    off, cnt, hk, est = eng.match_packed(t_bytes, t_off, N.TM_MATCH_UNIQUE)
    assert np.array_equal(est, st)
    bad = []
    for t in range(len(cnt)):
        got = sorted(look(h) for h in hk[off[t]:off[t] + cnt[t]])
        if got != _unique_reference(walks[t], ids):
            bad.append(t)
    assert not bad, f"UNIQUE winners differ at topics {bad[:8]}"
    return eng


def _with_repeated_ids(w, n_ids, seed, word_frac=0.3):
    rng = np.random.default_rng(seed)
    fs = w.filters()
    ids = rng.integers(0, n_ids, len(fs))
    wf = (rng.random(len(fs)) < word_frac).astype(int)
    keys = _canon_keys(fs, ids, wf)
    # every exact filter also in the other form under the same id: binary and word-list keys
    # of one filter compete for the id (lists sort before binaries)
    extra = [(f, i, 1 - x) for f, i, x in keys[: len(keys) // 4]
             if not any(l in (b"+", b"#") for l in f.split(b"/"))]
    return _canon_keys([k[0] for k in keys + extra], [k[1] for k in keys + extra], [k[2] for k in keys + extra])


@pytest.mark.parametrize("name,scale,nt,n_ids", [("A", 1.0, 20_000, 50), ("E", 0.02, 20_000, 200),
                                                 ("C", 0.002, 10_000, 30)])
def test_unique_winner_keys_vs_oracle_walk(name, scale, nt, n_ids):
    w = workloads.generate(name, scale=scale, n_topics=nt)
    keys = _with_repeated_ids(w, n_ids, seed=7)
    eng = _unique_case(keys, w.t_bytes, w.t_off)
    assert eng.stats()["n_deep_keys"] == 0


def test_unique_term_order_kats():
    """Term order decides the winner per id (Erlang: '#' < '+' < binary words, a list
    that ends first sorts first, every {Binary, {ID}} key after every list)."""
    sets = [
        [(b"a/b", 1, 0), (b"a/b", 1, 1), (b"a/+", 1, 0), (b"+/b", 1, 0), (b"#", 1, 0), (b"a/#", 1, 0),
         (b"+/+", 1, 0)],                                 # the binary "a/b" wins
        [(b"a/b", 1, 1), (b"a/+", 1, 0), (b"+/b", 1, 0), (b"#", 1, 0), (b"a/#", 1, 0)],  # words [a, b]
        [(b"a/+", 1, 0), (b"+/b", 1, 0), (b"#", 1, 0), (b"a/#", 1, 0), (b"a/b/#", 1, 0)],  # [a, b, '#']
        [(b"+/+", 7, 0), (b"+/#", 7, 0), (b"#", 7, 0), (b"+/b", 8, 0), (b"+", 8, 0), (b"+/b/#", 8, 0)],
        [(b"+", 3, 0), (b"#", 3, 0), (b"/", 3, 0), (b"/", 3, 1), (b"+/+", 3, 0), (b"+/", 3, 1), (b"/+", 3, 0)],
    ]
    topics = [b"a/b", b"a", b"/", b"a/b/c", b"x/b", b"$SYS/b", b"a//"]
    t_bytes, t_off = N.pack_topics(topics)
    for keys in sets:
        _unique_case(_canon_keys(*zip(*[(k[0], k[1], k[2]) for k in keys])), t_bytes, t_off)


def test_unique_many_keys_per_topic_multi_pass():
    """A topic with thousands of keys takes several LDS passes (DD_PASS keys each)."""
    keys = []
    rng = np.random.default_rng(3)
    for j in range(5000):  # 5000 keys on the same few filters, 2500 distinct ids
        f = [b"hot/#", b"hot/+", b"+/x", b"#", b"hot/x"][j % 5]
        keys.append((f, int(rng.integers(0, 2500)), int(j % 3 == 0)))
    keys = _canon_keys(*zip(*keys))
    t_bytes, t_off = N.pack_topics([b"hot/x", b"hot/y", b"z/x", b"hot", b"$SYS/x"])
    _unique_case(keys, t_bytes, t_off)


def test_unique_id_all_ones_and_zero():
    keys = _canon_keys([b"a/+", b"a/#", b"#", b"a/b", b"+/b"], [2**64 - 1, 2**64 - 1, 0, 0, 2**64 - 1],
                       [0, 0, 0, 1, 0])
    t_bytes, t_off = N.pack_topics([b"a/b", b"a/c", b"q"])
    _unique_case(keys, t_bytes, t_off)


def test_unique_churn_id_multiplicity():
    """Only keys whose id another live key shares enter k_dedupe's table (KR_MULTI).  Ids
    go 1 -> 2 -> 1 -> 2 keys over epochs, the first key of an id is flagged when a second
    arrives, and a flagged key keeps its flag after the other one leaves; every epoch's
    UNIQUE winners equal the oracle walk's over the live keys."""
    rng = np.random.default_rng(11)
    pool = [b"a/#", b"a/+", b"+/b", b"#", b"a/b", b"+/+", b"a/b/#", b"+/#", b"x/#", b"a/+/#"]
    topics = [b"a/b", b"a", b"a/c", b"x/b", b"a/b/c", b"q/b"]
    t_bytes, t_off = N.pack_topics(topics)
    eng = N.Engine(0)
    live = set()
    for epoch in range(12):
        ops = []
        for _ in range(6):
            k = (pool[int(rng.integers(0, len(pool)))], int(rng.integers(0, 4)), 0)
            if k in live:
                live.discard(k)
                ops.append((N.TM_OP_DEL, k[0], k[1]))
            else:
                live.add(k)
                ops.append((N.TM_OP_ADD, k[0], k[1]))
        eng.apply(ops)
        eng.commit()
        keys = sorted(live)
        if not keys:
            continue
        ix = oracle.OrderedIndex.from_filters([k[0] for k in keys], ids=[k[1] for k in keys],
                                              word_form=[0] * len(keys))
        walks, st = _walks(ix, t_bytes, t_off)
        look = _engine_key_index(eng, keys)
        off, cnt, hk, est = eng.match_packed(t_bytes, t_off, N.TM_MATCH_UNIQUE)
        assert np.array_equal(est, st)
        for t in range(len(topics)):
            got = sorted(look(h) for h in hk[off[t]:off[t] + cnt[t]])
            assert got == _unique_reference(walks[t], [k[1] for k in keys]), (epoch, topics[t])
    eng.close()


def test_unique_deep_filters_reduce_on_host():
    """Shapes deeper than the device order code (31 levels) are counted; tm_match_batch
    then reduces on the host and the device form refuses (TM_ESTATE)."""
    deep = b"/".join([b"l"] * 40)
    keys = _canon_keys([deep, deep[:-1] + b"+", b"l/#", deep + b"/#"], [1, 1, 1, 2], [0, 0, 0, 0])
    t_bytes, t_off = N.pack_topics([deep, deep + b"/m", b"l"])
    eng = _unique_case(keys, t_bytes, t_off)
    assert eng.stats()["n_deep_keys"] == 2  # the exact 40-level key is a binary key: not deep
    import torch
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(t_bytes).to(dev)
    d_off = torch.from_numpy(t_off.view(np.int32)).to(dev)
    with pytest.raises(RuntimeError):
        eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), 3, int(t_off[-1]), N.TM_MATCH_UNIQUE)
    eng.apply([(N.TM_OP_DEL, k[0], k[1]) for k in keys if len(k[0].split(b"/")) > 31])
    eng.commit()
    assert eng.stats()["n_deep_keys"] == 0


def _d2h_u32(ptr, n):
    import ctypes as C

    import torch
    t = torch.empty(max(n, 1), dtype=torch.int32, device="cuda:0")
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    if n:
        assert lib.hipMemcpy(C.c_void_p(t.data_ptr()), C.c_void_p(ptr), 4 * n, 3) == 0
    return t[:n].cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("mode", [N.TM_MATCH_UNIQUE, N.TM_MATCH_AGGRE])
def test_reducers_device_api_and_result_ids(mode):
    """tm_match_device_mode(UNIQUE | AGGRE) gives the same lists as tm_match_batch, and
    tm_result_ids_device compacts the reduced lists."""
    import torch
    w = workloads.generate("E", scale=0.02, n_topics=8000)
    keys = _with_repeated_ids(w, 100, seed=11)
    if mode == N.TM_MATCH_AGGRE:
        keys = [(f, N.shared_id(i % 3, i) if i % 2 else i, wf) for f, i, wf in keys]
    eng, _ = _load(keys)
    n = w.n_topics
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    r = eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), mode)
    eng.device_sync()
    d_cnt = _d2h_u32(r.d_cnt, n)
    d_offs = _d2h_u32(r.d_off, n)
    span = int((d_offs.astype(np.uint64) + d_cnt).max())
    d_keys = _d2h_u32(r.d_keys, span)
    d_ids_t = torch.empty(int(d_cnt.sum()) + 1, dtype=torch.int64, device=dev)
    d_ioff_t = torch.empty(n + 1, dtype=torch.int32, device=dev)
    eng.result_ids_device(d_ids_t.data_ptr(), d_ids_t.numel(), d_ioff_t.data_ptr())
    torch.cuda.synchronize()
    ioff = d_ioff_t.cpu().numpy().view(np.uint32)
    rids = d_ids_t.cpu().numpy().view(np.uint64)
    off, cnt, hk, _ = eng.match_packed(w.t_bytes, w.t_off, mode)
    assert np.array_equal(cnt, d_cnt)
    assert int(ioff[n]) == int(cnt.sum())
    for t in range(n):
        a = np.sort(d_keys[d_offs[t]:d_offs[t] + d_cnt[t]])
        b = np.sort(hk[off[t]:off[t] + cnt[t]])
        assert np.array_equal(a, b), t
        assert np.array_equal(np.sort(rids[ioff[t]:ioff[t + 1]]), np.sort(eng.key_ids(b))), t


def _aggre_reference(walk, keys):
    """emqx_broker:aggre/1 over the matched routes: {Filter, Node} for node dests,
    usort({Filter, Group}) once a shared dest is present."""
    plain, shared = [], set()
    for j in walk:
        f, i, _ = keys[j]
        if i >> 63:
            shared.add((f, (i >> 32) & 0x7FFFFFFF))
        else:
            plain.append((f, i))
    return sorted(plain), shared


@pytest.mark.parametrize("name,scale,nt", [("A", 1.0, 20_000), ("E", 0.02, 20_000)])
def test_aggre_vs_oracle_walk(name, scale, nt):
    w = workloads.generate(name, scale=scale, n_topics=nt)
    rng = np.random.default_rng(5)
    fs = w.filters()[: 4000]
    keys = []
    for f in fs:  # each filter to 1..6 dests: node dests and members of 3 shared groups
        for _ in range(int(rng.integers(1, 7))):
            if rng.random() < 0.6:
                keys.append((f, N.shared_id(int(rng.integers(0, 3)), int(rng.integers(0, 4))), 0))
            else:
                keys.append((f, int(rng.integers(0, 5)), 0))
    keys = _canon_keys(*zip(*keys))
    eng, ix = _load(keys)
    walks, st = _walks(ix, w.t_bytes, w.t_off)
    look = _engine_key_index(eng, keys)
    off, cnt, hk, est = eng.match_packed(w.t_bytes, w.t_off, N.TM_MATCH_AGGRE)
    assert np.array_equal(est, st)
    n_collapsed = 0
    for t in range(len(cnt)):
        plain, shared = _aggre_reference(walks[t], keys)
        got_plain, got_shared = [], []
        for h in hk[off[t]:off[t] + cnt[t]]:
            f, i, _ = keys[look(h)]
            if i >> 63:
                got_shared.append((f, (i >> 32) & 0x7FFFFFFF))
            else:
                got_plain.append((f, i))
        assert sorted(got_plain) == plain, t
        assert len(got_shared) == len(set(got_shared)) and set(got_shared) == shared, t
        n_collapsed += len(walks[t]) - int(cnt[t])
    assert n_collapsed > 0


def test_router_match_aggre_batch_vs_host_aggre():
    """Router.match_aggre_batch (device {Filter, Group} collapse) equals the host
    restatement of aggre/1 over match_routes/1."""
    from emqx_amd.router import Router, aggre
    r = Router(0, node="n0")
    rng = np.random.default_rng(9)
    filters = [b"s/+/t", b"s/#", b"#", b"s/1/t", b"+/1/+", b"$share-like/x", b"s/+/+"]
    for f in filters:
        for _ in range(int(rng.integers(1, 6))):
            if rng.random() < 0.5:
                r.add_route(f, (f"g{int(rng.integers(0, 3))}", f"n{int(rng.integers(0, 4))}"))
            else:
                r.add_route(f, f"n{int(rng.integers(0, 4))}")
    topics = [b"s/1/t", b"s/2/t", b"s", b"x/1/y", b"$SYS/1/t"]
    got = r.match_aggre_batch(topics)
    for t, g in zip(topics, got):
        assert sorted(g, key=repr) == sorted(aggre(r.match_routes(t)), key=repr), t
