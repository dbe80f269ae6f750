"""GPU parity of the runs form (tm_match_batch_runs): per topic, the route ids that the spans
of the host id arena cover must be exactly the oracle's sorted id multiset, on the fast
path and the spill path, across delta epochs and full rebuilds, and with a span output too
small for the first try (the engine re-runs it).  Integer work, bit-exact."""
import ctypes as C

import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads

pytestmark = pytest.mark.gpu


def _check(eng, t_bytes, t_off, ix, what=""):
    o, ids, kcnt, st = eng.match_runs(t_bytes, t_off)
    eo, eids, est = ix.match(t_bytes, t_off)
    assert np.array_equal(st, est), what
    assert np.array_equal(np.diff(o).astype(np.int64), np.diff(eo).astype(np.int64)), what
    bad = [i for i in range(len(kcnt)) if not np.array_equal(np.sort(ids[o[i]:o[i + 1]]), eids[eo[i]:eo[i + 1]])]
    assert not bad, f"{what}: topics {bad[:6]} differ"
    return int(kcnt.sum())


@pytest.mark.parametrize("force_slow", [False, True], ids=["fast", "spill"])
@pytest.mark.parametrize("cfg,scale,nt", [("A", 1.0, 20000), ("B", 0.02, 20000), ("C", 0.01, 8000),
                                          ("E", 0.02, 20000)])
def test_runs_configs_vs_oracle(cfg, scale, nt, force_slow):
    w = workloads.generate(cfg, scale=scale, n_topics=nt)
    eng = N.Engine(0, force_slow=force_slow)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    total = _check(eng, w.t_bytes, w.t_off, ix, cfg)
    assert total > 0
    eng.close()


def test_runs_match_the_key_form_and_pipeline_subbatches():
    """A batch past one sub-batch (131,072 topics) runs as several on two streams; the
    spans equal tm_match_batch's keys mapped through tm_key_ids, topic by topic."""
    w = workloads.generate("B", scale=0.05, n_topics=300000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    o, ids, kcnt, st = eng.match_runs(w.t_bytes, w.t_off)
    koff, kc, keys, kst = eng.match_packed(w.t_bytes, w.t_off)
    kid = eng.key_ids(keys)
    assert np.array_equal(st, kst) and np.array_equal(kcnt, kc)
    for i in range(0, len(kc), 97):
        assert np.array_equal(np.sort(ids[o[i]:o[i + 1]]), np.sort(kid[koff[i]:koff[i] + kc[i]])), i
    eng.close()


def test_runs_span_output_grows_and_reruns():
    """The span output is sized from the previous batch; a batch with many more spans per
    topic than the last one overflows it, and the engine grows it and runs again."""
    small = workloads.generate("A", scale=1.0, n_topics=2000)
    w = workloads.generate("C", scale=0.01, n_topics=6000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    _check(eng, small.t_bytes, small.t_off, ix, "few spans")  # sizes the next batch small
    _check(eng, w.t_bytes, w.t_off, ix, "many spans")
    eng.close()


def test_runs_across_delta_epochs_and_full_rebuilds():
    rng = np.random.default_rng(0xE11A0055)
    w = workloads.generate("E", scale=0.02, n_topics=6000)
    filters = w.filters()
    live = {(f, int(i)) for f, i in zip(filters, w.f_id.tolist())}
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    next_id = int(w.f_id.max()) + 1
    for epoch in range(5):
        order = sorted(live)
        # epoch 3 churns a quarter of the keys: past n_live/8 deltas, a full rebuild
        k = len(order) // 4 if epoch == 3 else max(1, len(order) // 100)
        ops = []
        for j in rng.choice(len(order), size=k, replace=False):
            f, i = order[int(j)]
            ops.append((N.TM_OP_DEL, f, i))
            live.discard((f, i))
        for _ in range(k):
            f = filters[int(rng.integers(len(filters)))]
            if rng.random() < 0.3:
                f = f + b"/#"
            ops.append((N.TM_OP_ADD, f, next_id))
            live.add((f, next_id))
            next_id += 1
        eng.apply(ops)
        eng.commit()
        lf, li = zip(*sorted(live))
        ix = oracle.OrderedIndex.from_filters(list(lf), list(li))
        _check(eng, w.t_bytes, w.t_off, ix, f"epoch {epoch}")
    s = eng.stats()
    assert s["n_full_rebuilds"] >= 2 and s["n_delta_commits"] >= 4
    eng.close()


def test_runs_empty_batch_and_badarg():
    eng = N.Engine(0)
    eng.apply([(N.TM_OP_ADD, b"a/#", 7), (N.TM_OP_ADD, b"#", 8), (N.TM_OP_ADD, b"a/+/c", 9)])
    eng.commit()
    buf, off = N.pack_topics([])
    o, ids, kcnt, st = eng.match_runs(buf, off)
    assert len(ids) == 0 and len(kcnt) == 0
    buf, off = N.pack_topics([b"a/b/c", b"a/+/c", b"$SYS/x", b"", b"a"])
    o, ids, kcnt, st = eng.match_runs(buf, off)
    assert st.tolist() == [0, 1, 0, 0, 0]
    got = [sorted(ids[o[i]:o[i + 1]].tolist()) for i in range(5)]
    assert got == [[7, 8, 9], [], [], [8], [7, 8]]
    eng.close()


def test_runs_view_is_zero_copy_into_the_id_arena():
    """The spans of a hot '#' list point into one arena run: one span carries all its ids."""
    eng = N.Engine(0)
    eng.apply([(N.TM_OP_ADD, b"hot/#", i) for i in range(5000)])
    eng.commit()
    buf, off = N.pack_topics([b"hot/x/y"])
    res = eng.match_runs_view(buf, off)
    assert res.total_ids == 5000 and res.total_spans == 1 and res.span_cnt[0] == 1
    sp = res.spans[res.span_off[0]]
    got = np.ctypeslib.as_array(C.cast(sp.ids, C.POINTER(C.c_uint64)), shape=(int(sp.n),))
    assert sorted(got.tolist()) == list(range(5000))
    eng.lib.tm_runs_release(eng.h)
    eng.close()
