"""The publish batching aggregator (include/emqx_tm_batcher.h, emqx_amd/csrc/batcher.cpp).

It stands between many concurrent publishers — each of which runs
emqx_router:match_routes/1 synchronously per publish in the reference
(apps/emqx/src/emqx_broker.erl:285-290, apps/emqx/src/emqx_router.erl:205-212) — and one
engine batch per window.

CPU tests drive the real native batcher over a Python batch matcher (tm_batcher_create_fn)
whose answers come from the oracle's emqx_topic:match/2: windowing, draining, per-publish
hand-back, badarg and failed batches.  The GPU tests run it over a real engine and check
every publish's ids bit-exactly against the oracle."""
import ctypes as C
import threading
import time

import numpy as np
import pytest

import oracle.emqx_topic as T
from emqx_amd import _native as N

ROUTES = [(b"a/+", 1), (b"a/#", 2), (b"#", 3), (b"+/b", 4), (b"a/b", 5), (b"$SYS/#", 6), (b"x/y/z", 7),
          (b"+/+", 8), (b"a/b", 9)]


def _oracle_backend(routes, calls=None):
    def backend(topics, mode):
        if calls is not None:
            calls.append(len(topics))
        lists, status = [], []
        for t in topics:
            if any(l in (b"+", b"#") for l in t.split(b"/")):
                lists.append([])
                status.append(N.TM_BADARG)
                continue
            ids = sorted(i for f, i in routes if T.match(t, f))
            lists.append(ids)
            status.append(N.TM_TOPIC_OK)
        return lists, status
    return backend


def _expect(topic, routes=ROUTES):
    return sorted(i for f, i in routes if T.match(topic, f))


def test_header_declares_batcher_surface():
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "emqx_tm_batcher.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decl = set(re.findall(r"\b(tm_batcher_[a-z_0-9]+)\s*\(", src))
    assert decl == set(N.BATCHER_EXPORTS)
    import subprocess
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH]).decode()
    exported = set(re.findall(r" T (tm_batcher_\w+)", out))
    assert decl <= exported


def test_blocking_match_one_publish():
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_wait_us=100)
    for t in (b"a/b", b"a", b"$SYS/x", b"q/r/s", b"x/y/z", b""):
        st, ids = b.match(t)
        assert st == N.TM_TOPIC_OK and sorted(ids) == _expect(t), t
    st, ids = b.match(b"a/+")
    assert st == N.TM_BADARG and ids == []
    assert b.stats()["publishes"] == 7
    b.close()


def test_window_trace_stamps_and_cpu_accounting():
    """tm_batcher_windows: per window the stage stamps in order, and the cutter's / delivery
    threads' CPU time and involuntary context switches (getrusage per thread), which tell a
    slow stage that worked from one whose thread was preempted."""
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_batch=8, max_wait_us=500, delivery_threads=2)
    b.reset_stats()
    th = [threading.Thread(target=lambda k=k: [b.match(b"a/b") for _ in range(20)]) for k in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    w = b.windows()
    b.close()
    assert len(w) >= 20 and int(w["n"].sum()) == 160
    assert np.all(w["t_oldest"] <= w["t_cut"]) and np.all(w["t_slot"] <= w["t_cut"])
    assert np.all(w["t_cut"] <= w["t_queued"]) and np.all(w["t_queued"] <= w["t_done"])
    # a thread's CPU time inside an interval never exceeds the interval (plus rusage's tick)
    cut_wall_us = (w["t_queued"] - w["t_cut"]) / 1e3
    assert np.all(w["cut_cpu_us"] <= cut_wall_us + 5000)
    assert np.all(w["del_cpu_us"] <= w["del_wall_us"] + 5000)
    assert np.all(w["del_wall_us"] > 0)


def test_concurrent_publishers_share_windows():
    calls = []
    b = N.Batcher(backend=_oracle_backend(ROUTES, calls), max_batch=16, max_wait_us=20000)
    rng = np.random.default_rng(5)
    words = [b"a", b"b", b"x", b"y", b"z", b"$SYS", b""]
    topics = [b"/".join(words[j] for j in rng.integers(0, len(words), rng.integers(1, 4))) for _ in range(400)]
    bad = []

    def worker(k):
        for t in topics[k::32]:
            st, ids = b.match(t)
            if st != N.TM_TOPIC_OK or sorted(ids) != _expect(t):
                bad.append(t)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(32)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    s = b.stats()
    b.close()
    assert not bad
    assert s["publishes"] == len(topics) == sum(calls)
    assert max(calls) <= 16 and s["max_batch_seen"] <= 16
    assert s["batches"] < len(topics)  # publishers really were batched together
    assert s["lat_p99_us"] >= s["lat_p50_us"] > 0


def test_window_closes_on_time():
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_batch=1 << 20, max_wait_us=2000)
    t0 = time.perf_counter()
    st, ids = b.match(b"a/b")
    dt = time.perf_counter() - t0
    b.close()
    assert st == N.TM_TOPIC_OK and sorted(ids) == _expect(b"a/b")
    assert 0.0015 <= dt < 2.0  # waited for the window, not for max_batch publishes


def test_destroy_drains_async_submissions():
    got = {}
    lock = threading.Lock()

    @N.tm_match_cb
    def cb(ctx, status, ids, n):
        with lock:
            got[ctx] = (status, sorted(ids[i] for i in range(n)))

    b = N.Batcher(backend=_oracle_backend(ROUTES), max_batch=64, max_wait_us=1_000_000)
    topics = [b"a/b", b"a/c", b"x/y/z", b"$SYS/q", b"b"] * 40
    for k, t in enumerate(topics):
        assert b.lib.tm_batcher_submit(b.h, t, len(t), cb, C.c_void_p(k + 1)) == N.TM_OK
    b.close()  # windows of 1 s: only the drain at destroy delivers them
    assert len(got) == len(topics)
    for k, t in enumerate(topics):
        assert got[k + 1] == (N.TM_TOPIC_OK, _expect(t)), t


def test_failed_batch_reaches_every_publisher():
    def broken(topics, mode):
        raise RuntimeError("device lost")
    b = N.Batcher(backend=broken, max_wait_us=100)
    st, ids = b.match(b"a/b")
    b.close()
    assert st == N.TM_EDEVICE and ids == []


def test_count_mode_and_write_calls_need_an_engine():
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_wait_us=100, mode=N.TM_MATCH_COUNT)
    assert b.match(b"a/b") == (N.TM_TOPIC_OK, len(_expect(b"a/b")))
    with pytest.raises(N.TMError):
        b.commit()
    with pytest.raises(N.TMError):
        b.apply([(N.TM_OP_ADD, b"a", 1)])
    b.close()
    lib = N.load()
    assert lib.tm_batcher_submit(None, b"a", 1, N.tm_match_cb(lambda *a: None), None) == N.TM_EINVAL
    bad = N.tm_batcher_config(0, 0, 99, 0)
    h = C.c_void_p()
    fn = N.tm_batch_fn(lambda *a: 0)
    assert lib.tm_batcher_create_fn(fn, None, C.byref(bad), C.byref(h)) == N.TM_EINVAL


# ------------------------------------------------------------------ GPU: over a real engine
@pytest.mark.gpu
@pytest.mark.parametrize("mode,transport", [(N.TM_MATCH_ALL, N.TM_TRANSPORT_AUTO), (N.TM_MATCH_ALL, N.TM_TRANSPORT_IDS),
                                            (N.TM_MATCH_COUNT, N.TM_TRANSPORT_AUTO),
                                            (N.TM_MATCH_FIRST, N.TM_TRANSPORT_AUTO)],
                         ids=["all-runs", "all-ids", "count", "first"])
def test_gpu_batcher_over_engine_vs_oracle(mode, transport):
    from emqx_amd import workloads
    import oracle
    w = workloads.generate("A", scale=0.3, n_topics=3000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eoff, eids, est = ix.match(w.t_bytes, w.t_off)
    topics = w.topics()
    b = N.Batcher(eng, max_batch=512, max_wait_us=500, mode=mode, transport=transport)
    bad = []

    def worker(k):
        for i in range(k, len(topics), 24):
            st, ids = b.match(topics[i])
            exp = eids[eoff[i]:eoff[i + 1]].tolist()
            if st != est[i]:
                bad.append(i)
            elif mode == N.TM_MATCH_ALL and sorted(ids) != exp:
                bad.append(i)
            elif mode == N.TM_MATCH_COUNT and ids != len(exp):
                bad.append(i)
            elif mode == N.TM_MATCH_FIRST and (len(ids) != (1 if exp else 0) or (ids and ids[0] not in exp)):
                bad.append(i)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(24)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    s = b.stats()
    b.close()
    eng.close()
    assert not bad, bad[:8]
    assert s["publishes"] == len(topics) and s["batches"] < len(topics)


@pytest.mark.gpu
def test_gpu_aggregators_one_after_another_on_one_engine():
    """Aggregators created and destroyed in turn over ONE engine (the bench's rows): each one's
    windows run on its own streams, and the engine must not keep those streams after it is
    gone (round 5: the next aggregator's first window was ordered after a destroyed stream).
    Every reply equals the oracle's; commits and direct matches between them still work."""
    from emqx_amd import workloads
    import oracle
    w = workloads.generate("A", scale=0.2, n_topics=2000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eoff, eids, est = ix.match(w.t_bytes, w.t_off)
    topics = w.topics()
    for rnd, transport in enumerate([N.TM_TRANSPORT_AUTO, N.TM_TRANSPORT_IDS, N.TM_TRANSPORT_AUTO] * 2):
        b = N.Batcher(eng, max_batch=256, max_wait_us=300, transport=transport)
        bad = []

        def worker(k):
            for i in range(k, len(topics), 16):
                st, ids = b.match(topics[i])
                if st != est[i] or sorted(ids) != eids[eoff[i]:eoff[i + 1]].tolist():
                    bad.append(i)
        th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        b.close()
        assert not bad, (rnd, bad[:5])
        # between aggregators: a commit (it waits for every stream that read the index) and
        # a host-form batch on the engine itself
        eng.apply([(N.TM_OP_ADD, b"zz/%d" % rnd, 10_000_000 + rnd)])
        eng.commit()
        k = eng.match([b"zz/%d" % rnd])[0]  # (the workload's wildcard filters match it too)
        assert 10_000_000 + rnd in eng.key_ids(np.asarray(k, dtype=np.uint32)).tolist()
    eng.close()


@pytest.mark.gpu
def test_gpu_batcher_epochs_swap_between_batches():
    """Writes through the batcher serialise with its worker: after commit returns, every
    later publish sees the new epoch."""
    eng = N.Engine(0)
    b = N.Batcher(eng, max_batch=64, max_wait_us=200)
    b.apply([(N.TM_OP_ADD, b"a/+", 1), (N.TM_OP_ADD, b"#", 2)])
    b.commit()
    assert sorted(b.match(b"a/b")[1]) == [1, 2]
    b.apply([(N.TM_OP_DEL, b"#", 2), (N.TM_OP_ADD, b"a/b", 3), (N.TM_OP_ADD, b"a/b", N.shared_id(0, 9))])
    b.commit()
    assert sorted(b.match(b"a/b")[1]) == sorted([1, 3, N.shared_id(0, 9)])
    assert b.match(b"$SYS/x") == (N.TM_TOPIC_OK, [])
    assert b.match(b"a/#")[0] == N.TM_BADARG
    b.close()
    eng.close()


def test_closed_loop_loadgen_over_python_backend():
    """tools/loadgen.cpp (bench tooling): publishers resubmit from their callbacks until the
    deadline, then the run drains; nothing fails and publishers share windows."""
    import os
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "libtm_loadgen.so"))
    lib.loadgen_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double,
                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                C.POINTER(C.c_double)]
    tb, to = N.pack_topics([b"a/b", b"x/y/z", b"a", b"$SYS/a"])
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_batch=256, max_wait_us=500)
    got, ids, errs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
    rc = lib.loadgen_run(b.h, tb.ctypes.data, to.ctypes.data, 4, 64, 0.3, C.byref(got), C.byref(ids), C.byref(errs),
                         C.byref(el))
    s = b.stats()
    b.close()
    assert rc == 0 and errs.value == 0 and got.value >= 64
    assert s["publishes"] == got.value and s["batches"] < got.value
    per = [len(_expect(t)) for t in (b"a/b", b"x/y/z", b"a", b"$SYS/a")]
    assert ids.value <= max(per) * got.value


def test_latency_window_covers_every_publish_and_obeys_littles_law():
    """tm_batcher_stats_reset / _get (ABI 9): the latency histogram covers every publish
    delivered in the window (not the last 65,536), and in a closed loop its mean equals
    publishers / throughput (Little's law) within the bench's 20 % check."""
    import os
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "libtm_loadgen.so"))
    U = C.POINTER(C.c_uint64)
    lib.loadgen_run3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                 C.c_int, U, U, U, U, C.POINTER(C.c_double), C.POINTER(N.tm_batcher_stats)]
    tb, to = N.pack_topics([b"a/b", b"x/y/z", b"a", b"$SYS/a"])
    calls = []

    def slow(topics, mode):  # a backend with a real service time: windows of ~2 ms
        time.sleep(0.002)
        return _oracle_backend(ROUTES, calls)(topics, mode)

    pubs = 128
    b = N.Batcher(backend=slow, max_batch=4096, max_wait_us=200)
    got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
    win = N.tm_batcher_stats()
    rc = lib.loadgen_run3(b.h, tb.ctypes.data, to.ctypes.data, 4, pubs, 0.3, 1.0, 0, C.byref(got), C.byref(ids),
                          C.byref(errs), C.byref(cs), C.byref(el), C.byref(win))
    whole = b.stats()
    b.close()
    assert rc == 0 and errs.value == 0
    assert 0.95 <= win.window_s <= 1.5
    # the window saw a share of the run's publishes, far more than a handful
    assert 0 < win.lat_count < got.value and win.lat_count > 10 * pubs
    rate = win.lat_count / win.window_s
    little_ms = pubs / rate * 1e3
    assert abs(win.lat_mean_us / 1e3 - little_ms) <= 0.2 * little_ms, (win.lat_mean_us, little_ms)
    # every window's service time (2 ms) is in every latency
    assert 2000 <= win.lat_p50_us <= win.lat_p99_us <= win.lat_p999_us <= win.lat_max_us * 1.02
    # after the drain, the whole window (no reset since) holds at least as many publishes
    assert whole["lat_count"] >= win.lat_count


def test_latency_histogram_without_reset_counts_all():
    b = N.Batcher(backend=_oracle_backend(ROUTES), max_wait_us=100)
    for t in (b"a/b", b"a", b"x/y/z") * 30:
        b.match(t)
    s = b.stats()
    assert s["lat_count"] == 90 and s["lat_mean_us"] > 0 and s["lat_p50_us"] <= s["lat_max_us"] * 1.02
    b.reset_stats()
    s2 = b.stats()
    assert s2["lat_count"] == 0 and s2["lat_p50_us"] == 0
    b.match(b"a/b")
    assert b.stats()["lat_count"] == 1
    b.close()


def test_batcher_pipeline_under_thread_sanitizer():
    """tests/native/batcher_tsan: the aggregator's threads (cutter, completion, delivery
    pool) and sharded submission under ThreadSanitizer, 8,192 closed-loop publishers over
    a custom backend (no device)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "batcher_tsan")
    if not os.path.exists(exe):
        pytest.fail("tests/native/batcher_tsan not built (run __graft_entry__.build())")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0")
    p = subprocess.run([exe, "8192", "16", "1", "4"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "ThreadSanitizer" not in p.stderr, p.stderr[-3000:]
    assert '"errors": 0' in p.stdout


@pytest.mark.gpu
def test_gpu_batcher_span_callbacks_vs_oracle():
    """tm_batcher_submit_spans: each publish gets spans of the engine's id arena (runs
    transport) whose concatenation is its oracle id set; on the ids transport, one span."""
    from emqx_amd import workloads
    import oracle
    w = workloads.generate("C", scale=0.003, n_topics=2000)
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    eoff, eids, est = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id).match(w.t_bytes, w.t_off)
    topics = w.topics()
    lib = N.load()
    for transport in (N.TM_TRANSPORT_RUNS, N.TM_TRANSPORT_IDS):
        b = N.Batcher(eng, max_batch=256, max_wait_us=300, transport=transport)
        got, done = {}, threading.Semaphore(0)

        def cb(ctx, status, spans, ns, nids):
            sp = C.cast(spans, C.POINTER(N.tm_span)) if ns else None
            ids = []
            for j in range(ns):
                ids += np.ctypeslib.as_array(C.cast(sp[j].ids, C.POINTER(C.c_uint64)), shape=(int(sp[j].n),)).tolist()
            got[ctx] = (status, sorted(ids), nids)
            done.release()

        fn = N.tm_spans_cb(cb)
        for i, t in enumerate(topics):
            assert lib.tm_batcher_submit_spans(b.h, t, len(t), fn, C.c_void_p(i + 1)) == 0
        for _ in topics:
            assert done.acquire(timeout=30)
        b.close()
        for i in range(len(topics)):
            st, ids, nids = got[i + 1]
            assert st == est[i] and ids == eids[eoff[i]:eoff[i + 1]].tolist() and nids == len(ids), (transport, i)
    eng.close()


@pytest.mark.gpu
def test_gpu_batcher_beside_direct_writers_and_device_callers():
    """The engine is shared: while 16 threads publish through the batcher (runs transport:
    windows hold read leases), another thread writes and commits the ENGINE directly, and
    another runs tm_match_device calls.  Every reply equals the oracle result of one committed
    epoch, and replies never go back to an older epoch for a publisher."""
    from emqx_amd import workloads
    import oracle
    import torch
    w = workloads.generate("A", scale=0.3, n_topics=1500)
    filters = w.filters()
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    rng = np.random.default_rng(77)
    live = {(f, int(i)) for f, i in zip(filters, w.f_id.tolist())}
    sets, opss, nid = [frozenset(live)], [], 10 ** 6
    for e in range(4):
        order = sorted(live)
        ops = []
        for j in rng.choice(len(order), size=40, replace=False):
            ops.append((N.TM_OP_DEL,) + order[int(j)])
            live.discard(order[int(j)])
        for _ in range(40):
            f = filters[int(rng.integers(len(filters)))] + (b"/#" if rng.random() < 0.5 else b"")
            ops.append((N.TM_OP_ADD, f, nid))
            live.add((f, nid))
            nid += 1
        opss.append(ops)
        sets.append(frozenset(live))
    exp = []
    for ks in sets:
        lf, li = zip(*sorted(ks))
        o, ids, st = oracle.OrderedIndex.from_filters(list(lf), list(li)).match(w.t_bytes, w.t_off)
        exp.append([ids[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)])
    topics = w.topics()
    b = N.Batcher(eng, max_batch=256, max_wait_us=300)
    stop, bad = threading.Event(), []

    def publisher(k):
        last = 0
        i = k
        while not stop.is_set():
            st, ids = b.match(topics[i % len(topics)])
            e = [x for x in range(last, len(exp)) if sorted(ids) == exp[x][i % len(topics)]]
            if not e:
                bad.append((k, i))
                return
            last = e[0]
            i += 16

    def device_caller():
        dev = torch.device("cuda:0")
        s = torch.cuda.Stream(device=dev)
        tb = torch.from_numpy(w.t_bytes).to(dev)
        to = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
        while not stop.is_set():
            with torch.cuda.stream(s):
                eng.match_device_mode(tb.data_ptr(), to.data_ptr(), len(topics), int(w.t_off[-1]), N.TM_MATCH_COUNT,
                                      s.cuda_stream)
            s.synchronize()

    th = [threading.Thread(target=publisher, args=(k,)) for k in range(16)] + [threading.Thread(target=device_caller)]
    for t in th:
        t.start()
    for ops in opss:
        time.sleep(0.05)
        eng.apply(ops)
        eng.commit()
    time.sleep(0.1)
    stop.set()
    for t in th:
        t.join(timeout=60)
    b.close()
    eng.close()
    assert not bad, bad[:5]


@pytest.mark.gpu
@pytest.mark.parametrize("idw", [8, 4], ids=["u64-arena", "u32-arena"])
@pytest.mark.parametrize("wide_ids", [False, True], ids=["u32-ids", "ids-past-32-bits"])
def test_gpu_batcher_span_kinds_vs_oracle(wide_ids, idw, monkeypatch):
    """Every reply kind vs the oracle: on windows of the engine's u32 id arena the u32-span
    callback (tm_batcher_submit_spans32) reads in place and the id-list and u64-span callbacks
    get the ids widened; on u64 windows the reverse.  Once an id needs 64 bits the windows fall
    back to the u64 arena: id lists and u64 spans stay exact, u32 spans get TM_ESTATE.  The
    default windows read the u64 arena (u32-span replies are narrowed); EMQX_TM_RUNS_IDW=4
    runs them on the u32 one."""
    import oracle
    from emqx_amd import workloads
    monkeypatch.setenv("EMQX_TM_RUNS_IDW", str(idw))
    w = workloads.generate("A", scale=0.3, n_topics=3000)
    ids = w.f_id.astype(np.uint64) + (np.uint64(1 << 40) if wide_ids else np.uint64(0))
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, ids)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, ids)
    eoff, eids, est = ix.match(w.t_bytes, w.t_off)
    topics = w.topics()
    got = {}
    lock = threading.Lock()
    done = threading.Event()
    want = 3 * len(topics)

    def put(key, st, vals):
        with lock:
            got[key] = (st, sorted(vals))
            if len(got) == want:
                done.set()

    @N.tm_match_cb
    def cb_ids(ctx, st, p, n):
        put(("ids", ctx), st, [p[i] for i in range(n)])

    def span_vals(sp, ns, width):
        out = []
        T = N.C.c_uint32 if width == 4 else N.C.c_uint64
        for j in range(ns):
            base = sp + 16 * j
            ptr = N.C.c_void_p.from_address(base).value
            n = N.C.c_uint64.from_address(base + 8).value
            arr = (T * n).from_address(ptr) if n else []
            out.extend(int(x) for x in arr)
        return out

    @N.tm_spans_cb
    def cb_spans(ctx, st, sp, ns, nids):
        put(("spans", ctx), st, span_vals(sp, ns, 8) if sp else [])

    @N.tm_spans32_cb
    def cb_spans32(ctx, st, sp, ns, nids):
        put(("spans32", ctx), st, span_vals(sp, ns, 4) if sp else [])

    b = N.Batcher(eng, max_batch=512, max_wait_us=300)
    for i, t in enumerate(topics):
        ctx = N.C.c_void_p(i + 1)
        assert b.lib.tm_batcher_submit(b.h, t, len(t), cb_ids, ctx) == N.TM_OK
        assert b.lib.tm_batcher_submit_spans(b.h, t, len(t), cb_spans, ctx) == N.TM_OK
        assert b.lib.tm_batcher_submit_spans32(b.h, t, len(t), cb_spans32, ctx) == N.TM_OK
    assert done.wait(120)
    b.close()
    for i in range(len(topics)):
        exp = [int(x) for x in eids[eoff[i]:eoff[i + 1]]]
        for kind in ("ids", "spans"):
            st, vals = got[(kind, i + 1)]
            assert st == est[i] and vals == (exp if st == N.TM_TOPIC_OK else []), (kind, i)
        st, vals = got[("spans32", i + 1)]
        if wide_ids and est[i] == N.TM_TOPIC_OK and exp:
            assert st == N.TM_ESTATE and vals == [], i
        elif st == N.TM_TOPIC_OK:
            assert vals == exp, i
        else:
            assert st == est[i] or (wide_ids and st == N.TM_ESTATE), i
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("transport", [N.TM_TRANSPORT_AUTO, N.TM_TRANSPORT_IDS], ids=["runs", "ids"])
def test_gpu_lone_high_fanout_publish_does_not_size_later_windows(transport):
    """with the default max_batch (65,536), one publish matching 16,384
    filters alone in its window must not set the per-publish sizing marks (they would size the
    next windows' buffers at 1.25 x 65,536 x 16,384 ids: GBs of HBM and pinned host memory).
    Device and host memory stay within a bound after it, and later windows stay correct."""
    import psutil
    import torch
    levels = 14
    topic = "/".join(f"l{k}" for k in range(levels)).encode()
    filters = ["/".join("+" if (m >> k) & 1 else f"l{k}" for k in range(levels)).encode() for m in range(1 << levels)]
    eng = N.Engine(0)
    eng.apply([(N.TM_OP_ADD, f, i) for i, f in enumerate(filters)] + [(N.TM_OP_ADD, b"x/+", 1 << 20)])
    eng.commit()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    rss0 = psutil.Process().memory_info().rss
    b = N.Batcher(eng, max_wait_us=200, transport=transport)  # max_batch 0: the default 65,536
    try:
        for _ in range(3):  # lone publishes, each its own window
            st, ids = b.match(topic)
            assert st >= 0 and sorted(int(i) for i in ids) == list(range(1 << levels))
        # then a window of ordinary publishes from many threads
        bad = []

        def worker(k):
            for j in range(200):
                st, ids = b.match(b"x/%d" % (k * 1000 + j))
                if sorted(int(i) for i in ids) != [1 << 20]:
                    bad.append((k, j))

        th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not bad, bad[:4]
        st, ids = b.match(topic)
        assert len(ids) == 1 << levels
        free1 = torch.cuda.mem_get_info(0)[0]
        rss1 = psutil.Process().memory_info().rss
    finally:
        b.close()
        eng.close()
    assert free0 - free1 < (1 << 30), (free0 - free1) / 2**20  # MiB of HBM the aggregator took
    assert rss1 - rss0 < (1 << 30), (rss1 - rss0) / 2**20
