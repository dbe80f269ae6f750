"""bench.py — matched publishes/s of the MI355X topic-matching engine on BASELINE config C.

    python bench.py [--gpus N --steps K --warmup W] [--config C --scale 1.0 --batch 1000000]

One step = one batch of `--batch` synthetic publishes matched against the 10M-key
config-C filter set (BASELINE.json configs[2]: the config the metric is quoted on).
Inputs are resident in HBM when the timed region starts; a step is the full device
pipeline (tokenise -> word lookup -> trie walk -> output compaction) through the C-ABI
(tm_match_device) on the current torch stream.

Multi-GPU (launched by torch.distributed.run): the trie is replicated, every rank owns
its own `--batch` publishes (weak scaling, no data-path collective); value = all ranks'
publishes / max-over-ranks time.

Rank 0 at N=1 also times the CPU baseline: the C++ restatement of the reference's
emqx_trie_search over an Erlang-term-ordered key set (oracle/, "kind": "port") on a
bounded sample of the same topics, and checks the GPU results of that sample bit-exactly.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

# Two device batches in flight need their two streams on different hardware queues; HIP's
# default is 4 queues per process, shared round-robin by every stream the process creates
# (torch's, each engine's two, three per calling thread per engine for the host-form calls,
# the aggregator's three).  With 8, the config-B engine built beside config C's ran its first
# ~6 runs-form calls at 3.1 ms instead of 1.2 ms (its H2D, walk and D2H streams landed on
# queues other streams held; profiles/r04_probe_hwq*_o.jsonl), so the bench asks for 16.
# Set before HIP starts.
if os.environ.get("EMQX_BENCH_HWQ"):  # development: A/B of the queue count
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["EMQX_BENCH_HWQ"]
elif int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "matched publishes/sec at 10M filters (1/2/4/8 GPU) + p99 batch latency"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(st, topic_bytes, n):
    """Bytes one batch must move at minimum under the frozen layout, from
    the kernel's own walk counters `st` (Engine.STAT_NAMES):
      topic bytes + u32 offsets in,
      16 B per word-table probe, 16 B per edge-table probe, 16 B per node record read,
      4 B per key read from the terminal-list arena (keys not inlined in an edge slot),
      4 B per key written, 12 B per topic of results (offset, count, status)."""
    arena_keys = st["keys"] - st["inline_keys"]
    return (topic_bytes + 4 * (n + 1) + 16 * st["word_probes"] + 16 * st["edge_probes"]
            + 16 * st["node_records"] + 4 * arena_keys + 4 * st["keys"] + 12 * n)


KERNEL_SRCS = ("emqx_amd/csrc/match_kernels.hip", "emqx_amd/csrc/layout.h", "emqx_amd/csrc/device_api.h",
               "emqx_amd/csrc/wave.h")


def kernel_src_sha():
    """Hash of the kernel sources, computed like tools/prof_pmc.sh's `sha256sum` listing."""
    import hashlib
    lines = "".join(f"{hashlib.sha256(open(os.path.join(ROOT, f), 'rb').read()).hexdigest()}  {f}\n"
                    for f in KERNEL_SRCS)
    return hashlib.sha256(lines.encode()).hexdigest()


def profiled_traffic(workload_keys, batch, any_config=False):
    """HBM bytes per k_match_fast launch from the committed PMC profile of THIS kernel
    source (profiles/*.json written by tools/summarize_prof.py from tools/prof_pmc.sh),
    or None.  rocprofv3 cannot run inside the process it profiles, so the counters come
    from a separate run of this same bench command; the source hash ties them to the code."""
    import glob
    sha = kernel_src_sha()
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if not isinstance(d, dict) or d.get("kernel_src_sha") != sha:
            continue
        cfg = d.get("bench_line", {}).get("config", {})
        if not any_config and (cfg.get("route_keys") != workload_keys
                               or cfg.get("publishes_per_step_per_gpu") != batch):
            continue
        t = dict(d["traffic"])
        pmc = d.get("pmc_per_launch", {})
        if "TCC_HIT_sum" in pmc:
            t["tcc_hit"], t["tcc_miss"] = pmc["TCC_HIT_sum"], pmc["TCC_MISS_sum"]
        best = (p, t)
    return best


def _loadgen():
    import ctypes as C
    lg = C.CDLL(os.path.join(ROOT, "tools", "libtm_loadgen.so"))
    lg.loadgen_run2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_int,
                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    from emqx_amd import _native as N
    lg.loadgen_run3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(N.tm_batcher_stats)]
    lg.loadgen_run4.argtypes = lg.loadgen_run3.argtypes + [C.POINTER(N.tm_batcher_window), C.c_uint32,
                                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
    lg.spans_checksum.restype = C.c_uint64
    lg.spans_checksum.argtypes = [C.c_void_p, C.c_uint32]
    return lg


def batcher_load(eng, tb, to32, seconds, plan=None, repin=None):
    """End to end through the batching aggregator (include/emqx_tm_batcher.h): P concurrent
    publishers, each with one publish in flight (tools/loadgen.cpp), each publish answered
    with its own route ids on the host, every id read once by the callback (a checksum, as a
    NIF building its reply reads each id).  Not the metric: the per-publish latency a broker
    process would see, and the rate once the results leave the GPU.  Default transport: runs
    (the walk's spans of the engine's host id arena cross PCIe); `ids` rows ship the ids."""
    import ctypes as C

    from emqx_amd import _native as N
    lg = _loadgen()
    runs = []
    # the cutter and the completion thread each keep a CPU of the 16-CPU share: 14 delivery
    # threads.  With the process pinned to 16 CPUs (placement.pin_to_gpu), 15 threads left the
    # cutter waiting for a CPU: 60.2 / 59.7 M/s id lists against 80.4-86.1 M/s at 14 in the
    # same box runs (profiles/r05_batcher_acct_quota.jsonl, r05_batcher_grow_quota.jsonl)
    dt = max(2, min(14, cpu_topology()["usable_cpus"] - 2))
    plan = plan or [(4096, N.TM_TRANSPORT_AUTO, 0), (65536, N.TM_TRANSPORT_AUTO, 0), (262144, N.TM_TRANSPORT_AUTO, 0),
            (65536, N.TM_TRANSPORT_AUTO, 1), (65536, N.TM_TRANSPORT_AUTO, 3), (65536, N.TM_TRANSPORT_IDS, 0),
            (65536, N.TM_TRANSPORT_IDS, 3),  # a replica's transport (no host id arena), u32 ids read in place
            (65536, N.TM_TRANSPORT_AUTO, 0), (65536, N.TM_TRANSPORT_AUTO, 0)]
    # the headline row (65,536 publishers, id lists) runs three times, spread over the leg: one
    # 2 s window of it ranged 42-78 M/s across box runs (round 6), so the row reports the
    # median of the three runs, with all three rates (`repeats`)
    warm = 0.5
    for pubs, transport, spans in plan:
        # each row's threads start on cores picked just before it: the rate follows the CPUs the
        # process gets (round 6: three runs of one row at 14.6 / 11.1 / 9.1 CPUs of use made
        # 76 / 58 / 46 M/s, 5.2 M/s per CPU each, the slow ones preempted by other jobs)
        placed_row = repin() if repin else None
        b = N.Batcher(eng, max_batch=65536, max_wait_us=200, delivery_threads=dt, transport=transport)
        got, ids, errs, cs, el = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_double()
        win = N.tm_batcher_stats()
        wbuf = (N.tm_batcher_window * N.TM_BATCHER_WINDOWS)()
        wn = C.c_uint32()
        cg = (C.c_uint64 * 4)()
        rc = lg.loadgen_run4(b.h, tb.ctypes.data, to32.ctypes.data, len(to32) - 1, pubs, warm, seconds, spans,
                             C.byref(got), C.byref(ids), C.byref(errs), C.byref(cs), C.byref(el), C.byref(win),
                             wbuf, N.TM_BATCHER_WINDOWS, C.byref(wn), cg)
        st = b.stats()
        b.close()
        if rc != 0 or errs.value or not win.lat_count:
            raise RuntimeError(f"batcher load failed: rc {rc}, {errs.value} failed publishes")
        rate = win.lat_count / win.window_s  # publishes delivered in the steady-state window
        little_ms = pubs / rate * 1e3        # closed loop: mean latency = publishers / throughput
        mean_ms = win.lat_mean_us / 1e3
        runs.append({"publishers": pubs,
                     "transport": "runs" if transport != N.TM_TRANSPORT_IDS else "ids (u32 over PCIe)",
                     "callback": {0: "id list (tm_batcher_submit)", 1: "spans (tm_batcher_submit_spans)",
                                  3: "u32 spans (tm_batcher_submit_spans32)"}[spans],
                     "publishes_per_s": round(rate, 1),
                     "publishes_per_s_whole_run": round(got.value / el.value, 1),
                     "ids_per_s": round(ids.value / el.value, 1),
                     "mean_batch": round(st["publishes"] / max(st["batches"], 1), 1),
                     "lat_mean_ms": round(mean_ms, 3),
                     "lat_p50_ms": round(win.lat_p50_us / 1e3, 3), "lat_p99_ms": round(win.lat_p99_us / 1e3, 3),
                     "lat_p999_ms": round(win.lat_p999_us / 1e3, 3), "lat_max_ms": round(win.lat_max_us / 1e3, 3),
                     "lat_sample": int(win.lat_count), "window_s": round(win.window_s, 3),
                     "littles_law": {"publishers_over_rate_ms": round(little_ms, 3),
                                     "mean_over_that": round(mean_ms / little_ms, 3),
                                     "ok": bool(abs(mean_ms - little_ms) <= 0.2 * little_ms)},
                     "backend_frac": round(st["backend_us"] * 1e-6 / el.value, 3),
                     # share of the run's wall time each pipeline stage was busy (stages overlap)
                     "stage_busy": {k: round(st[k + "_us"] * 1e-6 / el.value, 3)
                                    for k in ("cut", "enqueue", "gpu_wait", "copy", "deliver")},
                     "windows": window_stages(wbuf, wn.value),
                     "host_placement": placed_row,
                     "cgroup_cpu": {"usage_cpus": round(cg[0] * 1e-6 / max(win.window_s, 1e-9), 2),
                                    "periods": int(cg[1]), "throttled_periods": int(cg[2]),
                                    "throttled_ms": round(cg[3] / 1e3, 3)}})
        if not runs[-1]["littles_law"]["ok"]:
            log(f"batcher: latency mean {mean_ms:.3f} ms differs from publishers / rate {little_ms:.3f} ms by > 20%")
    merged, order = {}, []
    for r in runs:  # repeated rows: the run with the median rate stands for the row
        k = (r["publishers"], r["transport"], r["callback"])
        if k not in merged:
            order.append(k)
        merged.setdefault(k, []).append(r)
    runs = []
    for k in order:
        g = sorted(merged[k], key=lambda r: r["publishes_per_s"])
        r = dict(g[len(g) // 2])
        if len(g) > 1:
            r["repeats"] = [x["publishes_per_s"] for x in merged[k]]
            # what each repeat got from the host (a slow one: fewer CPUs, preempted delivery?)
            r["repeat_host"] = [{"publishes_per_s": x["publishes_per_s"], "cgroup_cpu": x["cgroup_cpu"],
                                 "host_placement": x.get("host_placement"),
                                 "stage_busy": x["stage_busy"],
                                 "slowest_1pct": (x.get("windows") or {}).get("stage_ms_slowest_1pct")}
                                for x in merged[k]]
        runs.append(r)
    return {"api": f"tm_batcher_submit (max_batch 65536, max_wait 200 us, {dt} delivery threads)", "runs": runs,
            "note": "closed loop: each publisher resubmits from its result callback, which reads every id once; "
                    "six windows in flight (GPU walk / PCIe / callbacks); runs transport: spans cross PCIe and "
                    "replies are read from the host id arena (one span: zero-copy; several: gathered); "
                    f"rate and latency over a {seconds:g} s steady-state window after {warm:g} s of warm-up "
                    "(every publish delivered in it, tm_batcher_stats_reset / _get), checked against Little's law; "
                    "stage_busy: share of wall time each stage worked (copy and deliver: per delivery thread)"}


def window_stages(wbuf, n):
    """Where the aggregator's windows spent their time (tm_batcher_window stamps of the windows
    completed in the measured steady state), to attribute the latency tail to a stage.  Per
    window: wait (its oldest publish's submit -> the cutter takes it: the window filling, or
    the cutter busy / off-CPU), cut (queue -> pinned staging -> GPU part queued), gpu (queued ->
    observed done, behind the windows ahead of it), ready (counters read, any re-run, D2H queued),
    queue (handed over -> a delivery thread starts on it), deliver (first -> last callback).  The
    window's span (oldest submit -> last callback) bounds the latency of every publish in it."""
    import numpy as np
    if not n:
        return None
    f = {k: np.array([getattr(wbuf[i], k) for i in range(n)], dtype=np.float64)
         for k in ("n", "flags", "t_oldest", "t_cut", "t_queued", "t_gpu", "t_ready", "t_deliver", "t_done", "epoch",
                   "t_slot", "cut_cpu_us", "cut_ivcsw", "wait_ivcsw", "del_cpu_us", "del_wall_us", "del_ivcsw")}
    t_del = np.where(f["t_deliver"] > 0, f["t_deliver"], f["t_ready"])
    t_slot = np.clip(f["t_slot"], f["t_oldest"], f["t_cut"])
    st = {"wait": f["t_cut"] - f["t_oldest"], "cut": f["t_queued"] - f["t_cut"], "gpu": f["t_gpu"] - f["t_queued"],
          "ready": f["t_ready"] - f["t_gpu"], "queue": t_del - f["t_ready"], "deliver": f["t_done"] - t_del,
          # wait = fill (the window filling / max_wait polling) + slot (no free slot: pipeline full)
          "wait_fill": t_slot - f["t_oldest"], "wait_slot": f["t_cut"] - t_slot,
          # CPU the cutter spent in its cut stage, and the delivery threads' CPU over their wall
          "cut_cpu": f["cut_cpu_us"] * 1e3, "del_cpu": f["del_cpu_us"] * 1e3, "del_wall": f["del_wall_us"] * 1e3}
    cnt = {"cut_ivcsw": f["cut_ivcsw"], "wait_ivcsw": f["wait_ivcsw"], "del_ivcsw": f["del_ivcsw"]}
    span = f["t_done"] - f["t_oldest"]
    order = np.argsort(span)
    k1 = max(1, n // 100)

    def ms(idx):
        out = {k: round(float(np.mean(v[idx])) / 1e6, 3) for k, v in st.items()}
        out.update({k: round(float(np.mean(v[idx])), 2) for k, v in cnt.items()})  # counts, not ms
        return out
    worst = int(order[-1])
    gaps = np.diff(np.sort(f["t_cut"])) if n > 1 else np.zeros(1)
    return {"windows": int(n), "mean_publishes": round(float(np.mean(f["n"])), 1),
            "span_ms": {"p50": round(float(np.percentile(span, 50)) / 1e6, 3),
                        "p99": round(float(np.percentile(span, 99)) / 1e6, 3),
                        "max": round(float(span[worst]) / 1e6, 3)},
            "stage_ms_median_window": ms(order[n // 2:n // 2 + 1]),
            "stage_ms_slowest_1pct": ms(order[-k1:]),
            "stage_ms_slowest": ms(np.array([worst])),
            "slowest_publishes": int(f["n"][worst]),
            "reruns": int(np.sum((f["flags"].astype(np.int64) & 1) != 0)),
            "epochs_seen": int(len(np.unique(f["epoch"]))),
            # delivery CPU per publish (all windows): the callbacks' own cost, which outside
            # contention for caches / DRAM raises without any preemption
            "deliver_cpu_ns_per_publish": round(float(np.sum(f["del_cpu_us"]) * 1e3 / max(np.sum(f["n"]), 1)), 1),
            "cut_cpu_ns_per_publish": round(float(np.sum(f["cut_cpu_us"]) * 1e3 / max(np.sum(f["n"]), 1)), 1),
            # preemption: involuntary context switches of the cutter (over its cut stage) and the
            # delivery threads, in the slowest 1 % of windows against all windows
            "ivcsw_per_window": {k: {"all": round(float(np.mean(v)), 3), "slowest_1pct": round(float(np.mean(v[order[-k1:]])), 3)}
                                 for k, v in cnt.items()},
            "max_gap_between_cuts_ms": round(float(np.max(gaps)) / 1e6, 3)}


def replica_batcher_leg(eng, tb, to32, seconds):
    """The aggregator on a READ REPLICA of the index (mode 1's other ranks, §6): the master's
    image copied into a replica on the same GPU, which keeps its own host id arena from its
    device copy, then the 65,536-publisher rows with both transports."""
    import torch

    from emqx_amd import _native as N
    nb = eng.image_size()
    img = torch.empty(nb, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    eng.image_export(img.data_ptr(), nb)
    t0 = time.perf_counter()
    rep = N.Engine.replica_from_image(0, img.data_ptr(), nb)
    t_load = time.perf_counter() - t0
    del img
    torch.cuda.empty_cache()
    try:
        r = batcher_load(rep, tb, to32, seconds,
                         plan=[(65536, N.TM_TRANSPORT_AUTO, 0), (65536, N.TM_TRANSPORT_AUTO, 1),
                               (65536, N.TM_TRANSPORT_IDS, 0)])
    finally:
        rep.close()
    r["replica_load_s"] = round(t_load, 3)
    r["image_bytes"] = nb
    return r


def host_runs_leg(eng, tb, to32, n, w, reps=10):
    """SURVEY §8(d)'s protocol on the runs form: H2D of the topics + walk + D2H of the spans
    and per-topic arrays + the host view (tm_match_batch_runs), with the batch in pinned
    memory as an aggregator holds it (and from pageable memory, staged by the engine); the
    same plus a read of every id (tools/loadgen.cpp spans_checksum, 8 threads).  Parity: the
    ids of the first 20,000 topics vs the oracle."""
    import ctypes as C

    import torch
    lg = _loadgen()
    pin = torch.empty(len(tb), dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:] = tb
    pinned = pin.numpy()
    out = {"api": "tm_match_batch_runs", "batch": n}
    for name, buf in (("pinned", pinned), ("pageable", tb)):
        eng.match_runs_view(buf, to32)
        eng.lib.tm_runs_release(eng.h)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.match_runs_view(buf, to32)
            ts.append(time.perf_counter() - t0)
            eng.lib.tm_runs_release(eng.h)
        dt = float(np.mean(ts))
        out[name] = {"ms_per_batch": round(dt * 1e3, 3), "p50_ms": round(float(np.percentile(ts, 50)) * 1e3, 3),
                     "p99_ms": round(float(np.percentile(ts, 99)) * 1e3, 3), "publishes_per_s": round(n / dt, 1)}
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        res = eng.match_runs_view(pinned, to32)
        lg.spans_checksum(C.byref(res), 8)
        ts.append(time.perf_counter() - t0)
        eng.lib.tm_runs_release(eng.h)
    dt = float(np.mean(ts))
    out["pinned_read_every_id"] = {"ms_per_batch": round(dt * 1e3, 3), "publishes_per_s": round(n / dt, 1),
                                   "p50_ms": round(float(np.percentile(ts, 50)) * 1e3, 3),
                                   "p99_ms": round(float(np.percentile(ts, 99)) * 1e3, 3), "threads": 8}
    res = eng.match_runs_view(pinned, to32)
    out["spans_per_batch"] = int(res.total_spans)
    out["ids_per_batch"] = int(res.total_ids)
    out["d2h_bytes"] = int(res.total_spans) * 16 + 16 * n
    eng.lib.tm_runs_release(eng.h)
    ps = min(n, 20000)
    o, ids, kcnt, st = eng.match_runs(tb, to32[:ps + 1])
    eo, eids, est = oracle_index(w).match(tb, to32[:ps + 1], threads=16)
    bad = sum(1 for i in range(ps) if not np.array_equal(np.sort(ids[o[i]:o[i + 1]]), eids[eo[i]:eo[i + 1]]))
    bad += int(np.sum(st != est))
    out["parity"] = {"sampled_topics": ps, "mismatches": int(bad), "oracle": "oracle/trie_search.cpp"}
    out["note"] = ("spans of the engine's host id arena (16 B each) cross PCIe instead of 4 B per key; the host view "
                   "is the spans themselves (the GPU writes their host addresses); pinned: the caller's batch is DMA'd "
                   "directly")
    if bad:
        log(f"PARITY FAILURE (runs): {bad}/{ps} topics differ")
    return out


def end_to_end(runs, keys):
    """SURVEY §8(d)'s timing protocol: publishes/s = B / mean(H2D of the topics + kernels + D2H
    + host result view), over the timed batches of the runs leg (tm_match_batch_runs: the
    host view is the spans of route ids in the engine's host id arena), and the same with
    every id then read by 8 host threads (what a consumer pays at least once); the keys form
    (every key handle copied to the host) beside it."""
    if not runs:
        return None
    pin, rd = runs["pinned"], runs["pinned_read_every_id"]
    return {
        "protocol": "SURVEY.md §8(d): B / mean(H2D + kernel + D2H + host result view), topics from host "
                    "memory, results as host spans of route ids; batches timed one after another",
        "api": "tm_match_batch_runs",
        "batch": runs["batch"],
        "publishes_per_s": pin["publishes_per_s"],
        "ms_per_batch": pin["ms_per_batch"],
        "p50_batch_ms": pin["p50_ms"],
        "p99_batch_ms": pin["p99_ms"],
        "read_every_id": {"publishes_per_s": rd["publishes_per_s"], "ms_per_batch": rd["ms_per_batch"],
                          "p50_batch_ms": rd["p50_ms"], "p99_batch_ms": rd["p99_ms"], "threads": rd["threads"],
                          "ids_per_batch": runs["ids_per_batch"]},
        "pageable_topics": runs["pageable"]["publishes_per_s"],
        "keys_form": ({"api": keys["api"], "publishes_per_s": keys["publishes_per_s"],
                       "ms_per_batch": keys["ms_per_batch"]} if keys else None),
        "parity": runs["parity"],
    }


def gather_roof(walk, kernel_ms, table_bytes):
    """The walk's second ceiling: independent random 16-B requests (edge + word probes).
    tools/gather_roof.hip measured what one MI355X serves with nothing dependent between
    loads, per table size (profiles/*gather_roof.jsonl); the row used is the one measured at
    the engine's allocated edge-table size (the smallest measured table >= it, else the
    largest): 16 GiB at config C (edge load 1/16), where random misses are served at ~39 G/s
    against ~49 G/s from a 4 GiB table."""
    import glob
    ceil = None
    want_mib = table_bytes / 2**20
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*gather_roof.jsonl"))):
        rows = [json.loads(x) for x in open(p) if x.strip().startswith("{")]
        sizes = sorted({r["table_MiB"] for r in rows if "table_MiB" in r})
        if not sizes:
            continue
        pick = next((m for m in sizes if m >= want_mib), sizes[-1])
        ceil = (os.path.relpath(p, ROOT), max(r["G_loads_per_s"] for r in rows if r.get("table_MiB") == pick), pick)
    probes = walk["edge_probes"] + walk["word_probes"]
    rate = probes / (kernel_ms * 1e-3) / 1e9
    out = {"probes_per_launch": probes, "achieved_G_probes_per_s": round(rate, 2),
           "edge_table_MiB": round(want_mib, 1)}
    if ceil:
        out.update({"ceiling_G_loads_per_s": ceil[1], "ceiling_table_MiB": ceil[2], "source": ceil[0]})
        # request model: every L2 miss at the random-miss rate, every L2 hit at the
        # L2-resident random rate (2 MiB table), the key writes at the stream rate; the
        # L2 hit/miss request counts come from the PMC profile of this kernel source
        rows = [json.loads(x) for x in open(os.path.join(ROOT, ceil[0])) if x.strip().startswith("{")]
        hit_rate = max([r["G_loads_per_s"] for r in rows if r.get("table_MiB") == 2] or [0])
        prof = profiled_traffic(None, None, any_config=True)
        if hit_rate and prof:
            pmc = prof[1]
            hits, misses = pmc.get("tcc_hit"), pmc.get("tcc_miss")
            if hits and misses:
                model_ms = (misses / (ceil[1] * 1e9) + hits / (hit_rate * 1e9)
                            + 4 * walk["keys"] / 6.29e12) * 1e3
                out["request_model"] = {"l2_miss_requests": int(misses), "l2_hit_requests": int(hits),
                                        "miss_rate_G_per_s": ceil[1], "hit_rate_G_per_s": hit_rate,
                                        "key_write_GBps": 6290.0, "model_ms": round(model_ms, 4),
                                        "frac": round(model_ms / kernel_ms, 3),
                                        "source": os.path.relpath(prof[0], ROOT)}
    return out


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model


def cpu_topology():
    """What the CPU baseline can use on this host: logical CPUs, this process's affinity
    set, the cgroup CPU quota (cpu.max, in CPUs; None if unlimited), the job's announced CPU
    share (OMP_NUM_THREADS), sockets and threads per core from /proc/cpuinfo.  The baseline's
    thread count is the smallest of affinity, quota and share (the CPUs this job may run on
    at once; one thread per BEAM scheduler), unless --cpu-threads says otherwise."""
    import math
    info = {"logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "sockets": None, "threads_per_core": None}
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()[:2]
            if q != "max":
                info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
    try:
        phys, cores, sib = set(), None, None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k = k.strip()
            if k == "physical id":
                phys.add(v.strip())
            elif k == "cpu cores" and cores is None:
                cores = int(v)
            elif k == "siblings" and sib is None:
                sib = int(v)
        info["sockets"] = len(phys) or None
        if cores and sib:
            info["threads_per_core"] = sib // cores
    except (OSError, ValueError):
        pass
    # the job's CPU share as the pool announces it (OMP_NUM_THREADS: 16 per GPU on the box)
    try:
        info["job_share_cpus"] = int(os.environ["OMP_NUM_THREADS"])
    except (KeyError, ValueError):
        info["job_share_cpus"] = None
    usable = info["affinity_cpus"]
    if info["cgroup_quota_cpus"]:
        usable = min(usable, max(1, math.floor(info["cgroup_quota_cpus"])))
    if info["job_share_cpus"]:
        usable = min(usable, info["job_share_cpus"])
    info["usable_cpus"] = usable
    return info


def cgroup_cpu_stat():
    """The job's cgroup CPU accounting (cgroup v2 cpu.stat): periods, throttled periods and
    throttled time.  With a quota (cpu.max), a period whose quota runs out stops every thread
    of the job until the period ends -- the match path's threads included.  {} when absent."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            kv = dict(line.split() for line in f if line.strip())
        return {k: int(kv[k]) for k in ("nr_periods", "nr_throttled", "throttled_usec") if k in kv}
    except (OSError, ValueError):
        return {}


def cgroup_delta(a, b):
    if not a or not b:
        return None
    return {"periods": b.get("nr_periods", 0) - a.get("nr_periods", 0),
            "throttled_periods": b.get("nr_throttled", 0) - a.get("nr_throttled", 0),
            "throttled_ms": round((b.get("throttled_usec", 0) - a.get("throttled_usec", 0)) / 1e3, 3)}


def host_rss_gib():
    """Peak resident host memory of this rank (the engine's host master copy + workload)."""
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, gpus, port):
    """The command that starts `gpus` ranks of this bench, one process per GPU, with the same
    arguments (torch.distributed.run on one node, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def world_plan(gpus, env):
    """What this process is, before anything touches the GPU: ("launch", N) when no launcher
    started it and N > 1 ranks are asked for (the parent starts N fresh rank processes and
    relays rank 0's line), ("rank", world) when a launcher did (WORLD_SIZE must equal
    --gpus), ("single", 1) otherwise."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("launch", gpus) if gpus > 1 else ("single", 1)
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} set by the launcher but --gpus {gpus}: refusing to "
                         f"report a {ws}-rank run as {gpus} GPUs")
    return ("rank", int(ws))


def launch_ranks(argv, gpus):
    """Parent of an N-rank run started without a launcher: no GPU call happens here; the ranks
    are child processes (their stdout, where rank 0 prints the JSON line, is this process's)."""
    import subprocess
    cmd = launcher_cmd(argv, gpus, _free_port())
    log(f"bench.py: starting {gpus} ranks: {' '.join(cmd)}")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launch_check():
    """--launch-check: each rank joins a gloo group and all-reduces its rank; rank 0 prints
    one JSON line (CPU test of the launcher plumbing, no GPU)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([rank + 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        emit(json.dumps({"n_gpus": world, "rank_sum": int(t.item()),
                          "local_ranks": os.environ.get("LOCAL_WORLD_SIZE")}))
    if world > 1:
        dist.destroy_process_group()



LINE_MAX = 12 * 1024  # the driver parses the one printed line; round 5's 32 KB line was not parsed


def _pick(d, *keys):
    return {k: d[k] for k in keys if d and k in d} if d else None


def compact_line(out, detail_path):
    """The ONE printed JSON line: the headline fields, the roofline and CPU baseline, parity,
    and a one-level summary of every leg.  Everything else (window traces, per-depth walk
    counters, per-publisher-count aggregator rows, per-epoch churn timings) goes to
    `detail_path` beside it."""
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                                "p50_batch_ms", "p99_batch_ms") if k in out}
    rf = out.get("roofline") or {}
    line["roofline"] = _pick(rf, "bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms",
                             "algorithmic_bytes_per_launch", "frac_per_step")
    if rf.get("traffic_source"):
        line["roofline"]["traffic_source"] = rf["traffic_source"][:160]
    cpu = out.get("cpu_baseline")
    if cpu:
        line["cpu_baseline"] = _pick(cpu, "value", "unit", "cores", "kind", "value_1_thread")
        line["cpu_baseline"]["sample"] = cpu.get("sample", "")[:240]
        if cpu.get("host"):
            line["cpu_baseline"]["cpu_model"] = cpu["host"].get("model")
    else:
        line["cpu_baseline"] = None
    line["parity"] = out.get("parity")
    if out.get("replica_parity") is not None:
        line["replica_parity"] = out["replica_parity"]
    line["one_batch_in_flight"] = _pick(out.get("one_batch_in_flight"), "publishes_per_s", "ms_per_step", "p99_batch_ms")
    e2e = out.get("end_to_end")
    line["end_to_end"] = _pick(e2e, "api", "publishes_per_s", "ms_per_batch", "p99_batch_ms")
    if e2e and e2e.get("parity"):
        line["end_to_end"]["parity_mismatches"] = e2e["parity"].get("mismatches")
    b = out.get("batcher")
    if b and b.get("runs"):
        cpu_v = cpu["value"] if cpu else None
        rows = {}
        for r in b["runs"]:
            key = f"{r['publishers']} {r['transport'].split()[0]} {r['callback'].split(' (')[0]}"
            rows[key] = {"publishes_per_s": r["publishes_per_s"], "lat_p99_ms": r["lat_p99_ms"],
                         "x_cpu": round(r["publishes_per_s"] / cpu_v, 1) if cpu_v else None}
            if r.get("repeats"):
                rows[key]["repeats"] = r["repeats"]
                rows[key]["stat"] = f"median of {len(r['repeats'])} runs"
        line["batcher"] = {"api": b.get("api"), "rows": rows}
        head = [r for r in b["runs"] if r["publishers"] == 65536 and r["transport"] == "runs"
                and r["callback"].startswith("id list")]
        if head:
            line["batcher"]["headline_65536_id_list"] = rows[next(k for k in rows if k.startswith("65536 runs id list"))]
        rep = b.get("on_replica")
        if rep and rep.get("runs"):
            line["batcher"]["on_replica"] = {f"{r['publishers']}": r["publishes_per_s"] for r in rep["runs"]}
    line["other_modes_ms"] = {k: v["ms_per_batch"] for k, v in (out.get("other_modes") or {}).items()}
    rb = out.get("rebuild_under_load")
    if rb:
        line["rebuild_under_load"] = _pick(rb, "ops", "full_rebuild", "commit_s", "commit_phase_s", "max_at_ms")
        line["rebuild_under_load"]["match_ms_during_commit"] = rb.get("match_ms_during_commit")
        line["rebuild_under_load"]["match_ms_before"] = rb.get("match_ms_before")
        if rb.get("slowest_matches"):
            line["rebuild_under_load"]["slowest_matches"] = rb["slowest_matches"][:2]
            line["rebuild_under_load"]["publish_reallocs"] = rb.get("publish_reallocs")
    ch = out.get("churn_E")
    if ch:
        line["churn_E"] = _pick(ch, "epochs", "ops_per_epoch", "route_ops_per_s", "commit_ms_p50", "commit_ms_p99",
                                "commit_stall_ms_p50", "match_ms_p50", "publishes_per_s_incl_commit", "full_rebuilds")
        if ch.get("parity"):
            line["churn_E"]["parity_mismatches"] = ch["parity"].get("mismatches")
    cb = out.get("config_B")
    if cb:
        line["config_B"] = _pick(cb, "publishes_per_s", "ms_per_batch", "p99_batch_ms", "kernel_ms")
        if cb.get("roofline"):
            line["config_B"]["roofline_frac"] = cb["roofline"].get("frac")
    mf = out.get("matches_filter")
    if mf:
        line["matches_filter"] = _pick(mf, "queries", "queries_per_s", "ms_per_batch")
        if mf.get("cpu_baseline"):
            line["matches_filter"]["cpu_queries_per_s"] = mf["cpu_baseline"].get("value")
        if mf.get("parity"):
            line["matches_filter"]["parity_mismatches"] = mf["parity"].get("mismatches")
    it = out.get("intersection")
    if it:
        line["intersection"] = _pick(it, "pairs", "pairs_per_s", "ms_per_batch")
        if it.get("cpu_baseline"):
            line["intersection"]["cpu_pairs_per_s"] = it["cpu_baseline"].get("value")
        if it.get("parity"):
            line["intersection"]["parity_mismatches"] = it["parity"].get("mismatches")
    for k in ("spill_topics", "build_s", "batches_in_flight", "host_peak_rss_gib_max_over_ranks"):
        if k in out:
            line[k] = out[k]
    if out.get("library"):
        line["library"] = _pick(out["library"], "path", "src_sha")
    if out.get("replication"):
        line["replication"] = out["replication"]
    line["detail"] = detail_path
    s = json.dumps(line)
    if len(s) > LINE_MAX:  # never print a line the driver cannot take: drop the widest legs first
        for k in ("batcher", "rebuild_under_load", "churn_E", "matches_filter", "intersection", "config_B"):
            line.pop(k, None)
            s = json.dumps(line)
            if len(s) <= LINE_MAX:
                break
    return s


def write_detail(out, name="bench_detail.json"):
    """The full record (every leg, every trace) beside the printed line; returns its path."""
    d = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, name)
        with open(path, "w") as f:
            json.dump(out, f)
        return os.path.relpath(path, ROOT)
    except OSError as e:
        return f"not written: {e}"


_STDOUT = sys.stdout


def json_stdout_only():
    """From here on, stdout carries this process's JSON line and nothing else: whatever else
    writes to fd 1 (gloo's and RCCL's connection banners, a library's print) goes to stderr,
    so the driver reads one parseable line per run.  (A process that launches the ranks keeps
    its stdout: they inherit it.)"""
    global _STDOUT
    sys.stdout.flush()
    _STDOUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr


def emit(s: str):
    print(s, file=_STDOUT, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # >= 100 timed batches
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--distinct-batches", type=int, default=4,
                    help="N = 1: the timed steps cycle through this many distinct batches of --batch publishes "
                         "(N > 1: through the ranks' slices)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work (s)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: every CPU this process may use, see cpu_topology)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--in-flight", type=int, default=2, help="device batches in flight (1-3; --sequential: 1)")
    ap.add_argument("--sequential", action="store_true",
                    help="one batch in flight (default: two, alternating the engine's two direct buffer "
                         "sets on two streams; the sequential rate is reported beside either way)")
    ap.add_argument("--no-pin", action="store_true",
                    help="leave the process on every CPU (default: pin to the GPU's own socket, "
                         "emqx_amd/placement.py)")
    ap.add_argument("--batcher-seconds", type=float, default=2.0,
                    help="closed-loop load per publisher count through the batching aggregator (0: skip)")
    ap.add_argument("--profile", action="store_true", help="short run for rocprofv3 (no CPU baseline)")
    ap.add_argument("--quick", action="store_true",
                    help="development run: skip the CPU baseline and the matches_filter / intersection legs")
    ap.add_argument("--mode", choices=("replicated", "sharded"), default="replicated",
                    help="replicated trie, publishes data-parallel (default); or filters hash-sharded over "
                         "ranks with an RCCL all-gather merge (config D; DESIGN.md §6)")
    ap.add_argument("--exchange", choices=("padded", "exact", "local", "a2a"), default="padded",
                    help="sharded mode: padded all-gather (no host sync), exact all-gather-v by grouped "
                         "send/recv, local (each rank D2H's its own shard lists, no collective), or a2a "
                         "(all-to-all by topic range: each rank keeps 1/G of the batch's merged results)")
    ap.add_argument("--shard-of", type=int, default=0, metavar="G",
                    help="sharded mode on one process: hold shard 0 of a G-way split (per-GPU share of G GPUs)")
    ap.add_argument("--churn", type=int, default=0, metavar="EPOCHS",
                    help="config-E style run: EPOCHS delta epochs of 1%% adds + 1%% deletes, each committed "
                         "between match batches (commit and match timed separately)")
    ap.add_argument("--filter-search", type=int, default=0, metavar="Q",
                    help="matches_filter/3 run: Q topic-filter queries (the config's own filters, "
                         "generalised) walked on the GPU (tm_match_filter_batch), oracle beside it")
    ap.add_argument("--filter-kinds", default="", help="development: comma list of query kinds to keep "
                    "(0 stored filters, 1 one level '+', 2 prefix + '#')")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    # N ranks, one process per GPU: started here when no launcher did (before any GPU call)
    kind, _ = world_plan(args.gpus, os.environ)
    if kind == "launch":
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    json_stdout_only()
    if args.launch_check:
        return launch_check()
    if args.filter_search:
        return run_filter(args)
    if args.mode == "sharded":
        return run_sharded(args)
    if args.churn:
        return run_churn(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EMQX_BENCH_BACKEND=gloo: rehearse the multi-rank path on fewer GPUs than ranks (ranks
    # share devices, barrier/all-reduce over gloo); the default is RCCL, one rank per GPU
    backend = os.environ.get("EMQX_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    # Host placement: the engine's staging buffers, the host id arena the
    # runs-form replies read and the aggregator's delivery threads live in host memory, so
    # the rank runs on its GPU's socket; done before the workload and the engine allocate.
    from emqx_amd import placement
    placed = {"pinned": False, "reason": "--no-pin"} if args.no_pin else placement.pin_to_gpu(local)

    from emqx_amd import _native as N
    from emqx_amd import workloads
    lib_sha = N.check_build()  # the mapped library is the one built from these sources

    # ---------------------------------------------------------------- build
    # N = 1: one engine.  N > 1 (mode 1): rank 0 generates the workload and
    # builds the ONE host master copy; every other rank gets a read replica of its device
    # index (tm_image_export -> RCCL broadcast -> tm_replica_create) and its topic slice
    # over the same group, so host memory and build work are one copy per node.
    # The timed steps walk DISTINCT batches: rank r's step k walks slice (r + k) % n_slices of
    # the generated publishes (N = 1: --distinct-batches slices; N > 1: the ranks' slices), so
    # no step re-walks the batch the step before it walked.
    n_slices = world if world > 1 else max(1, args.distinct_batches)
    t0 = time.time()
    w = None
    if rank == 0:
        w = workloads.generate(args.config, scale=args.scale, n_topics=args.batch * n_slices)
    t_gen = time.time() - t0
    t0 = time.time()
    eng = None
    if rank == 0:
        eng = N.Engine(local, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4, record_patch=world > 1)
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
    t_build = time.time() - t0
    dev = torch.device("cuda", local)
    image_s = None
    if world > 1:
        from emqx_amd.replica import EngineReplicaAdapter, ReplicatedIndex
        t0 = time.time()
        rix = ReplicatedIndex(EngineReplicaAdapter(local, eng), rank, world)
        rix.start()
        eng = rix.ad.eng
        image_s = time.time() - t0
        # topics: rank 0's whole batch to every rank (untimed)
        tdev = dev if backend != "gloo" else torch.device("cpu")
        sz = torch.tensor([len(w.t_bytes), len(w.t_off)] if rank == 0 else [0, 0], dtype=torch.int64, device=tdev)
        dist.broadcast(sz, 0)
        all_b = (torch.from_numpy(w.t_bytes).to(tdev) if rank == 0
                 else torch.empty(int(sz[0].item()), dtype=torch.uint8, device=tdev))
        all_o = (torch.from_numpy(w.t_off.view(np.int32)).to(tdev) if rank == 0
                 else torch.empty(int(sz[1].item()), dtype=torch.int32, device=tdev))
        dist.broadcast(all_b, 0)
        dist.broadcast(all_o, 0)
        all_b, all_o = all_b.to(dev), all_o.to(dev)
    else:
        all_b = torch.from_numpy(w.t_bytes).to(dev)
        all_o = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    st = eng.stats()
    log(f"[rank {rank}] {'generated ' + str(w.n_keys) + ' keys in ' + format(t_gen, '.1f') + 's, ' if w else ''}"
        f"engine build {t_build:.1f}s{', replica image ' + format(image_s, '.1f') + 's' if image_s else ''}, "
        f"keys {st['n_keys']}, nodes {st['n_nodes']}, words {st['n_words']}, "
        f"index {st['device_bytes'] / 2**30:.2f} GiB, host RSS {host_rss_gib()} GiB")

    n = args.batch
    slices = []  # per slice: (bytes view, rebased offsets, topic bytes), all in HBM
    for j in range(n_slices):
        a, b = j * n, (j + 1) * n
        base = int(all_o[a].item())
        slices.append((all_b[base:], (all_o[a:b + 1] - base).contiguous(), int(all_o[b].item()) - base))
    own = rank % n_slices
    d_bytes, d_off, topic_bytes = slices[own]
    lo, hi = own * n, (own + 1) * n
    tb, to = (w.topic_slice(lo, hi) if rank == 0 else (None, None))
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)  # kernels and timing events share this stream
    sp = stream.cuda_stream

    def step(j=own):
        sb, so, stb = slices[j]
        return eng.match_device(sb.data_ptr(), so.data_ptr(), n, stb, sp)

    # the timed steps rotate over the engine's direct buffer sets, one stream each
    # (tm_match_device_set): step k+1's walk starts while step k's last waves finish
    K = max(1, min(3, args.in_flight))
    streams2 = [stream] + [torch.cuda.Stream(dev) for _ in range(K - 1)]

    def step2(k):
        j = (own + k) % n_slices
        if args.sequential:
            return step(j)
        sb, so, stb = slices[j]
        return eng.match_device_set(k % K, sb.data_ptr(), so.data_ptr(), n, stb, N.TM_MATCH_ALL,
                                    streams2[k % K].cuda_stream)

    # size the output arena from one run of every slice (overflow -> grow -> rerun)
    total = 0
    for j in range(n_slices):
        r = step(j)
        eng.device_sync()  # also sizes the engine's chunk pools to this batch's demand
        total = max(total, _read_u64(r.d_total))
    if total > r.keys_cap:
        eng.reserve_matches(int(total * 1.1) + 1024)
        r = step()
        torch.cuda.synchronize()
    assert total <= r.keys_cap
    for _ in range(max(0, args.warmup - 1)):
        step()
    eng.device_sync()
    if not args.sequential:  # size sets 1.. (their chunk pools, their output) the same way
        for k in range(max(K * n_slices, args.warmup)):
            step2(k)
        for x in range(K):
            eng.device_sync(x)
        for k in range(K * n_slices):
            if k % K:
                r1 = step2(k)
                eng.device_sync(k % K)
                assert _read_u64(r1.d_total) <= r1.keys_cap
    torch.cuda.synchronize()

    # walk statistics for the algorithmic-byte count: one untimed, counted run per slice (the
    # per-launch figure is their mean); per-depth counters from this rank's own slice
    walks, algs = [], []
    by_depth = None
    for j in [own] + [x for x in range(n_slices) if x != own]:
        eng.debug_stats(True, read=False)
        step(j)
        torch.cuda.synchronize()
        if by_depth is None:
            by_depth = eng.depth_stats()  # per walk depth: probes, wave cycles, frontier, round trips
        wj = dict(zip(N.Engine.STAT_NAMES, [int(x) for x in eng.debug_stats(False)]))
        walks.append(wj)
        algs.append(algorithmic_bytes(wj, slices[j][2], n))
    eng.debug_stats(False, read=False)
    walk = {k: int(round(np.mean([x[k] for x in walks]))) for k in walks[0]}
    alg_bytes = float(np.mean(algs))
    total = walk["keys"]

    # ---------------------------------------------------------------- timed region
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        sk = stream if args.sequential else streams2[k % K]
        evs[k][0].record(sk)
        step2(k)
        evs[k][1].record(sk)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    lat_ms = np.array([a.elapsed_time(b) for a, b in evs])
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_pubs = n * args.steps * world
    value = total_pubs / elapsed

    # dominant kernel (k_match_fast) duration: HIP events on its launch stream
    kms = []
    for _ in range(min(args.steps, 10)):
        eng.timing(True)
        step()
        torch.cuda.synchronize()
        kms.append(eng.timing(False))
    kernel_ms = float(np.mean(kms))
    eng.device_sync()
    slow_topics = eng.stats()["n_slow_topics"]
    # N > 1: every replica matches the master's first topics too; their per-topic route-id
    # digests must equal rank 0's (the master's own parity vs the oracle is checked at N = 1)
    replica_parity = replica_check(eng, all_b, all_o, min(20000, n), dev, backend, sp, world) if world > 1 else None

    # ---------------------------------------------------------------- one batch in flight
    # (beside the metric): the same steps on one buffer set and one stream, each batch alone on
    # the device (its latency is the kernel's), rank 0
    sequential = None
    if rank == 0 and not args.profile and not args.sequential:
        ev1 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            ev1[k][0].record(stream)
            step()
            ev1[k][1].record(stream)
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t0
        l1 = np.array([a.elapsed_time(b) for a, b in ev1])
        sequential = {"api": "tm_match_device, one stream", "publishes_per_s": round(n * args.steps / el1, 1),
                      "ms_per_step": round(el1 * 1e3 / args.steps, 4),
                      "p50_batch_ms": round(float(np.percentile(l1, 50)), 4),
                      "p99_batch_ms": round(float(np.percentile(l1, 99)), 4)}
        log(f"[rank 0] one batch in flight: {sequential['publishes_per_s'] / 1e9:.3f} G publishes/s, "
            f"{sequential['ms_per_step']} ms per step, batch p99 {sequential['p99_batch_ms']} ms")

    # ---------------------------------------------------------------- latency vs batch size
    # (not the metric: the batching window's trade-off); rank 0 only
    lat_sweep = []
    host_path = None
    host_runs = None
    batcher = None
    mode_rates = {}
    if rank == 0 and not args.profile:
        for bs in (1024, 16384, 131072):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
            tbb = int(to[bs])
            for k in range(35):
                if k >= 5:
                    ev[k - 5][0].record(stream)
                eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), bs, tbb, sp)
                if k >= 5:
                    ev[k - 5][1].record(stream)
            torch.cuda.synchronize()
            ms = np.array([a.elapsed_time(b) for a, b in ev])
            lat_sweep.append({"batch": bs, "p50_ms": round(float(np.percentile(ms, 50)), 4),
                              "p99_ms": round(float(np.percentile(ms, 99)), 4),
                              "publishes_per_s": round(bs / (float(np.mean(ms)) * 1e-3), 1)})
        # the other reducers on the same batch: return_first (k_match_first), counts only, and
        # the full walk + k_dedupe ([unique]; aggre/1)
        for mname, mode in (("first", N.TM_MATCH_FIRST), ("count", N.TM_MATCH_COUNT), ("unique", N.TM_MATCH_UNIQUE),
                            ("aggre", N.TM_MATCH_AGGRE)):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for k in range(12):
                if k >= 2:
                    ev[k - 2][0].record(stream)
                eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), n, topic_bytes, mode, sp)
                if k >= 2:
                    ev[k - 2][1].record(stream)
            torch.cuda.synchronize()
            ms = np.array([a.elapsed_time(b) for a, b in ev])
            mode_rates[mname] = {"ms_per_batch": round(float(np.mean(ms)), 4),
                                 "publishes_per_s": round(n / (float(np.mean(ms)) * 1e-3), 1)}
    if rank == 0 and world == 1 and not args.profile:
        # host buffers in, host results out (H2D + kernels + D2H of every key): PCIe-inclusive;
        # N = 1 only (the N > 1 lines carry the metric and replica parity, the host legs once)
        to32 = np.ascontiguousarray(to, dtype=np.uint32)
        eng.match_packed_view(tb, to32)
        hl = []
        for _ in range(10):
            t0 = time.perf_counter()
            eng.match_packed_view(tb, to32)
            hl.append(time.perf_counter() - t0)
        dt = float(np.mean(hl))
        host_path = {"api": "tm_match_batch", "batch": n, "ms_per_batch": round(dt * 1e3, 3),
                     "p50_ms": round(float(np.percentile(hl, 50)) * 1e3, 3),
                     "p99_ms": round(float(np.percentile(hl, 99)) * 1e3, 3),
                     "publishes_per_s": round(n / dt, 1),
                     "note": "H2D of the topics + kernels + D2H of every key + host result view; "
                             "bounded by PCIe D2H of the keys"}
        host_runs = host_runs_leg(eng, tb, to32, n, w, reps=max(10, args.steps))
        # the host-bound legs re-pick their cores first: another job may have moved onto the
        # ones picked at start-up (threads created from here on inherit the new set)
        placed_b = placement.pin_to_gpu(local) if placed.get("pinned") and args.batcher_seconds > 0 else None
        repin = (lambda: placement.pin_to_gpu(local)) if placed.get("pinned") else None
        batcher = batcher_load(eng, tb, to32, args.batcher_seconds, repin=repin) if args.batcher_seconds > 0 else None
        if batcher is not None:
            batcher["host_placement"] = placed_b
            batcher["on_replica"] = replica_batcher_leg(eng, tb, to32, args.batcher_seconds)

    # ---------------------------------------------------------------- CPU baseline + parity sample
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile and not args.quick:
        placed_c = placement.pin_to_gpu(local) if placed.get("pinned") else None
        cpu, parity = cpu_baseline(args, w, eng, tb, to, n)
        if cpu is not None and placed_c is not None:
            cpu["host_placement"] = placed_c
    # the rest of the index API on the same engine, off the headline metric
    legs = rank == 0 and world == 1 and not args.profile and not args.quick
    filt = filter_leg(args, w, eng, 20000) if legs else None
    inter = intersect_leg(w, tb, to) if legs else None
    # BASELINE.md's other per-config rows (E churn, B), and a forced full rebuild of the headline
    # index with matches running beside it (after every parity check on this engine)
    extra = legs and world == 1
    rebuild = rebuild_leg(eng, w, d_bytes, d_off, n, topic_bytes, dev) if extra else None
    churn = churn_leg("E", 1.0, 1_000_000, 5, 1) if extra else None
    cfg_b = config_leg("B", 1_000_000) if extra else None

    rss = torch.tensor([host_rss_gib()], dtype=torch.float64, device=dev if backend != "gloo" else "cpu")
    if world > 1:
        dist.all_reduce(rss, op=dist.ReduceOp.MAX)
    if rank == 0:
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        prof = profiled_traffic(w.n_keys, n)
        traffic = int(prof[1]["hbm_bytes"]) if prof else None
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "publishes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic (seeded generator, emqx_amd/workloads.py config {args.config})",
            "config": {
                "workload": f"{args.config}: {w.n_keys} route keys, 10-level topics, '#'-heavy fan-out"
                if args.config == "C" else f"{args.config} (scale {args.scale}): {w.n_keys} route keys",
                "route_keys": w.n_keys,
                "publishes_per_step_per_gpu": n,
                "matches_per_step_per_gpu": int(total),
                "distinct_batches": n_slices,
                "parallelism": f"replicated trie, dp{world}"
                               + ("" if args.sequential else ", 2 batches in flight per GPU"),
            },
            # per-batch device time from enqueue to completion on its stream; with two batches
            # in flight a batch shares the device with its neighbour (one_batch_in_flight: alone)
            "p50_batch_ms": round(float(np.percentile(lat_ms, 50)), 4),
            "p99_batch_ms": round(float(np.percentile(lat_ms, 99)), 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                # the step's kernels between the two timing events (engine.cpp prepass_on: the
                # product build launches k_prescan ahead of the walk only with EMQX_TM_PREPASS=1)
                "kernel": ("k_prescan + k_match_fast" if os.environ.get("EMQX_TM_PREPASS", "0") != "0"
                           else "k_match_fast"),
                "kernel_ms": round(kernel_ms, 4),
                # the same bytes per timed step (launch ramp and tail overlapped by the second
                # batch in flight): what the device sustains, not one launch's rate
                "achieved_per_step": round(alg_bytes / (elapsed / args.steps) / 1e9, 1),
                "frac_per_step": round(alg_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": int(alg_bytes),
                "traffic_source": (f"{os.path.relpath(prof[0], ROOT)}: FETCH_SIZE+WRITE_SIZE per launch "
                                   f"(upper bound {int(prof[1]['hbm_bytes_upper'])} if the key-arena stream "
                                   f"is tallied at half), L2 hit {prof[1]['l2_hit_rate']:.3f}")
                if prof else "no PMC profile of this kernel source under profiles/",
                "walk": walk,
                "walk_by_depth": by_depth,
            },
            "gather": gather_roof(walk, kernel_ms, 16 * int(st["edge_slots"])),
            "latency_vs_batch": lat_sweep,
            # SURVEY §8(d)'s own protocol beside the device-resident value: host topics in, spans
            # of route ids on the host out, per batch of `publishes_per_step_per_gpu`
            "end_to_end": end_to_end(host_runs, host_path),
            "host_path": host_path,
            "host_path_runs": host_runs,
            "batcher": batcher,
            "other_modes": mode_rates,
            "matches_filter": filt,
            "intersection": inter,
            "rebuild_under_load": rebuild,
            "churn_E": churn,
            "config_B": cfg_b,
            "cpu_baseline": cpu,
            "parity": parity,
            "replica_parity": replica_parity,
            "spill_topics": int(slow_topics),
            "library": {"path": os.path.relpath(N.LIB_PATH, ROOT), "src_sha": lib_sha,
                        "build_info": N.load().tm_build_info().decode()},
            "build_s": round(t_build, 2),
            "host_placement": placed,
            "batches_in_flight": 1 if args.sequential else K,
            "one_batch_in_flight": sequential,
            "host_peak_rss_gib": host_rss_gib(),
            "host_peak_rss_gib_max_over_ranks": round(float(rss.item()), 2),
            "replication": ({"mode": "one host master on rank 0, device image broadcast to replicas",
                             "image_bytes": int(eng.image_size()), "image_s": round(image_s, 2)}
                            if world > 1 else None),
        }
        emit(compact_line(out, write_detail(out)))
    if world > 1:
        dist.destroy_process_group()


def run_sharded(args):
    """Filter-hash-sharded mode: every rank holds 1/G of the route keys (generated as that
    shard only) and matches the SAME batch; a step is walk + device id compaction + RCCL
    all-gathers + device merge (emqx_amd/shard.py).  Total work is fixed as G grows
    (strong scaling); value = the batch's publishes / max-over-ranks step time."""
    import torch
    import torch.distributed as dist

    from emqx_amd import _native as N
    from emqx_amd import shard as S
    from emqx_amd import workloads

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EMQX_BENCH_BACKEND=gloo: several ranks on fewer GPUs (the exchange goes through host
    # copies, shard.py _staged); the default is RCCL, one rank per GPU
    backend = os.environ.get("EMQX_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    hdev = dev if backend != "gloo" else torch.device("cpu")  # where this group's host-side collectives run
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    t0 = time.time()
    # --shard-of G on one process: this rank holds shard 0 of a G-way split (the per-GPU
    # share of a G-GPU run) and the exchange is the identity
    nshards = args.shard_of if (args.shard_of and world == 1) else world
    w = workloads.generate(args.config, scale=args.scale, n_topics=args.batch, shard_count=nshards,
                           shard_index=rank)
    eng = N.Engine(local, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)  # already this shard's keys only
    eng.commit()
    log(f"[rank {rank}] shard {rank}/{nshards}: {w.n_keys} keys, build {time.time() - t0:.1f}s")
    six = S.ShardedIndex(S.EngineShard(eng), rank, world, exchange=args.exchange)
    n = w.n_topics
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    tb = int(w.t_off[-1])

    def timed(exchange, steps, warmup):
        """(elapsed s over `steps` steps, per-step event ms, last result) of one exchange"""
        for _ in range(max(1, warmup)):
            out = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange=exchange)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        t_start = time.perf_counter()
        for k in range(steps):  # padded: no host sync inside a step
            evs[k][0].record()
            out = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange=exchange)
            evs[k][1].record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t_start
        if world > 1:
            dist.barrier()
            t = torch.tensor([el], dtype=torch.float64, device=hdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        if int(out[2].max().item()):
            raise RuntimeError("sharded step overflowed the sizes prepare_device fixed")
        return el, [a.elapsed_time(b) for a, b in evs], out

    six.prepare_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb)  # sizes: untimed, collective
    elapsed, lat, out = timed(args.exchange, args.steps, args.warmup)
    matches = int(out[0][-1].item())
    local_total = int(six.shard.eng.stats()["n_keys"])  # keys on this rank
    # the exchange variants side by side ("report both"), shorter runs
    G = nshards
    hdr_b = (n + 2) * 4
    variants = {}
    for ex in S.EXCHANGES:
        el, lt, o = timed(ex, max(5, args.steps // 2), 2)
        m_own = int(o[0][-1].item()) if ex == "local" else None
        variants[ex] = {"ms_per_step": round(el / max(5, args.steps // 2) * 1e3, 4),
                        "publishes_per_s": round(n * max(5, args.steps // 2) / el, 1),
                        "p99_batch_ms": round(float(np.percentile(lt, 99)), 4),
                        "wire_bytes": int(six.wire_bytes)}
        if ex == "local":
            variants[ex]["own_matches"] = m_own
            variants[ex]["d2h_bytes"] = hdr_b + m_own * six.id_bytes
    own = variants["local"]["own_matches"]
    if world > 1:
        # the bytes each exchange moved into THIS rank in its last step (the sizes it sent and
        # received: ids at the wire width + headers), max over ranks
        mx = torch.tensor([variants[ex]["wire_bytes"] for ex in S.EXCHANGES], dtype=torch.int64, device=hdev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        wire = {"measured_last_step_max_over_ranks": dict(zip(S.EXCHANGES, [int(x) for x in mx.tolist()])),
                "bound_(G-1)/G*sumM*id_bytes": int((G - 1) / G * matches * six.id_bytes)}
    else:  # one rank holding 1/G: what a G-rank exchange would move into each rank
        wire = {"model": f"{G}-rank exchange from this shard's sizes (every shard assumed to match as many)",
                "padded": (G - 1) * (six.stride * six.id_bytes + hdr_b),
                "exact": (G - 1) * (own * six.id_bytes + hdr_b), "local": 0,
                "a2a": int((G - 1) / G * own * six.id_bytes) + (G - 1) * ((n // G + 1) * 4 + (G + 2) * 4),
                "bound_(G-1)/G*sumM*4": int((G - 1) / G * (G * own) * 4),
                "exact_ids_only": (G - 1) * own * six.id_bytes}
    parity = sharded_parity(six, eng, w, d_bytes, d_off, n, tb, rank, world, hdev, min(n, 2000))
    rss = torch.tensor([host_rss_gib()], dtype=torch.float64, device=hdev)
    if world > 1:
        dist.all_reduce(rss, op=dist.ReduceOp.MAX)
    if rank == 0:
        emit(json.dumps({
            "metric": f"matched publishes/sec, filters hash-sharded over {nshards} GPU shard(s) (config {args.config})",
            "value": round(n * args.steps / elapsed, 1), "unit": "publishes/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u32",
            "data": f"synthetic (seeded generator, emqx_amd/workloads.py config {args.config}, scale {args.scale})",
            "config": {"workload": f"{args.config} filter-sharded {nshards} ways over {world} rank(s): "
                                   f"{local_total} keys on rank 0",
                       "publishes_per_step": n, "matches_per_step": matches,
                       "parallelism": f"filter hash-shard x{world}, exchange {args.exchange}"},
            "p50_batch_ms": round(float(np.percentile(lat, 50)), 4),
            "p99_batch_ms": round(float(np.percentile(lat, 99)), 4),
            "id_bytes_on_wire": six.id_bytes, "stride_ids": six.stride,
            "wire_bytes_per_rank": wire, "exchanges": variants, "parity": parity,
            "host_peak_rss_gib_max_over_ranks": round(float(rss.item()), 2),
            "backend": backend if world > 1 else None,
        }))
    if world > 1:
        dist.destroy_process_group()


def sharded_parity(six, eng, w, d_bytes, d_off, n, tb, rank, world, hdev, ps):
    """Parity of the sharded step on the first `ps` topics, in two parts that together pin it:
    (1) each rank's own shard lists (the walk through the same C-ABI, host form) equal the
    oracle over THAT shard's keys (w holds only this rank's keys); (2) the merged result of the
    padded step equals, per topic, the union of every rank's shard lists (count and the sum of
    a hash of the ids, all-gathered).  Shards are disjoint, so (1) + (2) = the unsharded set."""
    import torch
    import torch.distributed as dist
    import oracle
    tsub = np.ascontiguousarray(w.t_off[:ps + 1])
    roff, rids, rst = six.shard.match_ids(w.t_bytes, tsub)
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    eo, eids, est = ix.match(w.t_bytes, tsub, threads=8)
    bad_local = int(np.sum(rst != est))
    for t in range(ps):
        if not np.array_equal(np.sort(rids[roff[t]:roff[t + 1]]), eids[eo[t]:eo[t + 1]]):
            bad_local += 1

    def digest(off, ids):
        h = (ids.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(16)
        cs = np.zeros(len(ids) + 1, np.uint64)
        np.cumsum(h, out=cs[1:])
        o = off.astype(np.int64)
        return np.diff(o), (cs[o[1:]] - cs[o[:-1]]).view(np.int64)

    c_loc, h_loc = digest(np.asarray(roff, np.int64), np.asarray(rids, np.uint64))
    loc = torch.from_numpy(np.stack([c_loc, h_loc])).to(hdev)
    if world > 1:
        dist.all_reduce(loc)  # per topic: ids and hash sums over all shards (wrapping add)
    off, ids, flags = six.match_device(eng, d_bytes.data_ptr(), d_off.data_ptr(), n, tb, exchange="padded")
    torch.cuda.synchronize()
    o = off[:ps + 1].cpu().numpy().view(np.uint32).astype(np.int64)
    m = ids[:int(o[-1])].cpu().numpy().view(np.uint64)
    c_m, h_m = digest(o - o[0], m[o[0]:])
    lc = loc.cpu().numpy()
    bad_merged = int(np.sum((c_m != lc[0]) | (h_m != lc[1]))) + (1 if int(flags.max().item()) else 0)
    bad = torch.tensor([bad_local, bad_merged], dtype=torch.int64, device=hdev)
    if world > 1:
        dist.all_reduce(bad)
    return {"sampled_topics": ps, "shard_lists_vs_oracle_mismatches": int(bad[0].item()),
            "merged_vs_union_of_shards_mismatches": int(bad[1].item()),
            "oracle": "oracle/trie_search.cpp over each rank's shard keys",
            "compared": "per topic: each shard's sorted ids vs the oracle; merged (padded) step vs the union of "
                        "shards by count + hash sum"}


def _new_filter(f, n):
    """A new, VALID filter near f (emqx_topic:validate/1 rejects a '#' that is not the last
    level, emqx_topic.erl:206-207): one more level, inserted before a trailing '#'."""
    if f == b"#":
        return b"n%d/#" % n
    if f.endswith(b"/#"):
        return f[:-2] + b"/n%d/#" % n
    return f + b"/n%d" % n


def run_churn(args):
    """--churn EPOCHS: the churn leg alone, as its own JSON line."""
    cfg = args.config if args.config != "C" else "E"
    r = churn_leg(cfg, args.scale, args.batch, args.churn, args.warmup)
    emit(json.dumps(dict({"metric": "delta-epoch churn: route ops/s committed + matched publishes/s between epochs"},
                          **r)))


def churn_leg(cfg, scale, batch, epochs, warmup):
    """Live subscribe/unsubscribe churn (BASELINE configs[4]): every epoch deletes 1% of the
    live route keys and adds 1% new ones (half are new dests on existing filters, like a
    $share group joining: emqx_shared_sub.erl:450; half new filter strings), commits them as
    one delta epoch (tm_commit_epoch: host trie update + stream-ordered device patch), then
    matches a batch.  Rank 0, one GPU.  The last epoch is checked against the oracle on a
    sample of the batch."""
    import torch

    from emqx_amd import _native as N
    from emqx_amd import workloads
    w = workloads.generate(cfg, scale=scale, n_topics=batch)
    dev = torch.device("cuda", 0)
    eng = N.Engine(0, reserve_keys=w.n_keys * 2, reserve_nodes=w.n_keys * 8)
    t0 = time.time()
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    t_build = time.time() - t0
    n = w.n_topics
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)
    stream = torch.cuda.Stream(dev)
    sp = stream.cuda_stream
    rng = np.random.default_rng(0xE11A0005)
    # live key set as packed arrays: (filter bytes list, ids)
    fl = w.filters()
    live_f = list(fl)
    live_id = w.f_id.astype(np.uint64).copy()
    next_id = int(live_id.max()) + 1
    commit_ms, match_ms, nops, phases, full_eps = [], [], [], [], []
    reruns = 0

    def pack(fs, ids):
        off = np.zeros(len(fs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(f) for f in fs])
        return np.frombuffer(b"".join(fs) + b"\0" * 16, dtype=np.uint8), off, np.asarray(ids, dtype=np.uint64)

    r = eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), sp)
    eng.device_sync()
    tot = _read_u64(r.d_total)
    eng.reserve_matches(int(tot * 1.5) + 1024)
    for ep in range(warmup + epochs):
        k = max(1, len(live_id) // 100)
        dsel = rng.choice(len(live_id), size=k, replace=False)
        keep = np.ones(len(live_id), dtype=bool)
        keep[dsel] = False
        del_f = [live_f[i] for i in dsel]
        del_id = live_id[dsel]
        src = rng.integers(0, len(fl), size=k)
        add_f = [fl[j] if (i & 1) else _new_filter(fl[j], next_id + i) for i, j in enumerate(src)]
        add_id = np.arange(next_id, next_id + k, dtype=np.uint64)
        next_id += k
        db, do, di = pack(del_f, del_id)
        ab, ao, ai = pack(add_f, add_id)
        torch.cuda.synchronize()
        n_full_before = int(eng.stats()["n_full_rebuilds"])
        t0 = time.perf_counter()
        eng.apply_packed(N.TM_OP_DEL, db, do, di)
        eng.apply_packed(N.TM_OP_ADD, ab, ao, ai)
        eng.commit()
        t1 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r = eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), sp)
        e1.record(stream)
        eng.device_sync()
        torch.cuda.synchronize()
        got = _read_u64(r.d_total)
        if got > r.keys_cap:
            # the walk counts what it could not store: size the arena to it and run the batch
            # again (the timed match is the first run; the rerun is counted in the line)
            log(f"churn epoch {ep}: {got} matched keys > output arena {r.keys_cap} (first batch: {tot}); re-run")
            reruns += 1
            eng.reserve_matches(int(got * 1.25) + 1024)
            r = eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), n, int(w.t_off[-1]), sp)
            eng.device_sync()
            torch.cuda.synchronize()
            if _read_u64(r.d_total) > r.keys_cap:
                raise RuntimeError("output arena overflow during churn bench")
        live_f = [f for f, kk in zip(live_f, keep) if kk] + add_f
        live_id = np.concatenate([live_id[keep], add_id])
        if ep >= warmup:
            cs = eng.stats()
            full_eps.append(int(cs["n_full_rebuilds"]) > n_full_before)
            phases.append((cs["commit_apply_us"], cs["commit_lists_us"], cs["commit_upload_us"], cs["commit_stall_us"]))
            commit_ms.append((t1 - t0) * 1e3)
            match_ms.append(e0.elapsed_time(e1))
            nops.append(2 * k)
    # parity of the last epoch on a sample
    import oracle
    ps = min(n, 20000)
    lb, lo, li = pack(live_f, live_id)
    ix = oracle.OrderedIndex(lb, lo, li)
    eo, eids, _ = ix.match(w.t_bytes, w.t_off[:ps + 1], threads=16)
    off, cnt, keys, _ = eng.match_packed(w.t_bytes, w.t_off[:ps + 1])
    ids = eng.key_ids(keys)
    bad = sum(not np.array_equal(np.sort(ids[off[i]:off[i] + cnt[i]]), eids[eo[i]:eo[i + 1]]) for i in range(ps))
    st = eng.stats()
    eng.close()
    return {
        "config": {"workload": f"{cfg} (scale {scale}): {w.n_keys} initial route keys, 1% adds + 1% deletes "
                               f"per epoch", "publishes_per_batch": n},
        "epochs": epochs, "ops_per_epoch": int(np.mean(nops)),
        "commit_ms_p50": round(float(np.percentile(commit_ms, 50)), 3),
        "commit_ms_p99": round(float(np.percentile(commit_ms, 99)), 3),
        "commit_stall_ms_p50": round(float(np.percentile([x[3] for x in phases], 50)) / 1e3, 3),
        "commit_phase_ms_p50": dict(zip(("apply", "lists", "upload"),
                                        (round(float(x) / 1e3, 3)
                                         for x in np.percentile(np.array(phases)[:, :3], 50, axis=0)))),
        "route_ops_per_s": round(float(np.sum(nops) / (np.sum(commit_ms) * 1e-3)), 1),
        "match_ms_p50": round(float(np.percentile(match_ms, 50)), 4),
        "publishes_per_s_incl_commit": round(n * len(match_ms) / ((np.sum(match_ms) + np.sum(commit_ms)) * 1e-3), 1),
        "full_rebuilds": st["n_full_rebuilds"], "delta_commits": st["n_delta_commits"],
        "commit_ms_per_epoch": [round(x, 2) for x in commit_ms],
        "commit_phase_ms_per_epoch": [[round(x / 1e3, 2) for x in ph[:3]] for ph in phases],
        "full_rebuild_epochs": [i for i, f in enumerate(full_eps) if f],
        "match_reruns": reruns,
        "build_s": round(t_build, 2),
        "host_peak_rss_gib": host_rss_gib(),
        "parity": {"sampled_topics": ps, "mismatches": int(bad), "oracle": "oracle/trie_search.cpp"},
    }


def config_leg(cfg, batch, steps=20):
    """BASELINE.md's per-config row for another config on one GPU: device-resident batches of
    `batch` publishes (tm_match_device), p50/p99 batch latency, k_match_fast time, HBM bytes
    (algorithmic), the runs host path, and a 20,000-topic parity sample vs the oracle."""
    import torch

    from emqx_amd import _native as N
    from emqx_amd import workloads
    t0 = time.time()
    w = workloads.generate(cfg, n_topics=batch)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    t_build = time.time() - t0
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sp = stream.cuda_stream
    n = w.n_topics
    tbytes = int(w.t_off[-1])
    d_bytes = torch.from_numpy(w.t_bytes).to(dev)
    d_off = torch.from_numpy(w.t_off.view(np.int32)).to(dev)

    def step():
        return eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), n, tbytes, sp)

    r = step()
    eng.device_sync()
    total = _read_u64(r.d_total)
    if total > r.keys_cap:
        eng.reserve_matches(int(total * 1.1) + 1024)
        step()
        eng.device_sync()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    eng.debug_stats(True, read=False)
    step()
    torch.cuda.synchronize()
    by_depth = eng.depth_stats()  # per walk depth: probes, wave cycles, frontier, round trips
    walk = dict(zip(N.Engine.STAT_NAMES, [int(x) for x in eng.debug_stats(False)]))
    eng.debug_stats(False, read=False)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lat = [a.elapsed_time(b) for a, b in evs]
    kms = []
    for _ in range(5):
        eng.timing(True)
        step()
        torch.cuda.synchronize()
        kms.append(eng.timing(False))
    kernel_ms = float(np.mean(kms))
    alg = algorithmic_bytes(walk, tbytes, n)
    to32 = np.ascontiguousarray(w.t_off, dtype=np.uint32)
    runs = host_runs_leg(eng, w.t_bytes, to32, n, w, reps=5)
    eng.close()
    return {"config": {"workload": f"{cfg}: {w.n_keys} route keys", "route_keys": w.n_keys, "publishes_per_batch": n,
                       "matches_per_batch": int(walk["keys"])},
            "publishes_per_s": round(n * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 4),
            "p50_batch_ms": round(float(np.percentile(lat, 50)), 4),
            "p99_batch_ms": round(float(np.percentile(lat, 99)), 4),
            "kernel_ms": round(kernel_ms, 4), "kernel_publishes_per_s": round(n / (kernel_ms * 1e-3), 1),
            "roofline": {"bound": "hbm", "achieved": round(alg / (kernel_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": int(alg)},
            "host_path_runs": {k: runs[k] for k in ("pinned", "pageable", "pinned_read_every_id", "parity")},
            "build_s": round(t_build, 2)}


def rebuild_leg(eng, w, d_bytes, d_off, n, topic_bytes, dev, frac=0.13):
    """A forced FULL rebuild at the headline scale, with matches running beside it: one epoch
    deletes `frac` of the route keys and re-adds the same keys (last op per key wins, so the key
    set is unchanged but 2 x frac of it are deltas: past n_live / 8, a full rebuild: every list
    rebuilt, the whole index uploaded into a standby image, then swapped).  A second thread keeps
    matching batches of 131,072 publishes on its own stream; their latency during the commit,
    against before it, is the stall the match path sees (plus tm_stats.commit_stall_us: how long
    the swap held matches back).  A compaction takes the same path."""
    import threading

    import torch

    from emqx_amd import _native as N
    rng = np.random.default_rng(0xB1D)
    k = int(len(w.f_id) * frac)
    sel = np.sort(rng.choice(len(w.f_id), size=k, replace=False))
    lens = (w.f_off[sel + 1] - w.f_off[sel]).astype(np.uint64)
    off = np.zeros(k + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    idx = np.concatenate([np.arange(int(w.f_off[j]), int(w.f_off[j + 1])) for j in sel]) if k else np.zeros(0, np.int64)
    fb = np.ascontiguousarray(w.f_bytes[idx])
    ids = np.ascontiguousarray(w.f_id[sel])
    s2 = torch.cuda.Stream(dev)
    m = min(n, 131072)
    lat = []
    stop = threading.Event()

    def matcher():
        while not stop.is_set():
            t0 = time.monotonic()  # CLOCK_MONOTONIC, as the engine's commit marks
            eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), m, int(topic_bytes_m), s2.cuda_stream)
            s2.synchronize()
            lat.append((t0, time.monotonic() - t0))

    import gc
    gc_was = gc.isenabled()
    gc.disable()  # no collector pauses in the matcher's timings
    topic_bytes_m = int(d_off[m].item())
    th = threading.Thread(target=matcher)
    th.start()
    time.sleep(0.5)
    n_full0 = eng.stats()["n_full_rebuilds"]
    cg0 = cgroup_cpu_stat()
    t0 = time.monotonic()
    eng.apply_packed(N.TM_OP_DEL, fb, off, ids)
    eng.apply_packed(N.TM_OP_ADD, fb, off, ids)
    eng.commit()
    t1 = time.monotonic()
    cg1 = cgroup_cpu_stat()
    time.sleep(0.3)
    stop.set()
    th.join()
    if gc_was:
        gc.enable()
    st = eng.stats()
    marks = eng.commit_marks()
    steps = [(k, v) for k, v in marks.items() if k != "reallocs" and v]

    def phase(t):  # the publish step running at time t (or the host phases before the upload)
        cur = "apply+lists" if t >= t0 else "before"
        for k, v in steps:
            if t >= v:
                cur = k
        return cur if t <= t1 else "after"

    before = [d for t, d in lat if t < t0]
    during = [d for t, d in lat if t0 <= t < t1]
    worst = max(((d, t) for t, d in lat if t0 <= t < t1), default=None)
    slow = sorted(((d, t) for t, d in lat if t0 <= t < t1), reverse=True)[:4]
    return {"ops": 2 * k, "full_rebuild": int(st["n_full_rebuilds"]) > int(n_full0),
            "commit_s": round(t1 - t0, 3),
            "commit_phase_s": {"apply": round(st["commit_apply_us"] / 1e6, 3),
                               "lists": round(st["commit_lists_us"] / 1e6, 3),
                               "upload_standby": round(st["commit_upload_us"] / 1e6, 3)},
            "matches_held_back_ms": round(st["commit_stall_us"] / 1e3, 3),
            "concurrent_match_batch": m,
            "concurrent_batches_during_commit": len(during),
            "match_ms_before": {"p50": round(float(np.percentile(before, 50)) * 1e3, 3) if before else None,
                                "max": round(float(np.max(before)) * 1e3, 3) if before else None},
            "match_ms_during_commit": {"p50": round(float(np.percentile(during, 50)) * 1e3, 3) if during else None,
                                       "p99": round(float(np.percentile(during, 99)) * 1e3, 3) if during else None,
                                       "max": round(float(np.max(during)) * 1e3, 3) if during else None},
            "max_at_ms": round((worst[1] - t0) * 1e3, 1) if worst else None,
            # the publish's steps (ms from the commit call) and the slowest matches beside them,
            # each with the step running when it started and when it ended
            "publish_steps_ms": {k: round((v - t0) * 1e3, 1) for k, v in steps},
            "publish_reallocs": marks["reallocs"],
            "slowest_matches": [{"ms": round(d * 1e3, 3), "at_ms": round((t - t0) * 1e3, 1),
                                 "step_at_start": phase(t), "step_at_end": phase(t + d)} for d, t in slow],
            "cgroup_during_commit": cgroup_delta(cg0, cg1),
            "note": "one epoch re-keys a share of the route keys (deleted and re-added: the same key set, all of them "
                    "deltas) so the commit takes the full-rebuild path; the index is uploaded into a standby device "
                    "image while the second thread keeps matching; match latency is wall time per batch incl. "
                    "the host call"}


def replica_check(eng, all_b, all_o, s, dev, backend, sp, world):
    """Collective: match topics [0, s) of the whole batch on every rank and compare each
    rank's per-topic (count, sum of a hash of the route ids) with rank 0's."""
    import torch
    import torch.distributed as dist
    d_off = all_o[:s + 1].contiguous()
    r = eng.match_device(all_b.data_ptr(), d_off.data_ptr(), s, int(all_o[s].item()), sp)
    eng.device_sync()
    total = _read_u64(r.d_total)
    if total > r.keys_cap:
        raise RuntimeError("replica check: output arena overflow")
    ids = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    off = torch.empty(s + 1, dtype=torch.int32, device=dev)
    eng.result_ids_device(ids.data_ptr(), ids.numel(), off.data_ptr(), sp)
    eng.device_sync()
    torch.cuda.synchronize()
    o = off.long() & 0xFFFFFFFF
    h = (ids[:total] * 0x9E3779B97F4A7C15) >> 16
    cs = torch.zeros(total + 1, dtype=torch.int64, device=dev)
    cs[1:] = torch.cumsum(h, 0)
    dig = torch.stack([o[1:] - o[:-1], cs[o[1:]] - cs[o[:-1]]])
    if backend == "gloo":
        dig = dig.cpu()
    got = [torch.empty_like(dig) for _ in range(world)]
    dist.all_gather(got, dig)
    return {"sampled_topics": s, "ranks": world, "matched_keys": int(o[-1].item()),
            "ranks_differing_from_master": [i for i, g in enumerate(got) if not torch.equal(g, got[0])],
            "compared": "per topic: route-id count and the sum of a hash of the ids"}


def _read_u64(ptr):
    """Read one u64 from device memory (the batch's requested-keys counter)."""
    import ctypes as C

    import torch
    h = torch.empty(1, dtype=torch.int64)
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    rc = lib.hipMemcpy(C.c_void_p(h.data_ptr()), C.c_void_p(ptr), 8, 2)  # hipMemcpyDeviceToHost
    assert rc == 0, rc
    return int(h.item())


_ORACLE_IX = {}


def oracle_index(w):
    """The oracle's ordered key set for workload w, built once per run (checker / CPU
    baseline only)."""
    import oracle
    if id(w) not in _ORACLE_IX:
        _ORACLE_IX[id(w)] = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    return _ORACLE_IX[id(w)]


def filter_queries(w, q, seed=0xF11, kinds=None):
    """Q topic filters from the workload's own filters: a third as stored, a third with one
    level turned '+', a third cut to a deep prefix (at most 2 levels off) + '#' (valid
    filters: '#' only last; shallow '#' queries would return most of the index)."""
    rng = np.random.default_rng(seed)
    nf = len(w.f_id)
    pick = rng.integers(0, nf, q)
    kind = rng.integers(0, 3, q)
    if kinds:  # development: only these query kinds (0 stored, 1 one '+', 2 prefix + '#')
        keep = np.isin(kind, kinds)
        pick, kind = pick[keep], kind[keep]
        q = len(pick)
    out = []
    for j, k in zip(pick, kind):
        ws = bytes(w.f_bytes[w.f_off[j]:w.f_off[j + 1]]).split(b"/")
        if ws[-1] == b"#":
            ws = ws[:-1] or [b"a"]
        if k == 1:
            ws[int(rng.integers(0, len(ws)))] = b"+"
        elif k == 2:
            ws = ws[:int(rng.integers(max(1, len(ws) - 2), len(ws) + 1))] + [b"#"]
        out.append(b"/".join(ws))
    off = np.zeros(q + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in out])
    return np.frombuffer(b"".join(out) + b"\0", dtype=np.uint8), off


def filter_leg(args, w, eng, q):
    """matches_filter/3 on the loaded engine: q topic-filter queries made from
    the workload's filters, walked on the GPU (filter_kernels.hip) through
    tm_match_filter_batch end to end (H2D of the queries, count walk, scan, emit walk, D2H)
    after the per-epoch index build; the oracle's restatement (oracle/trie_search.cpp
    ALGO_FILTER) timed on the same queries; walk order compared on a sample."""
    import oracle
    qb, qo = filter_queries(w, q, kinds=[int(x) for x in args.filter_kinds.split(",")] if args.filter_kinds else None)
    qo = np.ascontiguousarray(qo, dtype=np.uint32)
    q = len(qo) - 1  # --filter-kinds keeps only the chosen kinds' share of the queries
    t0 = time.perf_counter()
    eng.match_filter_view(qb, qo[:2])  # first call after the commit builds the index
    t_index = time.perf_counter() - t0
    for _ in range(args.warmup):
        eng.match_filter_view(qb, qo)
    ts = []
    for _ in range(max(1, min(args.steps, 20))):
        t0 = time.perf_counter()
        eng.match_filter_view(qb, qo)  # the C-ABI call: host result view, no Python copies
        ts.append(time.perf_counter() - t0)
    dt = float(np.mean(ts))
    o, c, k, st = eng.match_filter_packed(qb, qo)
    total = int(c.sum())
    threads = args.cpu_threads or cpu_topology()["usable_cpus"]
    ix = oracle_index(w)
    t0 = time.perf_counter()
    ix.count(qb, qo, algo=oracle.ALGO_FILTER, threads=threads)
    dt_cpu = time.perf_counter() - t0
    ps = min(q, 20000)
    eo, eids, est, src = ix.match(qb, qo[:ps + 1], algo=oracle.ALGO_FILTER, with_src=True)
    eng_ids = eng.key_ids(k) if len(k) else np.zeros(0, np.uint64)  # ranges are in any order
    bad = 0
    for i in range(ps):
        if not np.array_equal(eng_ids[o[i]:o[i] + c[i]], w.f_id[src[eo[i]:eo[i + 1]]]):
            bad += 1
    if bad:
        log(f"PARITY FAILURE (matches_filter): {bad}/{ps} queries differ")
    # the runs form: the walk's ranges cross PCIe and become spans of the sorted key ids
    import ctypes as C
    lg = _loadgen()
    for _ in range(args.warmup):
        eng.match_filter_runs_view(qb, qo)
    tr, trr = [], []
    for _ in range(max(1, min(args.steps, 20))):
        t0 = time.perf_counter()
        res = eng.match_filter_runs_view(qb, qo)
        tr.append(time.perf_counter() - t0)
        lg.spans_checksum(C.byref(res), 8)
        trr.append(time.perf_counter() - t0)
    dtr, dtrr = float(np.mean(tr)), float(np.mean(trr))
    spans = int(res.total_spans)
    ro, rids, rk, rst = eng.match_filter_runs(qb, qo[:ps + 1])
    bad_r = int(np.sum(rst != st[:ps]))
    for i in range(ps):
        if not np.array_equal(rids[ro[i]:ro[i + 1]], eng_ids[o[i]:o[i] + c[i]]):
            bad_r += 1
    if bad_r:
        log(f"PARITY FAILURE (matches_filter runs): {bad_r}/{ps} queries differ")
    return {
        "api": "tm_match_filter_batch (matches_filter/3)", "queries": q,
        "query_mix": "stored filters / one level '+' / deep prefix + '#', a third each",
        "queries_per_s": round(q / dt, 1), "ms_per_batch": round(dt * 1e3, 3), "keys_returned": total,
        "runs_form": {"api": "tm_match_filter_batch_runs", "queries_per_s": round(q / dtr, 1),
                      "ms_per_batch": round(dtr * 1e3, 3), "spans": spans, "d2h_bytes": spans * 8 + 12 * q,
                      "read_every_id": {"ms_per_batch": round(dtrr * 1e3, 3), "queries_per_s": round(q / dtrr, 1),
                                        "threads": 8},
                      "parity": {"sampled_queries": ps, "mismatches": bad_r,
                                 "compared": "ids in walk order vs the keys form's"}},
        "index_build_ms": round(t_index * 1e3, 1),
        "cpu_baseline": {"value": round(q / dt_cpu, 1), "unit": "queries/s", "cores": threads, "kind": "port",
                         "sample": f"all {q} queries, oracle/trie_search.cpp ALGO_FILTER, counts only"},
        "parity": {"sampled_queries": ps, "mismatches": bad, "compared": "key ids in walk order"},
    }


def _gather_bytes(buf, starts, lens):
    """Concatenate buf[starts[i]: starts[i] + lens[i]] for lens[i] > 0 (vectorised)."""
    lens = np.where(lens > 0, lens, 0).astype(np.int64)
    tot = int(lens.sum())
    if not tot:
        return np.zeros(0, np.uint8)
    cs = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=cs[1:])
    idx = np.repeat(starts.astype(np.int64) - cs[:-1], lens) + np.arange(tot, dtype=np.int64)
    return buf[idx]


def intersect_leg(w, tb, to, n_pairs=1_000_000, threads=0):
    """emqx_topic:intersection/2 batched on the GPU (tm_intersect_batch,
    k_intersect): n_pairs (filter, generalised filter or topic) pairs from the workload, end to end
    through the C-ABI.  CPU baseline: oracle/trie_search.cpp's C++ restatement
    (ots_intersect) on the box's job share of CPUs over the SAME pairs, and the whole batch
    compared with it (lengths, false / badhash, bytes)."""
    import oracle
    from emqx_amd import _native as N
    threads = threads or cpu_topology()["usable_cpus"]
    rng = np.random.default_rng(0x1A7)
    nf, nt = len(w.f_id), len(to) - 1
    fi = rng.integers(0, nf, n_pairs)
    ti = rng.integers(0, nt, n_pairs)
    use_f = rng.random(n_pairs) < 0.5
    fbytes = [bytes(w.f_bytes[w.f_off[j]:w.f_off[j + 1]]) for j in fi]
    cut = rng.integers(0, 1 << 30, n_pairs)

    def variant(f, r):  # the same filter generalised: one level '+', or a prefix + '#'
        ws = f.split(b"/")
        if r & 1:
            ws[(r >> 1) % len(ws)] = b"+"
        else:
            ws = ws[:(r >> 1) % len(ws)] + [b"#"]
        return b"/".join(ws)

    # half the pairs: a filter and a variant of it (mostly intersecting); half: a filter
    # and a topic of the batch
    other = [variant(f, int(r)) if u else bytes(tb[to[k]:to[k + 1]])
             for f, r, k, u in zip(fbytes, cut, ti, use_f)]
    a_buf, a_off = N.pack_topics(fbytes)
    b_buf, b_off = N.pack_topics(other)
    del fbytes, other
    eng = N.Engine(0)
    res = N.tm_intersect_result()
    ts = []
    for k in range(6):
        t0 = time.perf_counter()
        eng._check(eng.lib.tm_intersect_batch(eng.h, a_buf.ctypes.data, a_off.ctypes.data, b_buf.ctypes.data,
                                              b_off.ctypes.data, n_pairs, N.C.byref(res)))
        if k:
            ts.append(time.perf_counter() - t0)
    dt = float(np.mean(ts))
    g_off = np.ctypeslib.as_array(res.off, shape=(n_pairs,)).copy()
    g_len = np.ctypeslib.as_array(res.len, shape=(n_pairs,)).copy()
    cap = int(g_off[-1]) + max(int(g_len[-1]), 0)
    g_raw = np.ctypeslib.as_array(res.bytes, shape=(max(cap, 1),)).copy()
    cts = []
    for _ in range(3):
        t0 = time.perf_counter()
        c_len, c_start, c_raw = oracle.intersect_packed(a_buf, a_off, b_buf, b_off, threads=threads)
        cts.append(time.perf_counter() - t0)
    dt_cpu = float(np.median(cts))
    t0 = time.perf_counter()
    oracle.intersect_packed(a_buf, a_off[:100_001], b_buf, b_off[:100_001], threads=1)
    dt_cpu1 = (time.perf_counter() - t0) * n_pairs / 100_000
    g_code = np.where(g_len == N.TM_INTERSECT_FALSE, oracle.INTERSECT_FALSE,
                      np.where(g_len == N.TM_INTERSECT_BADHASH, oracle.INTERSECT_BADHASH, g_len))
    bad_len = np.nonzero(g_code != c_len)[0]
    same_bytes = bool(np.array_equal(_gather_bytes(g_raw, g_off, g_len), _gather_bytes(c_raw, c_start, c_len)))
    eng.close()
    return {"api": "tm_intersect_batch (intersection/2)", "pairs": n_pairs, "pairs_per_s": round(n_pairs / dt, 1),
            "ms_per_batch": round(dt * 1e3, 3), "non_false": int((g_len != N.TM_INTERSECT_FALSE).sum()),
            "cpu_baseline": {"value": round(n_pairs / dt_cpu, 1), "unit": "pairs/s", "cores": threads,
                             "kind": "port", "value_1_thread": round(n_pairs / dt_cpu1, 1),
                             "sample": f"all {n_pairs} pairs, oracle/trie_search.cpp ots_intersect (C++ restatement "
                                       f"of emqx_topic:intersection/2 + join/1), {threads} threads, median of 3; "
                                       f"1 thread timed on the first 100,000 pairs"},
            "note": "through the C-ABI from host buffers: H2D of both sides + kernel + D2H of the results",
            "parity": {"compared_pairs": n_pairs, "mismatches": int(len(bad_len)) + (0 if same_bytes or len(bad_len)
                                                                                       else 1),
                       "checker": "oracle/trie_search.cpp ots_intersect, pinned by the 17 reference KATs"}}


def run_filter(args):
    """--filter-search Q: the matches_filter/3 leg alone, as its own JSON line."""
    from emqx_amd import _native as N
    from emqx_amd import workloads
    w = workloads.generate(args.config, scale=args.scale, n_topics=1000)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    r = filter_leg(args, w, eng, args.filter_search)
    emit(json.dumps({
        "metric": "matches_filter/3 topic-filter queries/s (host API, walk-order exact)",
        "value": r["queries_per_s"], "unit": "queries/s", "n_gpus": 1,
        "config": {"workload": f"{args.config}: {w.n_keys} route keys", "queries": r["queries"],
                   "query_mix": r["query_mix"]},
        "ms_per_batch": r["ms_per_batch"], "keys_returned": r["keys_returned"],
        "index_build_ms": r["index_build_ms"], "cpu_baseline": r["cpu_baseline"], "parity": r["parity"],
    }))


def cpu_baseline(args, w, eng, tb, to, n):
    """Time oracle/'s emqx_trie_search restatement on a bounded sample of the same
    batch, and check the engine's results for that sample bit-exactly."""
    import oracle
    from emqx_amd import _native as N
    topo = cpu_topology()
    threads = args.cpu_threads or topo["usable_cpus"]
    t0 = time.time()
    ix = oracle_index(w)
    t_build = time.time() - t0
    # calibrate: rate on a small slice, then size the sample for ~cpu_seconds
    cal = 2000
    t0 = time.perf_counter()
    ix.count(tb, to[:cal + 1], threads=threads)
    rate = cal / max(time.perf_counter() - t0, 1e-6)
    m = int(min(n, max(cal, rate * args.cpu_seconds)))
    t0 = time.perf_counter()
    passes, done = 0, 0
    while True:  # whole passes over the first m publishes until ~cpu_seconds have elapsed
        ix.count(tb, to[:m + 1], threads=threads)
        passes += 1
        done += m
        if time.perf_counter() - t0 >= 0.8 * args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    # single-thread reference point
    m1 = int(min(m, max(4000, rate / threads * 2.0)))
    t0 = time.perf_counter()
    ix.count(tb, to[:m1 + 1], threads=1)
    dt1 = time.perf_counter() - t0
    # parity on a sample of the batch (host path through the same C-ABI)
    ps = min(m, 20000)
    eo, eids, est = ix.match(tb, to[:ps + 1], threads=threads)
    buf = tb
    off, cnt, keys, st = eng.match_packed(buf, to[:ps + 1])
    ids = eng.key_ids(keys)
    bad = 0
    for i in range(ps):
        if not np.array_equal(np.sort(ids[off[i]:off[i] + cnt[i]]), eids[eo[i]:eo[i + 1]]):
            bad += 1
    cpu = {
        "value": round(done / dt, 1),
        "unit": "publishes/s",
        "cores": threads,
        "kind": "port",
        "host": dict(topo, model=cpu_info(), threads_used=threads),
        "value_1_thread": round(m1 / dt1, 1),
        "sample": f"{passes} pass(es) over {m} publishes ({dt:.1f} s) of the same batch vs the same {w.n_keys} keys; C++ restatement of "
                  f"emqx_trie_search over an Erlang-term-ordered key set (oracle/trie_search.cpp), "
                  f"{threads} threads on {cpu_info()}; 1 thread: {round(m1 / dt1, 1)} publishes/s "
                  f"({m1} publishes); "
                  f"index build {t_build:.1f}s untimed",
    }
    parity = {"sampled_topics": ps, "mismatches": bad, "oracle": "oracle/trie_search.cpp (emqx_trie_search)",
              "matches_in_sample": int(eo[-1])}
    if bad:
        log(f"PARITY FAILURE: {bad}/{ps} topics differ")
    return cpu, parity


if __name__ == "__main__":
    main()
