"""Kernel-parameter sweep on one GPU (development tool, not the product or the bench).

    python tools/sweep.py build                      # here: compile the variants (hipcc, gfx950)
    python tools/sweep.py run [--config C] [...]     # on the GPU box: time every variant

Each variant is the same engine.cpp + kernels compiled with different -D knobs into
emqx_amd/variants/libemqx_tm_<name>.so (git-ignored, travels to the box like the product
.so), optionally with a different edge-table load (tm_config.edge_load_inv).  The workload
is generated once; every variant builds its own index, runs warm-up + timed batches through
tm_match_device and reports the k_match_fast time (HIP events on its stream), the batch
time and the walk counters.  Results are checked against the product build's key counts.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "emqx_amd", "variants")
CSRC = os.path.join(ROOT, "emqx_amd", "csrc")

# name -> (extra hipcc flags, edge_load_inv[, topics_per_wave])
# "head": the committed match_kernels.hip (git HEAD) with the working tree's engine, as the
# same-process reference point.
VARIANTS = {
    "head": ([], 0),  # match_kernels.hip as committed (git HEAD)
    "prev": ([], 0),
    "ntd2": (["-DTM_NT_DEPTH=2"], 0),
    "ntd3": (["-DTM_NT_DEPTH=3"], 0),
    "ntd4": (["-DTM_NT_DEPTH=4"], 0),  # match_kernels.hip at SWEEP_PREV (default af8ba73: before the fused-id copy-out)
    "base": ([], 0),
    "base2": ([], 0),  # the same build again: run-to-run noise and the digest's self-check
    "nopre": (["-DTM_PRELOOK=0"], 0),
    "nodpp": (["-DTM_DPP_SCAN=0"], 0),
    "alive": (["-DTM_ALIVE_REG=1"], 0),
    "rpl3": (["-DTM_RPL=3"], 0),
    "tb2048_f384": (["-DTM_TBCAP=2048", "-DTM_FCAP=384"], 0),
    "tb2048_f352": (["-DTM_TBCAP=2048", "-DTM_FCAP=352"], 0),
    "alive_tb2048_f384": (["-DTM_ALIVE_REG=1", "-DTM_TBCAP=2048", "-DTM_FCAP=384"], 0),
    "w20": (["-DTM_TBCAP=1536", "-DTM_FCAP=320", "-DTM_SCAP=96", "-DTM_MIN_WAVES=5"], 0),
    "f416": (["-DTM_FCAP=416"], 0),
    "s96": (["-DTM_SCAP=96"], 0),
    "noalive": (["-DTM_ALIVE_REG=0"], 0),
    "rpl1": (["-DTM_RPL=1"], 0),
    "r1p4_f256s96": (["-DTM_RPL=1", "-DTM_PRELOOK=4", "-DTM_FCAP=256", "-DTM_SCAP=96"], 0),
    "r1p6_f256s96": (["-DTM_RPL=1", "-DTM_PRELOOK=6", "-DTM_FCAP=256", "-DTM_SCAP=96"], 0),
    "r1p4_f192s64": (["-DTM_RPL=1", "-DTM_PRELOOK=4", "-DTM_FCAP=192", "-DTM_SCAP=64"], 0),
    "r1p10": (["-DTM_RPL=1", "-DTM_PRELOOK=10"], 0),
    "ff256": (["-DTM_FCAP_FIRST=256"], 0),
    "ff192": (["-DTM_FCAP_FIRST=192"], 0),
    "noalive_first": (["-DTM_ALIVE_REG=0"], 0),
    "cpu4": (["-DTM_CP_UNROLL=4"], 0),
    "cpu16": (["-DTM_CP_UNROLL=16"], 0),
    "qcopy16": (["-DTM_QCOPY=16"], 0),
    "qcopy4": (["-DTM_QCOPY=4"], 0),
    "el32": ([], 32),
    "tb2560_f448": (["-DTM_TBCAP=2560", "-DTM_FCAP=448"], 0),
    "tb2048_f512": (["-DTM_TBCAP=2048", "-DTM_FCAP=512"], 0),
    "tb2304_f480": (["-DTM_TBCAP=2304", "-DTM_FCAP=480"], 0),
    "tb2048_f576": (["-DTM_TBCAP=2048", "-DTM_FCAP=576"], 0),
    "tb1792_f544": (["-DTM_TBCAP=1792", "-DTM_FCAP=544"], 0),
    "plusnear": (["-DTM_PLUS_NEAR=1"], 0),  # '+' edges probe from their parent's slot + 1
    "plushash": (["-DTM_PLUS_NEAR=0"], 0),  # '+' edges hashed like every other edge (the product)
    "plusnear2": (["-DTM_PLUS_NEAR=1"], 0),
    "plushash2": (["-DTM_PLUS_NEAR=0"], 0),
    # round 5: edge-table load (translation pressure vs probe-chain length), 2 / 4 / 8 GiB
    "el2": ([], 2),
    "el4": ([], 4),
    "el8": ([], 8),
    # round 5: the pre-scan as its own kernel (k_prescan) ahead of k_match_fast<PRE>
    "pre": (["-DTM_PREPASS=1"], 0),
    "nopass": (["-DTM_PREPASS=0"], 0),
    "pre_w20": (["-DTM_PREPASS=1", "-DTM_MIN_WAVES=5"], 0),
    "pre2": (["-DTM_PREPASS=1"], 0),
    "nopass2": (["-DTM_PREPASS=0"], 0),
    # round 6: the PRE walk held at 16 waves/CU (LDS padded), to price the word-table probes
    "pre16": (["-DTM_PREPASS=1", "-DTM_PRE_PAD=1"], 0),
}


def build(names):
    os.makedirs(VDIR, exist_ok=True)
    procs = []
    for name in names:
        flags = VARIANTS[name][0]
        out = os.path.join(VDIR, f"libemqx_tm_{name}.so")
        kern = os.path.join(CSRC, "match_kernels.hip")
        if name in ("head", "prev"):
            ref = "HEAD" if name == "head" else os.environ.get("SWEEP_PREV", "af8ba73")
            kern = os.path.join(CSRC, f"_{name}_match_kernels.hip")
            with open(kern, "w") as f:
                f.write(subprocess.check_output(["git", "-C", ROOT, "show", f"{ref}:emqx_amd/csrc/match_kernels.hip"],
                                                text=True))
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-function", *flags, os.path.join(CSRC, "engine.cpp"),
               os.path.join(CSRC, "batcher.cpp"), kern, os.path.join(CSRC, "result_kernels.hip"),
               os.path.join(CSRC, "filter_kernels.hip"), "-o", out]
        procs.append((name, subprocess.Popen(cmd)))
        if len(procs) >= 4:
            n, p = procs.pop(0)
            assert p.wait() == 0, n
    for n, p in procs:
        assert p.wait() == 0, n


def run(args):
    import numpy as np
    import torch

    from emqx_amd import workloads
    w = workloads.generate(args.config, scale=args.scale, n_topics=args.batch)
    tb, to = w.topic_slice(0, args.batch)
    n = args.batch
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(tb).to(dev)
    d_off = torch.from_numpy(to.view(np.int32)).to(dev)
    stream = torch.cuda.Stream(dev)
    import importlib
    results = []
    digests = []
    for name in args.variants:
        lib = os.path.join(VDIR, f"libemqx_tm_{name}.so")
        os.environ["EMQX_TM_LIB"] = lib
        from emqx_amd import _native
        importlib.reload(_native)
        N = _native
        t0 = time.time()
        print(f"variant {name}: building the index", file=sys.stderr, flush=True)
        v = VARIANTS[name]
        eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4, edge_load_inv=v[1],
                       topics_per_wave=v[2] if len(v) > 2 else 0)
        eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
        eng.commit()
        tbuild = time.time() - t0
        sp = stream.cuda_stream

        def step():
            if args.mode == "first":  # return_first (k_match_first_wave)
                return eng.match_device_mode(d_bytes.data_ptr(), d_off.data_ptr(), n, int(to[-1]), N.TM_MATCH_FIRST, sp)
            return eng.match_device(d_bytes.data_ptr(), d_off.data_ptr(), n, int(to[-1]), sp)

        r = step()
        eng.device_sync()
        total = _read_u64(r.d_total)
        if total > r.keys_cap:
            eng.reserve_matches(int(total * 1.1) + 1024)
        for _ in range(3):
            step()
        eng.device_sync()
        torch.cuda.synchronize()
        eng.debug_stats(True, read=False)
        r = step()  # this launch's result (reserve_matches above re-allocated the key arena)
        torch.cuda.synchronize()
        walk = dict(zip(N.Engine.STAT_NAMES, [int(x) for x in eng.debug_stats(False)]))
        digest = _topic_digest(eng, r, n, _read_u64(r.d_total), sp) if args.mode == "all" else None
        eng.debug_stats(False, read=False)
        kms = []
        for _ in range(args.steps):
            eng.timing(True)
            step()
            torch.cuda.synchronize()
            kms.append(eng.timing(False))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        bms = (time.perf_counter() - t0) / args.steps * 1e3
        st = eng.stats()
        rec = {"variant": name, "kernel_ms": round(float(np.mean(kms)), 4), "kernel_ms_min": round(float(min(kms)), 4),
               "batch_ms": round(bms, 4), "keys": walk["keys"], "edge_probes": walk["edge_probes"],
               "word_probes": walk["word_probes"], "edge_slots": st["edge_slots"], "build_s": round(tbuild, 1),
               "cyc": [walk["cyc_prescan"], walk["cyc_walk"], walk["cyc_copyout"]]}
        if digest is not None:
            if digests:
                rec["same_keys_per_topic"] = bool(torch.equal(digest, digests[0]))
            digests.append(digest)
        print(json.dumps(rec), flush=True)
        results.append(rec)
        eng.close()
        del eng
    keys = {r["keys"] for r in results}
    print(json.dumps({"consistent_key_counts": len(keys) == 1}), flush=True)


def _topic_digest(eng, r, n, total, stream):
    """Per topic: the count and the sum of a hash of its route ids (order-independent; key
    handles are build-specific, ids are not), from tm_result_ids_device on the device."""
    import torch
    if total > r.keys_cap:
        raise RuntimeError(f"batch overflowed its key arena ({total} > {r.keys_cap})")
    dev = torch.device("cuda", 0)
    ids = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng.result_ids_device(ids.data_ptr(), ids.numel(), off.data_ptr(), stream)
    eng.device_sync()
    torch.cuda.synchronize()
    o = off.long() & 0xFFFFFFFF
    h = (ids[:total] * 0x9E3779B97F4A7C15) >> 16
    cs = torch.zeros(total + 1, dtype=torch.int64, device=dev)
    cs[1:] = torch.cumsum(h, 0)
    return torch.stack([o[1:] - o[:-1], cs[o[1:]] - cs[o[:-1]]])


def _read_u64(ptr):
    import torch
    h = torch.empty(1, dtype=torch.int64)
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert lib.hipMemcpy(C.c_void_p(h.data_ptr()), C.c_void_p(ptr), 8, 2) == 0
    return int(h.item())


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=("build", "run"))
    ap.add_argument("--variants", nargs="*", default=list(VARIANTS))
    ap.add_argument("--config", default="C")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", choices=("all", "first"), default="all")
    a = ap.parse_args()
    if a.cmd == "build":
        build(a.variants)
    else:
        import torch  # noqa: F401  (torch's HIP runtime first: see emqx_amd/_native.py)
        run(a)
