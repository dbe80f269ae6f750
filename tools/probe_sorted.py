"""Probe (development): does grouping a batch's topics by their first levels cut k_match_fast's
L2 misses?  The batch is reordered on the HOST (numpy) and walked by the unchanged kernel, so
this measures the walk's gain alone, before any device-side grouping pass is built.

Variants of the same 1 M config-C publishes:
  orig      the generator's order (what the bench walks);
  sort2     stable-sorted by (level 0, level 1) bytes;
  sort3     by (level 0, level 1, level 2);
  sortall   by the whole topic;
  sort3x    sort3, then the 64-topic wave chunks interleaved so that blocks b, b+8, b+16, ...
            (one XCD under round-robin dispatch) walk CONSECUTIVE sorted chunks.
  xcd1/xcd2/xcd3  XCD-aware: the topics' first 1 / 2 / 3 levels are dealt to 8 groups
            (largest prefix first, to the group with the most room), and block b takes its 64
            topics from group b % 8 in the generator's (random) order.  Each XCD's L2 then sees
            only its groups' subtries below that level, while every wave still walks
            unrelated topics (no clustering, unlike the sorts).
Prints per variant: k_match_fast ms (HIP events on its stream, mean of 10), matched keys, and
that per-topic counts equal the original order's (permuted).

    python tools/probe_sorted.py [--scale 1.0] [--n 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import placement, workloads  # noqa: E402


def reorder(w, perm):
    to = w.t_off.astype(np.int64)
    lens = (to[1:] - to[:-1])[perm]
    noff = np.zeros(len(perm) + 1, np.int64)
    np.cumsum(lens, out=noff[1:])
    idx = np.repeat(to[:-1][perm] - noff[:-1], lens) + np.arange(int(noff[-1]), dtype=np.int64)
    nb = np.concatenate([w.t_bytes[idx], np.zeros(16, np.uint8)])
    return nb, noff.astype(np.uint32)


def level_keys(w, levels):
    """Per topic: its first `levels` levels as one bytes key (for np.argsort on an object array)."""
    ks = []
    tb = w.t_bytes.tobytes()
    to = w.t_off
    for i in range(w.n_topics):
        t = tb[int(to[i]):int(to[i + 1])]
        ks.append(t if levels is None else b"/".join(t.split(b"/")[:levels]))
    return np.array(ks, dtype=object)


def xcd_perm(keys, n, nx=8):
    """Topic permutation for the xcdK variants (see the module doc); None if n % 64 != 0."""
    if n % 64:
        return None
    _, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
    nw = n // 64
    blocks = [np.arange(x, nw, nx) for x in range(nx)]
    cap = np.array([len(b) * 64 for b in blocks], np.int64)
    load = np.zeros(nx, np.int64)
    assign = np.empty(len(cnt), np.int64)
    for g in np.argsort(-cnt, kind="stable"):
        x = int(np.argmax(cap - load))
        assign[g] = x
        load[x] += cnt[g]
    xt = assign[inv.reshape(-1)]
    lists = [np.nonzero(xt == x)[0] for x in range(nx)]
    spill = np.concatenate([lst[cap[x]:] for x, lst in enumerate(lists)])
    lists = [lst[:cap[x]] for x, lst in enumerate(lists)]
    for x in range(nx):  # overflowing prefixes' tails go to the groups with room
        need = int(cap[x] - len(lists[x]))
        if need:
            lists[x], spill = np.concatenate([lists[x], spill[:need]]), spill[need:]
    perm = np.empty(n, np.int64)
    for x in range(nx):
        perm[(blocks[x][:, None] * 64 + np.arange(64)).reshape(-1)] = lists[x]
    return perm, int(sum(max(0, int(l) - int(c)) for l, c in zip(load, cap)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--variants", nargs="*", default=["orig", "sort2", "sort3", "sortall", "sort3x"])
    args = ap.parse_args()
    placement.pin_to_gpu(0)
    w = workloads.generate("C", scale=args.scale, n_topics=args.n)
    eng = N.Engine(0, reserve_keys=w.n_keys, reserve_nodes=w.n_keys * 4)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id)
    eng.commit()
    eng.reserve_matches(int(18 * w.n_keys))  # config C: 142 M keys per 1 M publishes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    n = w.n_topics
    want = set(args.variants)
    variants = {"orig": np.arange(n)}
    for name, lv in (("sort2", 2), ("sort3", 3), ("sortall", None)):
        if name in want or (name == "sort3" and "sort3x" in want):
            variants[name] = np.argsort(level_keys(w, lv), kind="stable")
    nw = (n + 63) // 64
    if "sort3x" in want and n % 64 == 0 and nw % 8 == 0:  # block b walks sorted chunk (b % 8) * (nw / 8) + b / 8
        b = np.arange(nw)
        chunk = (b % 8) * (nw // 8) + b // 8
        variants["sort3x"] = variants["sort3"].reshape(nw, 64)[chunk].reshape(-1)
    for lv in (1, 2, 3):
        if f"xcd{lv}" in want:
            r = xcd_perm(level_keys(w, lv), n)
            if r is not None:
                variants[f"xcd{lv}"] = r[0]
                print(json.dumps({"variant": f"xcd{lv}", "spilled_topics": r[1]}), flush=True)
    variants = {k: v for k, v in variants.items() if k in want or k == "orig"}
    base_cnt = None
    for name, perm in variants.items():
        nb, no = reorder(w, perm)
        d_b = torch.from_numpy(nb).to(dev)
        d_o = torch.from_numpy(no.view(np.int32)).to(dev)
        r = eng.match_device(d_b.data_ptr(), d_o.data_ptr(), n, int(no[-1]), stream.cuda_stream)
        eng.device_sync()
        ms = []
        for k in range(13):
            eng.timing(True)
            r = eng.match_device(d_b.data_ptr(), d_o.data_ptr(), n, int(no[-1]), stream.cuda_stream)
            torch.cuda.synchronize()
            t = eng.timing(False)
            if k >= 3:
                ms.append(t)
        eng.device_sync()
        cnt = torch.zeros(n, dtype=torch.int32)
        import ctypes as C
        lib = C.CDLL("libamdhip64.so")
        lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        assert lib.hipMemcpy(C.c_void_p(cnt.data_ptr()), C.c_void_p(r.d_cnt), n * 4, 2) == 0
        c = cnt.numpy().astype(np.int64)
        got = np.empty(n, np.int64)
        got[perm] = c  # back to original topic order
        if base_cnt is None:
            base_cnt = got
        print(json.dumps({"variant": name, "kernel_ms": round(float(np.mean(ms)), 4),
                          "kernel_ms_min": round(float(np.min(ms)), 4), "keys": int(c.sum()),
                          "counts_equal_orig": bool(np.array_equal(got, base_cnt))}), flush=True)
        del d_b, d_o
    eng.close()


if __name__ == "__main__":
    main()
