"""Summarise a tools/prof_pmc.sh output directory into one JSON + markdown table.

    python tools/summarize_prof.py gpurun_out/prof2 profiles/r01_prof

Per-launch HBM traffic of k_match_fast from the PMC passes, with the gfx950
corrections of MI355X_MICROARCH.md §HBM:
  * FETCH_SIZE/WRITE_SIZE are in KiB;
  * tools/calib_fetch.hip measured on this pool: a random 16-B load that misses L2 is
    counted as 64 B (16.78 M loads -> FETCH_SIZE 1,048,839 KiB), a wide coalesced
    stream is counted at exactly half its bytes (4 GiB -> 2,097,160 KiB);
  * k_match_fast is dominated by random 16-B gathers (edge / word slots), so its
    FETCH_SIZE is used as measured (x1); the factor-2 stream correction would apply
    only to the key-arena copy-out, an upper bound given separately.
"""
from __future__ import annotations

import csv
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_match_fast<false, 0"  # STATS off, keys output (the headline step; <.., PRE> since round 5)
PRE = "k_prescan<false>"            # round 5: the pre-scan kernel launched ahead of it (if any)


def per_kernel(path, kernel=KERNEL):
    vals = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main(src, dst):
    out = {"source": src}
    sha = os.path.join(src, "src.sha")
    if os.path.exists(sha):
        import hashlib
        out["kernel_src_sha"] = hashlib.sha256(open(sha, "rb").read()).hexdigest()
    stats_csv = os.path.join(src, "trace", "trace_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats_csv)))
    out["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "Percentage", "MinNs", "MaxNs")}
                           for r in rows]
    fast = [r for r in rows if KERNEL in r["Name"]][0]
    pre = [r for r in rows if PRE in r["Name"]]
    # the step's kernels: k_prescan (when launched) + k_match_fast, per launch pair
    avg_ns = float(fast["AverageNs"]) + (float(pre[0]["AverageNs"]) if pre else 0.0)
    out["kernels"] = [KERNEL] + ([PRE] if pre else [])
    pmc, pmc_pre = {}, {}
    for name in ("fetch", "write", "tcc", "sq"):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if os.path.exists(p):
            pmc.update(per_kernel(p))
            if pre:
                pmc_pre.update(per_kernel(p, PRE))
    for k in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
        if k in pmc and k in pmc_pre:
            pmc[k] += pmc_pre[k]
    out["pmc_per_launch_prescan"] = pmc_pre
    out["pmc_per_launch"] = pmc
    bench = json.load(open(os.path.join(src, "trace.bench.json")))
    out["bench_line"] = bench
    fetch = pmc.get("FETCH_SIZE", 0) * 1024
    write = pmc.get("WRITE_SIZE", 0) * 1024
    walk = bench["roofline"].get("walk")
    if walk is None:  # round 6: the compact line keeps the walk counters in its side file
        det = json.load(open(DETAIL or os.path.join(os.path.dirname(os.path.normpath(src)), "bench_detail.json")))
        walk = det["roofline"]["walk"]
    keys = walk["keys"]
    traffic = fetch + write
    out["traffic"] = {
        "fetch_bytes": fetch, "write_bytes": write, "hbm_bytes": traffic,
        "hbm_bytes_upper": traffic + 4 * keys,  # if the arena copy-out stream is undercounted 2x
        "algorithmic_bytes": bench["roofline"]["algorithmic_bytes_per_launch"],
        "kernel_avg_ns_rocprof": avg_ns,
        "achieved_hbm_GBps": traffic / avg_ns,
        "l2_hit_rate": pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"]) if "TCC_HIT_sum" in pmc else None,
    }
    if "SQ_WAVE_CYCLES" in pmc:
        out["traffic"]["wait_fraction"] = pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
        # GRBM_GUI_ACTIVE sums the 8 XCDs; SQ_*_CYCLES count quad-cycles
        out["traffic"]["avg_resident_waves"] = 4 * pmc["SQ_WAVE_CYCLES"] / (pmc["GRBM_GUI_ACTIVE"] / 8)
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst + ".json", "w") as f:
        json.dump(out, f, indent=1)
    t = out["traffic"]
    md = [f"# {os.path.basename(dst)} — rocprofv3 summary of `bash tools/prof_pmc.sh` (config C, 1M publishes/launch)",
          "", "| kernel | calls | avg ns | % |", "|---|---|---|---|"]
    for r in out["kernel_stats"]:
        md.append(f"| `{r['Name']}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {float(r['Percentage']):.2f} |")
    md += ["", "| k_match_fast per launch | value |", "|---|---|"]
    for k, v in t.items():
        md.append(f"| {k} | {v:.4g} |" if isinstance(v, float) else f"| {k} | {v} |")
    md += ["", "PMC (per launch, raw): " + ", ".join(f"{k}={v:.4g}" for k, v in sorted(pmc.items()))]
    with open(dst + ".md", "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


DETAIL = None  # the default bench line's side file (argv[3]): walk counters of a full 1 M batch

if __name__ == "__main__":
    if len(sys.argv) > 3:
        DETAIL = sys.argv[3]
    main(sys.argv[1], sys.argv[2])
