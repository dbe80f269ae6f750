"""Summarise tools/prof_latency.sh passes: per-launch counters of k_match_fast (the headline
launch) and the derived latencies.

    python tools/summarize_latency.py gpurun_out/lat profiles/r04_prof_latency
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_prof import KERNEL, per_kernel  # noqa: E402


def main(src, dst):
    pmc = {}
    for name in ("lat", "tlb", "utc"):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if os.path.exists(p):
            pmc.update(per_kernel(p))
    g = pmc.get
    d = {}
    if g("TCP_TCC_READ_REQ_sum"):
        d["l1_to_l2_read_latency_cycles"] = g("TCP_TCC_READ_REQ_LATENCY_sum", 0) / g("TCP_TCC_READ_REQ_sum")
    if g("TCC_EA0_RDREQ_sum"):
        d["l2_to_fabric_read_latency_cycles"] = g("TCC_EA0_RDREQ_LEVEL_sum", 0) / g("TCC_EA0_RDREQ_sum")
        d["fabric_reads_to_dram_frac"] = g("TCC_EA0_RDREQ_DRAM_sum", 0) / g("TCC_EA0_RDREQ_sum")
    if g("TCP_UTCL1_REQUEST_sum"):
        d["utcl1_miss_frac"] = g("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / g("TCP_UTCL1_REQUEST_sum")
    if g("GRBM_GUI_ACTIVE"):
        d["utcl2_busy_frac"] = g("GRBM_UTCL2_BUSY", 0) / g("GRBM_GUI_ACTIVE")
    out = {"source": src, "kernel": KERNEL, "pmc_per_launch": pmc, "derived": d}
    with open(dst + ".json", "w") as f:
        json.dump(out, f, indent=1)
    with open(dst + ".md", "w") as f:
        f.write(f"# {os.path.basename(dst)} — latency / translation counters of `{KERNEL}` per launch\n\n")
        f.write("| counter | value |\n|---|---|\n")
        for k in sorted(pmc):
            f.write(f"| {k} | {pmc[k]:.4g} |\n")
        f.write("\n| derived | value |\n|---|---|\n")
        for k, v in d.items():
            f.write(f"| {k} | {v:.4g} |\n")
    print(json.dumps(d))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
