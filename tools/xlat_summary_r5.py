"""Summarise tools/prof_translation_r5.sh OUT into markdown (profiles/r05_prof_translation.md):
the region-grouped gather ceiling (two runs), its UTCL1 / TA / UTCL2 counters per timed
dispatch, and k_match_fast's translation counters at edge load 1/16 and 1/4 with the 1/4
kernel trace.  python tools/xlat_summary_r5.py [OUT]"""
import collections
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/xlat"


def counters(name, kernel=None):
    for root, _, files in os.walk(os.path.join(D, name)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                by = collections.OrderedDict()
                for r in csv.DictReader(open(os.path.join(root, f))):
                    if kernel and kernel not in r["Kernel_Name"]:
                        continue
                    by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
                return [by[k] for k in sorted(by)]
    return []


def trace_ms(name, kernel):
    for root, _, files in os.walk(os.path.join(D, name)):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                        for r in csv.DictReader(open(os.path.join(root, f))) if kernel in r["Kernel_Name"]]
    return []


print("# Address translation, round 5 (`tools/prof_translation_r5.sh`)\n")
print("## Random 16-B gathers over a 16 GiB table, lanes of a load grouped G per 2 MiB region\n")
print("| G lanes / region | in flight / lane | G loads/s run a | run b | UTCL1 miss / request | UTCL1 stall on UTCL2 credits (M cycles) | UTCL2 busy / GUI active (M cycles) | TA addr stalled by TC (M cycles) |")
print("|---|---|---|---|---|---|---|---|")
ra = [json.loads(x) for x in open(os.path.join(D, "regions_a.jsonl"))]
rb = [json.loads(x) for x in open(os.path.join(D, "regions_b.jsonl"))]
cu = counters("gr_utc")[1::2]  # every run_grp: a warm-up dispatch, then the timed one
ct = counters("gr_ta")[1::2]
for i, (a, b) in enumerate(zip(ra, rb)):
    u = cu[i] if i < len(cu) else {}
    t = ct[i] if i < len(ct) else {}
    miss = u.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / max(u.get("TCP_UTCL1_REQUEST_sum", 1), 1)
    print(f"| {a['lanes_per_2MiB_region']} | {a['inflight_per_lane']} | {a['G_loads_per_s']} | {b['G_loads_per_s']} | "
          f"{miss:.3f} | {u.get('TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum', 0) / 1e6:.1f} | "
          f"{t.get('GRBM_UTCL2_BUSY', 0) / 1e6:.1f} / {t.get('GRBM_GUI_ACTIVE', 0) / 1e6:.1f} | "
          f"{t.get('TA_ADDR_STALLED_BY_TC_CYCLES_sum', 0) / 1e6:.0f} |")
print("\n## `k_match_fast`, config C, 1 M publishes: edge load 1/16 (16 GiB table) vs 1/4 (4 GiB)\n")
print("Counter values per launch, mean of the last 8 launches of `bench.py --profile --sequential --steps 4` "
      "(4 timed steps + 4 kernel-timing runs; the earlier ones are sizing runs whose copy-out overflowed and the "
      "counted debug-statistics runs).\n")
print("| load | UTCL1 hits (M) | UTCL1 misses (M) | stall on UTCL2 credits (M cycles) | UTCL2 busy (M cycles) | GUI active (M cycles) |")
print("|---|---|---|---|---|---|")
for name, load in (("utc16", "1/16"), ("utc4", "1/4")):
    c = counters(name, "k_match_fast")[-8:]
    if not c:
        continue
    m = {k: sum(x.get(k, 0) for x in c) / len(c) / 1e6 for k in c[0]}
    print(f"| {load} | {m.get('TCP_UTCL1_TRANSLATION_HIT_sum', 0):.2f} | {m.get('TCP_UTCL1_TRANSLATION_MISS_sum', 0):.2f} | "
          f"{m.get('TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum', 0):.2f} | {m.get('GRBM_UTCL2_BUSY', 0):.2f} | "
          f"{m.get('GRBM_GUI_ACTIVE', 0):.2f} |")
t4 = trace_ms("trace4", "k_match_fast")[-8:]
if t4:
    print(f"\nKernel trace at load 1/4, the same 8 launches: mean {sum(t4) / len(t4):.4f} ms, "
          f"min {min(t4):.4f} ms (load 1/16 in the same round: 0.689-0.729 ms, `profiles/r05_sweep_load.jsonl`).")
