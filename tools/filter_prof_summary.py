"""Summarise a tools/gpu_r2f3.sh run: k_filter_walk / k_filter_bulk launches of the mixed
100K-query batch and of each query kind, and FETCH/WRITE per launch (MI355X_MICROARCH.md:
FETCH_SIZE/WRITE_SIZE in KiB).  python tools/filter_prof_summary.py TAG > profiles/...md"""
import csv
import sys

T = sys.argv[1]


def launches(path):
    out = []
    for r in csv.DictReader(open(path)):
        if "k_filter" not in r["Kernel_Name"]:
            continue
        name = "k_filter_bulk" if "bulk" in r["Kernel_Name"] else "k_filter_walk"
        out.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return out


def fmt(ls):
    return ", ".join(f"{n[9:]} {t:.2f}" for n, t in ls)


print(f"# k_filter_walk at config C (10.65 M keys), 100 K queries — `tools/gpu_r2f3.sh {T}`\n")
print("Per-launch durations in ms, in launch order (the first launches are the 1-query index build "
      "call and the two-pass sizing batch; then one-pass walk + bulk pairs):\n")
print(f"- mixed batch: {fmt(launches(f'gpurun_out/prof_filter_{T}/trace/trace_kernel_trace.csv'))}")
for k, name in enumerate(("stored filters", "one level '+'", "prefix + '#'")):
    print(f"- kind {k} ({name}) only: {fmt(launches(f'gpurun_out/prof_fk{k}/trace_kernel_trace.csv'))}")
print("\nPMC per launch of the mixed batch (GB):\n")
for n in ("fetch", "write"):
    vals = []
    for r in csv.DictReader(open(f"gpurun_out/prof_filter_{T}/{n}/{n}_counter_collection.csv")):
        if "k_filter" in r["Kernel_Name"]:
            kn = "bulk" if "bulk" in r["Kernel_Name"] else "walk"
            vals.append(f"{kn} {float(r['Counter_Value']) * 1024 / 1e9:.3f}")
    print(f"- {n.upper()}_SIZE: {', '.join(vals)}")
