"""Summarise tools/prof_filter_r5.sh OUT: k_filter_walk / k_filter_bulk launches in launch order
(each bench call: the 1-query index-build call, warm-up + 3 keys-form batches and the parity
batch, then warm-up + 3 runs-form batches and the runs parity batch; the runs form is one walk
launch per call), and FETCH / WRITE per launch of the mixed batch (MI355X_MICROARCH.md:
FETCH_SIZE / WRITE_SIZE in KiB).  python tools/filter_prof_r5.py OUT > profiles/r05_prof_filter_walk.md"""
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_filter_r5"


def trace(name):
    for root, _, files in os.walk(os.path.join(D, name)):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                rows = list(csv.DictReader(open(os.path.join(root, f))))
                rows.sort(key=lambda r: int(r["Start_Timestamp"]))
                return [("bulk" if "bulk" in r["Kernel_Name"] else "walk",
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                        for r in rows if "k_filter" in r["Kernel_Name"]]
    return []


def counters(name):
    for root, _, files in os.walk(os.path.join(D, name)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return [("bulk" if "bulk" in r["Kernel_Name"] else "walk", float(r["Counter_Value"]) * 1024 / 1e9)
                        for r in csv.DictReader(open(os.path.join(root, f))) if "k_filter" in r["Kernel_Name"]]
    return []


def line(name):
    try:
        return json.loads(open(os.path.join(D, name + ".json")).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        return {}


print("# `k_filter_walk` at config C (10.65 M keys), round 5 source — `tools/prof_filter_r5.sh`\n")
for name, what in (("mixed", "mixed 100 K-query batch (stored / one '+' / prefix + '#')"),
                   ("plus", "one-'+' queries only (≈ 3 K), split into parts (16384:4096, the round's first default)"),
                   ("plus_nosplit", "one-'+' queries only, unsplit (EMQX_TM_FILTER_SPLIT=0)")):
    ls = trace(name)
    j = line(name)
    print(f"## {what}\n")
    print(f"- bench line: queries {j.get('config', {}).get('queries')}, keys form {j.get('ms_per_batch')} ms per "
          f"batch through the C-ABI")
    print(f"- launches in order (ms): {', '.join(f'{n} {t:.3f}' for n, t in ls)}")
    runs = [t for n, t in ls if n == "walk"][-5:]
    if runs:
        print(f"- runs-form walks (the last 5 walk launches: warm-up, 3 timed, parity): "
              f"{', '.join(f'{t:.3f}' for t in runs)}; mean of the 3 timed {sum(runs[1:4]) / 3:.3f} ms")
    print()
print("## PMC per launch, mixed batch (GB)\n")
for n in ("fetch", "write"):
    print(f"- {n.upper()}_SIZE: {', '.join(f'{k} {v:.3f}' for k, v in counters(n))}")
