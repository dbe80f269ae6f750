"""Per-kernel call count, average and total duration (ms) from rocprofv3 result databases
(`-o name` without --output-format csv writes <dir>/<name>_results.db).
Usage: python tools/kstats.py gpurun_out/r3o_prof_mix [more dirs]"""
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    for db in sorted(glob.glob(f"{d}/**/*_results.db", recursive=True)):
        c = sqlite3.connect(db)
        rows = c.execute("select name, count(*), avg(end-start)/1e6, sum(end-start)/1e6 from kernels "
                         "group by name order by 4 desc limit 6").fetchall()
        print(db)
        for n, k, avg, tot in rows:
            print(f"  {n[:70]:70s} {k:6d} avg {avg:9.4f} ms total {tot:9.2f} ms")
