"""Summarise a rocprofv3 --kernel-trace run (per-step ms by kernel).

Reads either the CSV output (``run_kernel_trace.csv``) or the rocpd SQLite
database (``*_results.db``, rocprofv3's default format in ROCm 7).

  python tools/prof_summary.py <dir> [steps] [--skip-first-ms MS]
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def rows_from_dir(d):
    csvp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(csvp):
        for r in csv.DictReader(open(csvp)):
            yield (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["Start_Timestamp"]),
                   int(r["End_Timestamp"]))
        return
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        q = ("select s.kernel_name, k.grid_size_x, k.workgroup_size_x, k.start, k.end "
             "from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s on k.kernel_id = s.id")
        yield from c.execute(q)


def short_name(name):
    s = name.replace("(anonymous namespace)::", "").split("(")[0]
    if "Cijk" in s:
        s = "hipBLASLt:" + s[:50]
    return s[:90]


def main(argv):
    d = argv[0]
    steps = float(argv[1]) if len(argv) > 1 and not argv[1].startswith("--") else 1.0
    skip_ms = float(argv[argv.index("--skip-first-ms") + 1]) if "--skip-first-ms" in argv else 0.0
    rows = sorted(rows_from_dir(d), key=lambda r: r[3])
    if not rows:
        print("no kernel records found")
        return
    t0 = rows[0][3] + skip_ms * 1e6
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, gx, wx, st, en in rows:
        if st < t0:
            continue
        short = short_name(name)
        grid = gx // max(1, wx)
        key = (short, grid if any(x in short for x in ("gemm", "Cijk", "lora", "attn")) else "")
        agg[key][0] += 1
        agg[key][1] += (en - st) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot:.3f} ms  ({tot / steps:.3f} ms/step over {steps:g} steps)")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{t / steps:8.3f} ms/step  {n / steps:7.1f}/step  avg {t / n * 1000:8.1f} us  grid={k[1]!s:>6}  {k[0]}")


if __name__ == "__main__":
    main(sys.argv[1:])
