"""Print the kernel sequence of one training step from a rocprofv3 kernel trace.

  python tools/step_timeline.py <kernel_trace.csv> [delimiter_kernel=opt_apply_kernel] [which=-2]

Steps are delimited by the optimizer kernel; prints duration, the idle gap
before each kernel and the workgroup count, then the step's kernel-time sum
vs its wall span (the difference is host/launch idle time).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    delim = sys.argv[2] if len(sys.argv) > 2 else "opt_apply_kernel"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if delim in r["Kernel_Name"]]
    a, b = idx[which - 1], idx[which]
    prev_end = int(rows[a]["End_Timestamp"])
    tot = 0.0
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3
        prev_end = e
        n = r["Kernel_Name"].replace("_ZN12_GLOBAL__N_1", "")[:70]
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{(e - s) / 1e3:8.1f}us gap {gap:6.1f} wg={wg:6d} {n}")
        tot += (e - s) / 1e3
    span = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
    print(f"kernel sum {tot:.1f} us, step span {span:.1f} us")


if __name__ == "__main__":
    main()
