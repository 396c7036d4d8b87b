"""One graph-replayed decode step's kernels (between the last two ``decode_tail`` kernels of a
rocprofv3 kernel trace of apps/gen_probe.py), with durations and the idle gap before each.

  python tools/decode_step_kernels.py <kernel_trace.csv>
"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    tails = [i for i, r in enumerate(rows) if "decode_tail" in r["Kernel_Name"]]
    a, b = tails[-2], tails[-1]
    tot = 0.0
    prev_end = int(rows[a]["End_Timestamp"])
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        tot += d
        print(f"{d:8.2f} us  gap {(s - prev_end) / 1e3:6.2f}  {r['Kernel_Name'][:110]}")
        prev_end = e
    span = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
    print(f"{b - a} kernels, kernel sum {tot:.1f} us, step span {span:.1f} us")


if __name__ == "__main__":
    main()
