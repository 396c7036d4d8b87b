"""Summarise a rocprofv3 --kernel-trace --stats CSV directory (per-step ms by kernel)."""
import csv
import sys
import collections

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r["Kernel_Name"]
    short = name.replace("(anonymous namespace)::", "").split("(")[0]
    if "Cijk" in short:
        short = "hipBLASLt:" + short[:50]
    grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    key = (short[:90], grid if ("gemm" in short or "Cijk" in short or "lora" in short) else "")
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot:.3f} ms  ({tot/steps:.3f} ms/step over {steps:g} steps)")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{t/steps:8.3f} ms/step  {n/steps:6.1f}/step  avg {t/n*1000:8.1f} us  grid={k[1]!s:>6}  {k[0]}")
