"""Where one greedy generate() call's time goes, from a rocprofv3 kernel trace of apps/gen_probe.py.

  python tools/gen_timeline.py <kernel_trace.csv> [new_tokens=16]

The last call's decode steps end with one ``decode_tail`` kernel each (new_tokens - 1 replays); its
prefill is everything between the previous call's last ``decode_tail`` and the first kernel of the
first replay.  Prints the prefill kernels with the idle gap before each, then per-phase kernel sums
against wall spans (the difference is host / launch time the GPU sat idle).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    new = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tails = [i for i, r in enumerate(rows) if "decode_tail" in r["Kernel_Name"]]
    # whole-call graph (round 5): the prefill ends with token 0's decode_tail, then new - 1 steps;
    # older traces (one replay per step, eager prefill) have new - 1 tails per call
    graph_call = len(tails) % new == 0 and len(tails) >= 2 * new
    reps = new - 1
    if len(tails) < 2 * reps:
        sys.exit(f"need two generate() calls in the trace ({len(tails)} decode_tail kernels)")
    last = tails[-reps:]
    prev_end = tails[-reps - 2] if graph_call else tails[-reps - 1]
    per_step = last[1] - last[0]
    first_rep = last[0] - per_step + 1
    t = lambda i, k: int(rows[i][k])  # noqa: E731
    print(f"# prefill + setup: kernels {prev_end + 1} .. {first_rep - 1}")
    for i in range(prev_end + 1, first_rep):
        d = (t(i, "End_Timestamp") - t(i, "Start_Timestamp")) / 1e3
        gap = (t(i, "Start_Timestamp") - t(i - 1, "End_Timestamp")) / 1e3
        print(f"{d:8.2f} us gap {gap:8.2f}  {rows[i]['Kernel_Name'][:90]}")

    def span(a, b):
        ks = sum(t(i, "End_Timestamp") - t(i, "Start_Timestamp") for i in range(a, b + 1)) / 1e3
        return ks, (t(b, "End_Timestamp") - t(a, "Start_Timestamp")) / 1e3

    pk, pw = span(prev_end + 1, first_rep - 1)
    dk, dw = span(first_rep, last[-1])
    gap = (t(first_rep, "Start_Timestamp") - t(first_rep - 1, "End_Timestamp")) / 1e3
    print(f"prefill: {first_rep - prev_end - 1} kernels, kernel sum {pk:.1f} us, span {pw:.1f} us")
    print(f"prefill -> first replay gap {gap:.1f} us")
    print(f"decode: {reps} replays x {per_step} kernels, kernel sum {dk:.1f} us, span {dw:.1f} us "
          f"({dw / reps:.1f} us per step)")
    print(f"call (prefill start .. last tail end): {(t(last[-1], 'End_Timestamp') - t(prev_end + 1, 'Start_Timestamp')) / 1e3:.1f} us"
          f" = {(t(last[-1], 'End_Timestamp') - t(prev_end + 1, 'Start_Timestamp')) / 1e3 / new:.1f} us per new token")


if __name__ == "__main__":
    main()
