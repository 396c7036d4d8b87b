"""Summarise rocprofv3 --pmc CSV runs per kernel, with a roofline table.

  python tools/pmc_summary.py <pmc_dir> [<pmc_dir> ...] [--top N] [--peak_tflops 2500] [--peak_hbm 6.3]

Every directory is ONE counter pass (rocprofv3 does not split counters over passes on gfx950, so the
SQ, FETCH_SIZE and WRITE_SIZE groups are collected by separate runs of the same command).  Each counter
is normalised by the kernel time of the pass that collected it (the passes differ in dispatch count and
in clock: MI355X_MICROARCH.md "DVFS give-back" item 2), then the passes are joined per kernel name.

Per kernel:
  mfma%      = SQ_VALU_MFMA_BUSY_CYCLES / (dur * 2.4 GHz * 1024 SIMDs)   (busy share at the max clock)
  wait/stall/issue = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as % of SQ_WAVE_CYCLES
  TF/s       = SQ_VALU_MFMA_BUSY_CYCLES * 1024 / dur: bf16/fp16 MFMA (16x16x32 and 32x32x16 both retire
               1024 FLOP per busy cycle; checked against the distilgpt2 LM head: 635 GF counted vs
               8192 x 50304 x 768 x 2 = 633 GF)
  rd/wr GB/s = 2 * FETCH_SIZE / dur (gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads,
               MI355X_MICROARCH.md "HBM") and WRITE_SIZE / dur; both count the memory side of the L2, so
               Infinity-Cache (MALL) hits are included: an upper bound on HBM traffic
  AI         = FLOP / (read + write bytes)
  clk GHz    = GRBM_GUI_ACTIVE / 8 XCDs / dur (reads high below ~0.3 ms per dispatch)
  bound      = the roof the kernel is closer to: MFMA (TF/s / peak) vs memory ((rd+wr) / peak HBM), with
               both shares printed; a kernel far from both is latency / issue bound ("lat")
"""
import collections
import csv
import glob
import os
import sys

CLK_GHZ = 2.4
SIMDS = 256 * 4


def load_pass(d):
    """-> {kernel: {"dur": ns summed, "n": dispatches, counter: summed value}} for one pass directory."""
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (p, r["Dispatch_Id"])
            if key not in seen[k]:
                seen[k].add(key)
                out[k]["dur"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                out[k]["n"] += 1
    return out


def main():
    argv = sys.argv[1:]
    opts = {"--top": 25, "--peak_tflops": 2500.0, "--peak_hbm": 6.3}
    dirs = []
    i = 0
    while i < len(argv):
        if argv[i] in opts:
            opts[argv[i]] = float(argv[i + 1])
            i += 2
        else:
            dirs.append(argv[i])
            i += 1
    top, peak_tf, peak_bw = int(opts["--top"]), opts["--peak_tflops"], opts["--peak_hbm"]
    # per kernel: counter -> (value, duration of its own pass); time/dispatch count from the first pass
    rates = collections.defaultdict(dict)
    base = {}
    for d in dirs:
        for k, c in load_pass(d).items():
            for name, v in c.items():
                if name in ("dur", "n"):
                    continue
                rates[k][name] = (v, c["dur"], c["n"])
            if k not in base:
                base[k] = (c["dur"], c["n"])
    rows = sorted(((base[k][0], k) for k in base), reverse=True)
    tot_all = sum(t for t, _ in rows)
    print(f"{'total_us':>9} {'%':>5} {'n':>4} {'avg_us':>8} {'mfma%':>6} {'wait%':>6} {'stall%':>6} {'issue%':>6} "
          f"{'ldsconf/d':>9} {'TF/s':>7} {'rdGB/s':>7} {'wrGB/s':>7} {'AI':>6} {'clk':>5} {'bound':>14}  kernel")
    nan = float("nan")
    for tot, k in rows[:top]:
        n = int(base[k][1])
        r = rates[k]

        def per_ns(name):  # counter per ns of its own pass
            if name not in r:
                return nan
            v, dur, _ = r[name]
            return v / dur if dur else nan

        def share(name):
            if name not in r or "SQ_WAVE_CYCLES" not in r:
                return nan
            return 100.0 * r[name][0] / r["SQ_WAVE_CYCLES"][0] if r["SQ_WAVE_CYCLES"][0] else nan

        mfma = 100.0 * per_ns("SQ_VALU_MFMA_BUSY_CYCLES") / (CLK_GHZ * SIMDS)
        tfs = per_ns("SQ_VALU_MFMA_BUSY_CYCLES") * 1024 / 1e3  # FLOP/ns -> TF/s
        rd = 2 * per_ns("FETCH_SIZE") * 1024  # KB/ns -> B/ns = GB/s
        wr = per_ns("WRITE_SIZE") * 1024
        clk = per_ns("GRBM_GUI_ACTIVE") / 8
        lds = r["SQ_LDS_BANK_CONFLICT"][0] / r["SQ_LDS_BANK_CONFLICT"][2] if "SQ_LDS_BANK_CONFLICT" in r else nan
        bw = (rd if rd == rd else 0.0) + (wr if wr == wr else 0.0)
        ai = tfs * 1e3 / bw if bw > 0 and tfs == tfs else nan
        fc = tfs / peak_tf if tfs == tfs else 0.0
        fm = bw / (peak_bw * 1e3)
        if max(fc, fm) < 0.25:
            bound = f"lat {fc:.2f}/{fm:.2f}"
        else:
            bound = (f"mfma {fc:.2f}/{fm:.2f}" if fc >= fm else f"mem {fc:.2f}/{fm:.2f}")
        print(f"{tot/1e3:9.1f} {100*tot/tot_all:5.1f} {n:4d} {tot/n/1e3:8.1f} {mfma:6.1f} {share('SQ_WAIT_ANY'):6.1f} "
              f"{share('SQ_WAIT_INST_ANY'):6.1f} {share('SQ_ACTIVE_INST_ANY'):6.1f} {lds:9.0f} {tfs:7.1f} {rd:7.0f} "
              f"{wr:7.0f} {ai:6.1f} {clk:5.2f} {bound:>14}  {k[:80]}")
    print(f"# {len(dirs)} pass(es): {', '.join(dirs)}; bound shares = TF/s / {peak_tf:.0f} and (rd+wr) / {peak_bw} TB/s")


if __name__ == "__main__":
    main()
