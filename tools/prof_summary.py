#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (engine kernels)
  profiles/<tag>_summary.md         durations, PMC counters per launch, derived rates
  profiles/traffic.json             HBM bytes per launch for bench.py's roofline.traffic

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of the
bytes of a wide (16 B/lane) streaming read on gfx950, so read bytes = 2 * FETCH_SIZE *
1024; WRITE_SIZE (KiB) is exact for 16-B stores and uncalibrated for the 8-B row stores
used here (reported as measured). Counter passes are separate runs (one per pass).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MI355X engine clock range (MI355X_MICROARCH.md: 2.4 GHz peak; idle-to-boost floor)
CLOCK_RANGE_GHZ = (0.8, 2.45)
ENGINE = re.compile(r"spectral64_kernel|tile_idx_kernel|iir_tile|filtfilt|order_kernel|order_sel_kernel|sampen_kernel|rqa_kernel|moments_indexed|tile_kernel|tile64_kernel|tile64_stream_kernel|moments_generic|span_kernel|spectral_kernel|spectral_wave_kernel|spectral_reg_kernel|iir_chunk|mhf_")


def clock_line(grbm_gui_active, avg_ns):
    """The effective clock line. The duration comes from the kernel-trace run, the busy
    cycles from a PMC run: a clock outside what the part can run means the two runs did not
    time the same thing (short kernels: the counter pass's dispatch overhead lands in
    GRBM_GUI_ACTIVE), and then no clock is derived."""
    clk = grbm_gui_active / 8 / (avg_ns * 1e-9) / 1e9
    if CLOCK_RANGE_GHZ[0] <= clk <= CLOCK_RANGE_GHZ[1]:
        return "effective clock (GRBM_GUI_ACTIVE / 8 / duration) = %.2f GHz" % clk
    return ("effective clock NOT derived: GRBM_GUI_ACTIVE / 8 over the trace run's duration "
            "gives %.2f GHz, outside %.1f-%.2f GHz (trace and PMC runs disagree)"
            % ((clk,) + CLOCK_RANGE_GHZ))


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:80]


def counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if ENGINE.search(r["Kernel_Name"]):
                out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--plan", default=None, help="engine plan name (bench config.kernel)")
    ap.add_argument("--algo-bytes", type=float, default=None)
    ap.add_argument("--windows", type=int, default=None, help="windows per launch profiled")
    ap.add_argument("--sum-kernels", action="store_true",
                    help="traffic = the sum over the profiled kernels (one bench step launches "
                         "several, e.g. filtfilt's two passes)")
    ap.add_argument("--features", default=None,
                    help="comma-separated feature names of the profiled launch (bench.py)")
    args = ap.parse_args()
    d = os.path.join(ROOT, "gpurun_out", "prof_" + args.tag)
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(d, "trace", "trace_kernel_stats.csv")
    rows = [r for r in csv.DictReader(open(stats)) if ENGINE.search(r["Name"])]
    with open(os.path.join(prof, args.tag + "_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    cnt = counters(d)
    lines = ["# rocprofv3 summary: %s (%s)" % (args.tag, args.config), "",
             "Kernel durations (`rocprofv3 --kernel-trace --stats`, engine kernels only):", "",
             "| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
    for r in rows:
        lines.append("| %s | %s | %.1f | %.1f | %.1f |" % (
            short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
            float(r["MaxNs"]) / 1e3))
    lines += ["", "PMC counters, mean per launch (each pass its own run):", "",
              "| kernel | counter | mean per launch |", "|---|---|---|"]
    traffic = {}
    summed = {"kernel": [], "bytes_per_launch": 0.0, "read_bytes": 0.0, "write_bytes": 0.0}
    for k, cs in cnt.items():
        for c, v in sorted(cs.items()):
            lines.append("| %s | %s | %.6g |" % (k, c, statistics.mean(v)))
        avg_ns = next((float(r["AverageNs"]) for r in rows if short(r["Name"]) == k), None)
        fetch = statistics.mean(cs["FETCH_SIZE"]) if "FETCH_SIZE" in cs else None
        write = statistics.mean(cs["WRITE_SIZE"]) if "WRITE_SIZE" in cs else None
        derived = []
        if fetch is not None:
            rd = 2 * fetch * 1024
            derived.append("HBM read  = 2 x FETCH_SIZE = %.4g B per launch" % rd)
            if args.algo_bytes:
                derived.append("read / algorithmic input+output bytes = %.3f" % (rd / args.algo_bytes))
            if write is not None:
                wr = write * 1024
                tot = rd + wr
                derived.append("HBM write = WRITE_SIZE = %.4g B per launch" % wr)
                derived.append("HBM total = %.4g B per launch" % tot)
                if avg_ns:
                    derived.append("HBM rate (total / avg duration) = %.1f GB/s" % (tot / avg_ns))
                traffic = {"kernel": k, "bytes_per_launch": tot, "read_bytes": rd,
                           "write_bytes": wr}
                summed["kernel"].append(k)
                summed["bytes_per_launch"] += tot
                summed["read_bytes"] += rd
                summed["write_bytes"] += wr
        if "GRBM_GUI_ACTIVE" in cs and avg_ns:
            derived.append(clock_line(statistics.mean(cs["GRBM_GUI_ACTIVE"]), avg_ns))
        if "SQ_ACTIVE_INST_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            derived.append("issue-active fraction of wave cycles = %.2f" % (
                statistics.mean(cs["SQ_ACTIVE_INST_ANY"]) / statistics.mean(cs["SQ_WAVE_CYCLES"])))
        if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            derived.append("waitcnt/barrier-parked fraction = %.2f" % (
                statistics.mean(cs["SQ_WAIT_ANY"]) / statistics.mean(cs["SQ_WAVE_CYCLES"])))
        if derived:
            lines += ["", "Derived (%s):" % k, ""] + ["- " + x for x in derived]
    if args.sum_kernels and summed["kernel"]:
        summed["kernel"] = " + ".join(summed["kernel"])
        traffic = summed
        lines += ["", "Sum over the kernels of one step: HBM total = %.4g B (read %.4g, write %.4g)"
                  % (summed["bytes_per_launch"], summed["read_bytes"], summed["write_bytes"])]
    open(os.path.join(prof, args.tag + "_summary.md"), "w").write("\n".join(lines) + "\n")
    if traffic and args.plan:
        p = os.path.join(prof, "traffic.json")
        db = json.load(open(p)) if os.path.exists(p) else {}
        feats = args.features.split(",") if args.features else None
        if feats is None:
            import sys
            sys.path.insert(0, ROOT)
            import bench
            cfg = bench.CONFIGS[args.config]
            feats = cfg["feats"] if "feats" in cfg else [args.plan]
        windows = args.windows
        if windows is None:                      # bench.py's launch: the config's windows
            import sys
            sys.path.insert(0, ROOT)
            import bench
            windows = bench.CONFIGS[args.config].get("nw")
        traffic.update({"plan": args.plan, "windows": windows, "features": feats,
                        "source": "profiles/%s_summary.md" % args.tag})
        db[args.config] = traffic
        json.dump(db, open(p, "w"), indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
