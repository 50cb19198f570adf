#!/usr/bin/env python3
"""README performance table from committed bench lines: one row per workload, every number
read from the JSON line of profiles/<prefix>_bench_<config>.log (the file is cited in the
row). Usage: python tools/readme_table.py r06i > /tmp/table.md"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ROWS = [
    ("default", "cfg2: 1e6 × 256 × 3-axis, moments + zero crossings (bench default)"),
    ("cfg2f64", "cfg2f64: cfg2 on a float64 record (`tile64_kernel`)"),
    ("cfg3", "cfg3: 1e7 × 256 PPG, moments + band power + spectral entropy"),
    ("cfg3f64", "cfg3f64: cfg3 on a float64 record (`spectral64_kernel`)"),
    ("cfg4", "cfg4: 1.25e7 × 256 × 3-axis, full feature set"),
    ("cfg5", "cfg5: 1e7 × 1024 ECG, stride 128, dominant frequency + band power"),
    ("cfgidx", "cfgidx: 1e6 time-indexed windows (240–272 samples) × 3-axis, cfg2 features (`tile_idx`)"),
    ("ovl250", "ovl250: 1e7 × 250, stride 125, moments (`tile_fix`, union-span image)"),
    ("filt", "filt: butterworth filtfilt of a 1e8-sample 3-axis record (LDS-streamed passes)"),
    ("cfg2med", "cfg2med: np.median over cfg2 shapes (range selection, `order_sel_kernel`)"),
    ("cfg2ord", "cfg2ord: median + percentile + IQR over cfg2 shapes (`order_sel_kernel`)"),
    ("sampen256", "sampen256: information.sampen, 1e6 × 256 (cyclic-diagonal match-word walk)"),
    ("cfg5m", "cfg5m (diagnostic): 2e6 × 1024, stride 128, moments (span kernel)"),
    ("ovl256", "ovl256 (diagnostic): 1e7 × 256, stride 128, moments"),
]


def fmt(x):
    return "%.3g" % x


def roofline(d):
    r = d.get("roofline") or {}
    parts = []
    if r:
        if r.get("unit") == "GB/s":
            parts.append("%.2f TB/s (%d %% of 8 TB/s)" % (r["achieved"] / 1e3, round(100 * r["frac"])))
        else:
            parts.append("%s %s (frac %.2f, %s-bound)" % (fmt(r["achieved"]), r.get("unit", ""), r["frac"],
                                                         r.get("bound", "")))
        tr, ab = r.get("traffic"), r.get("algorithmic_bytes_per_launch")
        if tr and ab:
            parts.append("PMC traffic %.2f ×" % (tr / ab))
    rv = d.get("roofline_valu")
    if rv:
        parts.append("VALU floor frac %.2f" % rv["frac"])
    return "; ".join(parts)


def main():
    prefix = sys.argv[1]
    print("| workload | kernel time | windows/s | roofline | CPU oracle (threads) | line |")
    print("|---|---|---|---|---|---|")
    for cfg, desc in ROWS:
        p = os.path.join(ROOT, "profiles", "%s_bench_%s.log" % (prefix, cfg))
        if not os.path.exists(p):
            print("| %s | not measured | | | | |" % desc)
            continue
        lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
        d = json.loads(lines[-1])
        r = d.get("roofline") or {}
        kms = r.get("kernel_ms", d.get("ms_per_step"))
        cb = d.get("cpu_baseline") or {}
        cpu = "%s %s (%s)" % (fmt(cb["value"]), cb.get("unit", ""), cb.get("cores")) if cb else "—"
        print("| %s | %.3f ms | %s %s | %s | %s | `profiles/%s` |" % (
            desc, kms, fmt(d["value"]), d.get("unit", ""), roofline(d), cpu, os.path.basename(p)))


if __name__ == "__main__":
    main()
