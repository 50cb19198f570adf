#!/usr/bin/env python3
"""Benchmark of the sliding-window feature hot path (BASELINE.json metric).

One "step" = one fused engine pass (libmhfeat.so, mhf_window_features) over one batch
of synthetic signal already resident in HBM. Default workload = BASELINE.json
configs[1] ("cfg2"): 1e6 windows x 256 fp32 samples x 3 axes (AoS (N,3) accelerometer,
fs 50 Hz), features {mean, var, skewness, kurtosis, zero-crossings} per axis, float64
feature rows (the reference's rolling_apply output dtype, windows.py:89).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5]
                    [--strong]

N > 1: one process per GPU. Launched under torch.distributed.run (WORLD_SIZE set) it runs
as that rank and checks WORLD_SIZE == N; launched plainly it starts N ranks itself
(torch.distributed.run on 127.0.0.1) before touching the GPU.

Default (the driver's SCALE line): weak scaling over one global record: rank r owns global
windows [r*nw, (r+1)*nw) and generates their samples on its GPU from a counter-based
generator keyed by global sample (so the N-GPU run computes exactly what one GPU computes
on the N*nw-window record; SURVEY §8e: cfg4-sized data is generated per rank, no input
exchange). `value` is the compute-only step (windows are independent, no data-path
collective); `with_gather` repeats the steps with the feature-row gather to rank 0 (RCCL,
or host buffers under gloo).

--strong: one global record of nw windows originates on rank 0; every step scatters each
rank its sample slice (+ the (W - S) halo of overlapping windows, point-to-point over
RCCL), computes that shard, and gathers the feature rows back to rank 0. `value` = nw /
the whole pipeline's step time; `phases` times scatter, compute and gather on their own.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, MI355X_MICROARCH.md

# name -> (windows per rank, W, S, channels, fs, features, description)
CONFIGS = {
    "cfg2": dict(nw=1_000_000, W=256, S=256, C=3, fs=50.0, signal="accel",
                 feats=["mean", "var", "skewness", "kurtosis", "zero_crossings"],
                 band=(None, None), dom=(None, None),
                 desc="1e6 x 256-sample fp32 3-axis accel, stat moments + zero-cross"),
    "cfg3": dict(nw=10_000_000, W=256, S=256, C=1, fs=64.0, signal="ppg",
                 feats=["mean", "var", "skewness", "kurtosis", "band_power",
                        "spectral_entropy"], band=(0.5, 4.0), dom=(None, None),
                 desc="1e7 x 256-sample PPG, stat + rFFT band power + spectral entropy"),
    "cfg4": dict(nw=12_500_000, W=256, S=256, C=3, fs=50.0, signal="accel",
                 feats=["mean", "var", "std", "skewness", "kurtosis", "rms", "zero_crossings",
                        "peak_count", "band_power", "relative_band_power",
                        "spectral_entropy", "dominant_frequency"],
                 band=(0.5, 4.0), dom=(0.5, 8.0),
                 desc="1e8 x 256-sample 3-axis full feature set, 1.25e7 windows per GPU"),
    # diagnostics (not BASELINE configs): moments on overlapping windows — tile kernel
    # (W = 256, S = 128) and LDS span kernel (cfg5 geometry W = 1024, S = 128)
    "ovl256": dict(nw=10_000_000, W=256, S=128, C=1, fs=64.0, signal="ppg",
                   feats=["mean", "var", "skewness", "kurtosis"], band=(None, None),
                   dom=(None, None), desc="1e7 x 256-sample windows, stride 128, moments"),
    "cfg5m": dict(nw=2_000_000, W=1024, S=128, C=1, fs=256.0, signal="ecg",
                  feats=["mean", "var", "skewness", "kurtosis"], band=(None, None),
                  dom=(None, None), desc="2e6 x 1024-sample windows, stride 128, moments"),
    # non-power-of-two windows (the skewness / kurtosis terms divide by len(x) per element):
    # LDS span kernel, overlapping
    "ovl250": dict(nw=10_000_000, W=250, S=125, C=1, fs=64.0, signal="ppg",
                   feats=["mean", "var", "skewness", "kurtosis"], band=(None, None),
                   dom=(None, None), desc="1e7 x 250-sample windows, stride 125, moments"),
    # float64 records (pandas' default dtype, the reference's common real input): the cfg2
    # workload with every lane feature in numba's fp64 models (mhf_window_features_f64)
    "cfg2f64": dict(nw=1_000_000, W=256, S=256, C=3, fs=50.0, signal="accel", dtype="f64",
                    feats=["mean", "var", "skewness", "kurtosis", "zero_crossings"],
                    band=(None, None), dom=(None, None),
                    desc="1e6 x 256-sample float64 3-axis accel, stat moments + zero-cross"),
    # a float64 PPG record (pandas' default dtype) through cfg3's feature set: the moments in
    # numba's fp64 models, the spectral features from the fp64 transform (spectral64.hip; the
    # reference transforms a.astype(complex128), fft/_fft.py:18-28)
    "cfg3f64": dict(nw=10_000_000, W=256, S=256, C=1, fs=64.0, signal="ppg", dtype="f64",
                    feats=["mean", "var", "skewness", "kurtosis", "band_power",
                           "spectral_entropy"], band=(0.5, 4.0), dom=(None, None),
                    desc="1e7 x 256-sample float64 PPG, stat + rFFT band power + spectral entropy"),
    # time-indexed windows (nonuniform_rolling_apply / indices_rolling_apply):
    # the cfg2 record and feature set, windows [b_i, b_i+1) between jittered boundaries
    # b_i = 256 i + j(i), j(i) in [0, 16] (lengths 240-272), through mhf_indexed_window_features
    "cfgidx": dict(nw=1_000_000, W=256, S=256, C=3, fs=50.0, signal="accel", indexed=True,
                   feats=["mean", "var", "skewness", "kurtosis", "zero_crossings"],
                   band=(None, None), dom=(None, None),
                   desc="1e6 time-indexed windows (jittered boundaries, 240-272 samples) of a "
                        "fp32 3-axis accel record, stat moments + zero-cross"),
    "cfg5": dict(nw=10_000_000, W=1024, S=128, C=1, fs=256.0, signal="ecg",
                 feats=["dominant_frequency", "band_power"], band=(0.5, 40.0),
                 dom=(0.5, 40.0),
                 desc="1e7 x 1024-sample ECG, stride 128, dominant freq + band power"),
    # §8f kernels on their own: np.median over the cfg2 shapes (order_kernel),
    # information.sampen at W = 256 (sampen_kernel, O(W^2) pairs per window), and the
    # upstream preprocessing accelerometer.linear_filter = butterworth highpass 0.5 Hz order 5
    # on every axis of a 1e8-sample 3-axis record (filtfilt, iir_chunk_kernel)
    "cfg2med": dict(nw=1_000_000, W=256, S=256, C=3, fs=50.0, signal="accel",
                    feats=["median"], band=(None, None), dom=(None, None),
                    desc="1e6 x 256-sample fp32 3-axis accel, np.median per axis"),
    "cfg2ord": dict(nw=1_000_000, W=256, S=256, C=3, fs=50.0, signal="accel",
                    feats=["median", "percentile", "interquartile_range"], band=(None, None),
                    dom=(None, None),
                    desc="1e6 x 256-sample fp32 3-axis accel, np.median + np.percentile(q 50) + IQR per axis"),
    "sampen256": dict(nw=1_000_000, W=256, S=256, C=1, fs=64.0, signal="ppg",
                      feats=["sampen"], band=(None, None), dom=(None, None),
                      desc="1e6 x 256-sample PPG, information.sampen (m 2, r 0.2 sd)"),
    "filt": dict(kind="filtfilt", n=100_000_000, C=3, fs=50.0, signal="accel", cutoff=0.5,
                 order=5, ftype="highpass", W=256, S=256,
                 desc="accelerometer.linear_filter: butterworth highpass 0.5 Hz order 5 "
                      "(scipy filtfilt) of a 1e8-sample 3-axis fp32 record, float64 out"),
}

FEATURE_IDS = {
    "mean": 0, "mean32": 1, "var": 2, "var32": 3, "std": 4, "std32": 5, "skewness": 6,
    "kurtosis": 7, "kurtosis_excess": 8, "rms": 9, "zero_crossings": 10, "peak_count": 11,
    "drange": 12, "line_length": 13, "band_power": 14, "relative_band_power": 15,
    "spectral_entropy": 16, "dominant_frequency": 17,
    # §8f widened rows, for --features diagnostics (include/mhfeat.h:79-103)
    "coeff_var": 18, "hjorth_mobility": 19, "hjorth_complexity": 20,
    "min": 30, "max": 31, "median": 32, "entropy": 33, "interquartile_range": 34, "mode": 35,
    "percentile": 36, "sampen": 37, "rqa_recurrence_rate": 38, "rqa_determinism": 39,
    "rqa_laminarity": 40, "rqa_length_entropy": 41,
}


def _i64(v):
    """uint64 constant as the int64 with the same bits (torch int64 arithmetic wraps)."""
    return v - (1 << 64) if v >= 1 << 63 else v


_M1, _M2, _GOLD = _i64(0xBF58476D1CE4E5B9), _i64(0x94D049BB133111EB), _i64(0x9E3779B97F4A7C15)


def _srl(z, s):
    """logical right shift of int64 bits"""
    return (z >> s) & ((1 << (64 - s)) - 1)


def _uniform(ctr, stream):
    """splitmix64(ctr + stream * golden) -> uniform float64 in [0, 1): a counter-based
    generator, so a sample's value depends only on (seed, global sample, channel)."""
    z = ctr * _GOLD + _i64((stream * 0xD1B54A32D192ED03) % (1 << 64))
    z = (z ^ _srl(z, 30)) * _M1
    z = (z ^ _srl(z, 27)) * _M2
    z = z ^ _srl(z, 31)
    return _srl(z, 11).double() * (1.0 / (1 << 53))


def _gauss(ctr, seed):
    """Box-Muller normal deviate of counter ctr (two counter-based uniforms)."""
    u1 = 1.0 - _uniform(ctr, 2 * seed + 1)       # (0, 1]
    u2 = _uniform(ctr, 2 * seed + 2)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2 * np.pi * u2)


def synth_device(cfg, n, device, seed, first_sample=0):
    """Synthetic signal samples [first_sample, first_sample + n) (x C channels) of the
    GLOBAL record, generated on the GPU in chunks from a counter-based generator keyed by
    (seed, global sample, channel) — SURVEY §8d: a rank generating only its own window
    shard gets bit-for-bit the samples a single GPU generating the whole record would."""
    C, fs = cfg["C"], cfg["fs"]
    f64 = cfg.get("dtype") == "f64"
    fdt = torch.float64 if f64 else torch.float32
    out = torch.empty((n, C) if C > 1 else (n,), dtype=fdt, device=device)
    chunk = 1 << 24
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        s = torch.arange(first_sample + a, first_sample + b, device=device, dtype=torch.int64)
        t = s.double() / fs
        if cfg["signal"] == "accel":
            e = _gauss((s * 3)[:, None] + torch.arange(3, device=device), seed)
            out[a:b, 0] = (0.3 * torch.sin(2 * np.pi * 1.7 * t) + 0.05 * e[:, 0]).to(fdt)
            out[a:b, 1] = (0.2 * torch.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * e[:, 1]).to(fdt)
            out[a:b, 2] = (1.0 + 0.1 * torch.sin(2 * np.pi * 2.3 * t + 2)
                           + 0.05 * e[:, 2]).to(fdt)
        elif cfg["signal"] == "ppg":
            W = cfg["W"]
            w0 = s // W
            f0 = 0.8 + 2.2 * torch.frac(torch.sin(w0.double() * 12.9898) * 43758.5453).abs()
            tt = (s % W).double() / fs
            e = _gauss(s, seed)
            out[a:b] = (torch.sin(2 * np.pi * f0 * tt) + 0.5 * torch.sin(4 * np.pi * f0 * tt + 1)
                        + 0.3 * e).to(fdt)
        else:  # ecg-like: narrow pulses at ~1.2 Hz + baseline wander + noise
            ph = torch.frac(t * 1.2)
            e = _gauss(s, seed)
            out[a:b] = (torch.exp(-0.5 * ((ph - 0.5) / 0.015) ** 2)
                        + 0.2 * torch.sin(2 * np.pi * 0.3 * t) + 0.02 * e).to(fdt)
    return out


def synth_host(cfg, n, seed):
    x = _synth_host(cfg, n, seed)
    return x.astype(np.float64) if cfg.get("dtype") == "f64" else x


def _synth_host(cfg, n, seed):
    rng = np.random.default_rng(seed)
    fs, W = cfg["fs"], cfg["W"]
    t = np.arange(n) / fs
    if cfg["signal"] == "accel":
        e = rng.standard_normal((n, 3))
        return np.stack([0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * e[:, 0],
                         0.2 * np.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * e[:, 1],
                         1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2) + 0.05 * e[:, 2]],
                        axis=1).astype(np.float32)
    if cfg["signal"] == "ppg":
        f0 = rng.uniform(0.8, 3.0, n // W + 1)[np.arange(n) // W]
        tt = (np.arange(n) % W) / fs
        return (np.sin(2 * np.pi * f0 * tt) + 0.5 * np.sin(4 * np.pi * f0 * tt + 1)
                + 0.3 * rng.standard_normal(n)).astype(np.float32)
    ph = np.mod(t * 1.2, 1.0)
    return (np.exp(-0.5 * ((ph - 0.5) / 0.015) ** 2) + 0.2 * np.sin(2 * np.pi * 0.3 * t)
            + 0.02 * rng.standard_normal(n)).astype(np.float32)


def host_threads():
    """Threads for the CPU baseline: every core of this process's affinity mask, capped by
    the cgroup CPU quota when one is set (the GPU box gives a job a share of a large host:
    running more threads than the quota only time-slices them)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:                                            # cgroup v2
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        try:                                        # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, -(-q // period))
        except (OSError, ValueError):
            pass
    threads = min(aff, quota) if quota else aff
    note = "%d affinity cores%s" % (aff, ", cgroup quota %d CPUs" % quota if quota else "")
    return threads, note


IDX_JITTER = 16


def idx_boundaries(j0, count, S, xp=np):
    """Window boundaries b_j = S j + jitter(j), jitter(j) = hash32(j) mod 17 in [0, 16], for
    global boundary ids j0 .. j0 + count - 1 (numpy or torch int64 ``xp.arange`` input)."""
    if xp is np:
        j = np.arange(j0, j0 + count, dtype=np.int64)
    else:
        j = xp
    h = (j * 2654435761) & 0xFFFFFFFF            # 32-bit mix (no int64 overflow)
    h = h ^ (h >> 16)
    h = (h * 0x45D9F3B) & 0xFFFFFFFF
    h = h ^ (h >> 16)
    return S * j + h % (IDX_JITTER + 1)


def cpu_baseline(cfg, budget_s=12.0):
    """The CPU oracle (C/OpenMP restatement, oracle/) on the host cores, on a bounded
    sample of the same workload: calibrate, then run ~budget_s seconds of windows."""
    import oracle
    oracle.build()
    threads, cores_note = host_threads()
    kw = dict(fs=cfg["fs"], band=cfg["band"], dom=cfg["dom"], threads=threads)
    W, S = cfg["W"], cfg["S"]

    cache = {}

    def run(nw, reps=1):
        need = (nw - 1) * S + W + (IDX_JITTER if cfg.get("indexed") else 0)
        if cache.get("n", 0) < need:      # one synthetic record, prefixes reused
            cache["x"], cache["n"] = synth_host(cfg, need, seed=1), need
        x = cache["x"][:need]
        if cfg.get("indexed"):
            b = idx_boundaries(0, nw + 1, S)
            ind = np.stack([b[:-1], b[1:]])
        t0 = time.perf_counter()
        for _ in range(reps):
            if cfg.get("indexed"):
                oracle.indexed_features(x, ind, cfg["feats"], threads=threads,
                                        out_dtype=np.float64)
            else:
                oracle.window_features(x, W, S, cfg["feats"], **kw)
        return time.perf_counter() - t0

    # calibrate until a probe takes >= 1/10 of the budget (a 2k-window probe is dominated
    # by thread start-up), then repeat passes of n1 windows until ~budget_s have run
    n0 = min(cfg["nw"], 20000)
    dt = run(n0)
    while dt < 0.1 * budget_s and n0 < cfg["nw"]:
        n0 = min(cfg["nw"], n0 * 4)
        dt = run(n0)
    n1 = int(min(cfg["nw"], max(n0, 0.25 * budget_s / max(dt, 1e-6) * n0)))
    reps, dt = 0, 0.0
    while dt < budget_s:
        dt += run(n1)
        reps += 1
    n1 *= reps
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": n1 / dt, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": "%d windows (%d pass(es)) of %s (oracle/mhf_oracle.c, %d OpenMP threads "
                      "= %s, %s), %.1f s" % (n1, reps, cfg["desc"], threads, cores_note, cpu,
                                             dt)}


def load_traffic(config, plan, windows, features):
    """HBM bytes per launch from the rocprofv3 PMC pass committed under profiles/, if it
    was taken on this exact workload (config, kernel plan, windows per launch, feature
    set — a different feature set can add kernels or change the variant)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        rec = json.load(open(p)).get(config)
    except (OSError, ValueError):
        return None
    if (not rec or rec.get("plan") != plan or rec.get("windows") != windows
            or rec.get("features") != list(features)):
        return None
    return rec.get("bytes_per_launch")


def launch_ranks(n):
    """Run this script as N ranks of ``torch.distributed.run`` on this node (master on
    127.0.0.1, a free port) with the same arguments; returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % n, "--master-addr=127.0.0.1", "--master-port=%d" % port,
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def run_filtfilt(args, rank, world, device, dist):
    """--config filt: zero-phase Butterworth (scipy.signal.filtfilt, generic/filters.py:7-35)
    of every axis of a 1e8-sample record per rank (independent records: weak scaling),
    through mhf_filtfilt (two iir_chunk_kernel passes, fp64 recurrence). Algorithmic bytes
    per sample-channel: 4 in + 8 out (float64, the reference's np.zeros(acc.shape)) + 16 for
    the fp64 forward pass written and read back (the backward pass needs all of it)."""
    from scipy import signal
    from pymhealth_amd import engine
    cfg = dict(CONFIGS[args.config])
    n = args.windows or cfg["n"]
    C = cfg["C"]
    x = synth_device(cfg, n, device, seed=1234, first_sample=rank * n)
    b, a = signal.butter(cfg["order"], cfg["cutoff"] / (0.5 * cfg["fs"]), cfg["ftype"])
    zi = signal.lfilter_zi(b, a)
    out = torch.empty((n, C), dtype=torch.float64, device=device)

    def step():
        engine.filtfilt(x, b, a, zi, out=out)

    for _ in range(args.warmup):
        step()
    stream = torch.cuda.current_stream(device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()

    def timed_steps():
        for k in range(args.steps):
            ev[k][0].record(stream)
            step()
            ev[k][1].record(stream)

    elapsed = _timed(timed_steps, 1, dist, device)
    kernel_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
    bytes_launch = n * C * (4 + 8 + 16)
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    # the per-lane kernel (opt-out, other channel counts) has no committed PMC pass
    per_lane = os.environ.get("MHF_NO_IIR_TILE") == "1" or C not in (1, 3)
    if rank == 0:
        res = {
            "metric": "samples/sec (%s)" % cfg["desc"],
            "value": n * C * world * args.steps / elapsed,
            "unit": "samples/s (sample-channels)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (on-device generated accel signal)",
            "config": {"workload": args.config, "description": cfg["desc"], "samples_per_gpu": n,
                       "channels": C,
                       "kernel": "iir_chunk_kernel x2 (filtfilt)" if per_lane else "iir_tile_kernel x2 (filtfilt)",
                       "parallelism": "independent records x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (None if per_lane else load_traffic(args.config, "filtfilt", n, ["filtfilt"])),
                         "algorithmic_bytes_per_launch": bytes_launch, "kernel_ms": kernel_ms},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_filtfilt(cfg, b, a, zi)
        print(json.dumps(res), flush=True)


def cpu_baseline_filtfilt(cfg, b, a, zi, budget_s=10.0):
    """The oracle's C restatement of scipy's filtfilt (oracle/mhf_oracle.c, serial: one core,
    axis by axis as the reference's linear_filter loops) on a bounded prefix of the record."""
    import oracle
    oracle.build()
    n = 20000
    x = synth_host(cfg, n, seed=1)
    t0 = time.perf_counter()
    oracle.filtfilt(b, a, x, zi)
    dt = time.perf_counter() - t0
    n = int(min(cfg["n"], max(n, n * 0.5 * budget_s / max(dt, 1e-6))))
    x = synth_host(cfg, n, seed=1)
    t0 = time.perf_counter()
    oracle.filtfilt(b, a, x, zi)
    dt = time.perf_counter() - t0
    return {"value": n * cfg["C"] / dt, "unit": "samples/s (sample-channels)", "cores": 1,
            "kind": "port",
            "sample": "%d x %d-axis samples (oracle/mhf_oracle.c mhf_oracle_filtfilt, serial), "
                      "%.1f s" % (n, cfg["C"], dt)}


def _timed(fn, steps, dist, device):
    """Seconds for `steps` calls of fn between barrier + synchronize on both sides, the
    maximum over ranks (the job ends when the slowest rank does)."""
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def run_strong(args, rank, world, device, dist):
    """--strong ("scatter of input batches when data originate on one device"):
    the nw-window record lives on rank 0; a step = scatter_signal (point-to-point slices with
    halos) -> the rank's fused launch over its global windows -> gather_features to rank 0.
    The pipeline is timed as a whole (`value`), then each phase on its own (`phases`)."""
    from pymhealth_amd.distributed import (gather_features, sample_range, scatter_signal,
                                           shard_range)
    from pymhealth_amd.engine import num_windows
    cfg = dict(CONFIGS[args.config])
    if cfg.get("indexed"):
        raise SystemExit("--strong takes fixed-window configs")
    if args.windows:
        cfg["nw"] = args.windows
    if args.features:
        cfg["feats"] = args.features.split(",")
    workload = "strong-%s" % args.config
    if cfg["feats"] != CONFIGS[args.config]["feats"] or cfg["nw"] != CONFIGS[args.config]["nw"]:
        workload = "strong-diag-%s" % args.config
        cfg["desc"] = "%d x %d-sample windows, stride %d, %d channel(s), %s signal; features: %s" % (
            cfg["nw"], cfg["W"], cfg["S"], cfg["C"], cfg["signal"], ", ".join(cfg["feats"]))
    W, S, C, nw = cfg["W"], cfg["S"], cfg["C"], cfg["nw"]
    n = (nw - 1) * S + W
    f64 = cfg.get("dtype") == "f64"
    dtype = torch.float64 if f64 else torch.float32
    ids = [FEATURE_IDS[f] for f in cfg["feats"]]
    out_dtype = torch.float32 if args.out_dtype == "f32" else torch.float64
    x = synth_device(cfg, n, device, seed=1234) if rank == 0 else None
    w0, w1 = shard_range(num_windows(n, W, S), rank, world)
    kw = dict(fs=cfg["fs"], band=cfg["band"], dom=cfg["dom"], out_dtype=out_dtype,
              first_window=w0, n_windows=w1 - w0, base_window=w0)
    state = {}

    def scatter():
        # one rank: the record is already where its windows are computed
        state["local"] = (scatter_signal(x, n, W, S, device=device, channels=C, dtype=dtype)[0]
                          if dist else x)

    def compute():
        if args.dry_run:   # CPU test hook: rows of the right shape, no engine call
            state["out"] = torch.zeros((C, len(ids), w1 - w0), dtype=out_dtype)
            return
        from pymhealth_amd import engine
        state["out"] = engine.window_features(state["local"], W, S, ids, **kw)

    def gather():
        state["rows"] = gather_features(state["out"], nw) if dist else state["out"]

    def step():
        scatter()
        compute()
        gather()

    for _ in range(args.warmup):
        step()
    elapsed = _timed(step, args.steps, dist, device)
    phases = {name: _timed(fn, args.steps, dist, device) * 1e3 / args.steps
              for name, fn in (("scatter_ms", scatter), ("compute_ms", compute),
                               ("gather_ms", gather))}
    if rank == 0:
        assert state["rows"].shape == (C, len(ids), nw)
        sent = 0                                   # samples rank 0 sends (slices + halos)
        for r in range(1, world):
            a0, a1 = shard_range(num_windows(n, W, S), r, world)
            b0, b1 = sample_range(a0, a1, W, S)
            sent += b1 - b0
        in_bytes = sent * C * (8 if f64 else 4)
        res = {
            "metric": "windows/sec (strong scaling: %s)" % cfg["desc"],
            "value": nw * args.steps / elapsed,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if f64 else "f32",
            "data": "synthetic (%s signal generated on rank 0)" % cfg["signal"],
            "config": {"workload": workload, "description": cfg["desc"],
                       "windows_total": nw, "wsize": W, "wstep": S, "channels": C,
                       "features": cfg["feats"], "out_dtype": args.out_dtype,
                       "parallelism": "record on rank 0 -> %d window shards (scatter with "
                                      "(W - S) halos) -> rows gathered to rank 0" % world,
                       "backend": args.backend if world > 1 else None},
            "phases": dict(phases, scatter_bytes_from_rank0=in_bytes,
                           gather_bytes_to_rank0=(nw - (w1 - w0)) * C * len(ids) *
                           (4 if out_dtype == torch.float32 else 8)),
            "roofline": None,
            "cpu_baseline": None,
        }
        if args.dry_run:
            res["dry_run"] = "collectives only on host tensors (gloo); no GPU, no feature compute"
        print(json.dumps(res), flush=True)


# VALU issue peak of the MI355X (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs x 16 lanes per
# cycle for a plain (non-packed) 32-bit VALU op (a wave64 instruction every 4 cycles per
# SIMD) at 2.4 GHz = 39.3e12 lane-ops/s
VALU_LANE_OPS = 256 * 4 * 16 * 2.4e9


# One wave per SIMD (the register tiles and spectral_reg's issue-bound rate): a wave64 VALU
# instruction issues every 4 cycles at best (MI355X_MICROARCH.md, 'vector-instruction ISSUE
# cost': v_add_f32 / v_fma_f32 / v_pk_* 4, the transcendentals 8), so the chip's issue
# peak for such kernels is 1024 SIMDs x 2.4 GHz / 4 wave-instructions per second.
WAVE_ISSUE_PEAK = 1024 * 2.4e9 / 4


def lane_fft_pk(W):
    """v_pk instructions of the in-lane rFFT of W real samples (spectral_lane.hip.inc): an
    N = W / 2 point complex FFT of radix-4 DIF stages (+ one radix-2 stage when log2 N is
    odd) — 8 packed complex adds / FMAs per butterfly, 2 v_pk per twiddle at a general
    angle, 1 for -i, +i or -1 — then the real-FFT split of the bin pairs (k, N - k): 8 v_pk
    per pair at a general twiddle, 7 for pair N / 2."""
    N = W // 2
    def cost(m):                      # twiddle exp(-2 pi i m / W)
        m %= W
        return 0 if m == 0 else (1 if 4 * m in (W, 3 * W) or 2 * m == W else 2)
    ops, L = 0, N
    while L >= 4:
        H, S = L // 4, W // L
        for j in range(H):
            per = 8 + cost(j * S) + cost(2 * j * S) + cost(3 * j * S)
            ops += per * (N // L)
        L //= 4
    if L == 2:
        ops += 2 * (N // 2)
    post = sum(6 + cost(k) for k in range(1, N // 2 + 1))     # E2, O2, re, im, pp (2) + twiddle
    return ops, post


def tile_valu_floor(cfg):
    """Instruction floor of the register-tile kernel for one (window, channel) lane = wave
    instructions per 64-unit tile: what the reference's models need
    with one lane per window-channel, the fewest instructions each operation takes on CDNA4
    — not a measurement of the current code.
      pass 1 (reference order): the fp32 sum, W adds; zero crossings 2 / sample (compare,
        carry-add; the mask xor is SALU); RMS 2 (mul, add: fp32 chain); peaks 3;
      pass 2 (exact): per sample pair 6 v_pk (d, q = d^2, d q, q^2, the two
        / W scalings) and per sample 4 sequential chain ops (cvt + fp64 add of array_var's
        sum, the fp32 skewness and kurtosis adds) — 7 W; rows >= 1 of np.var / np.std need
        nothing more (fast var; the exact replay would add 4 W);
      the window in the register file: 192 VGPRs + 64 AGPRs per lane, so 64 accvgpr writes
        (pass 1) and 64 reads (pass 2), and with spectral features 64 writes + 64 reads of
        the sub-FFT the split FFT parks there;
      spectral: the rFFT and split (lane_fft_pk); band power 1 v_pk per bin pair; the total
        power in fp64 (cvt + add per bin: the entropy's log1p correction needs it); entropy:
        the largest bin (v_max3 per pair), q = p / T + 1e-30 (1 v_pk per pair), ln q (v_log,
        8 cycles = 2 issue slots, per bin), q ln q summed (1 v_pk per pair); dominant
        frequency: a weighted key and a v_max_f64 per bin (3 per bin)."""
    W = cfg["W"]
    f = set(cfg["feats"])
    n = W
    p1 = W * (1 + (2 if "zero_crossings" in f else 0) + (2 if "rms" in f else 0)
              + (3 if "peak_count" in f else 0))
    p2 = 7 * W if f & {"var", "std", "skewness", "kurtosis", "kurtosis_excess"} else 0
    NA = 64 if W > 128 else 0
    acc = 2 * NA
    spec = 0
    spectral = f & {"band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"}
    if spectral:
        fft, post = lane_fft_pk(W)
        NP = W // 4 + 1
        spec = fft + post + 2 * 2 * NP                  # transform, split, fp64 total
        if f & {"band_power", "relative_band_power"}:
            spec += NP
        if "spectral_entropy" in f:
            spec += NP + NP + 2 * (W // 2 + 1) + NP       # max3, q, ln (x2), q ln q
        if "dominant_frequency" in f:
            spec += 3 * (W // 2 + 1)
        acc += 2 * NA
    return {"pass1": p1, "pass2": p2, "register_file": acc, "spectral": spec,
            "total": p1 + p2 + acc + spec}


def tile_valu_roofline(cfg, nw, C, kernel_ms, plan):
    """roofline_valu of the register-tile kernels: the instruction floor
    (tile_valu_floor) of a launch over the issue peak of one wave per SIMD."""
    if not plan.startswith("tile_w"):
        return None
    fl = tile_valu_floor(cfg)
    tiles = -(-nw * C // 64) if C == 1 else -(-nw // (64 // C))
    work = fl["total"] * tiles                     # wave-instructions per launch
    t = kernel_ms * 1e-3
    return {"bound": "valu", "achieved": work / t, "peak": WAVE_ISSUE_PEAK,
            "unit": "wave-instructions/s (floor count)", "frac": work / t / WAVE_ISSUE_PEAK,
            "floor_per_lane": fl, "floor_wave_instructions_per_launch": work,
            "floor_ms_at_peak": work / WAVE_ISSUE_PEAK * 1e3, "kernel_ms": kernel_ms}


# spectral_reg (W = 1024, one wave per window): LDS bytes per window of its design
#  — the ring reads of the window (4 KiB), two transposes of 512 complex
# fp32 points written and read back (2 x 2 x 4 KiB), the real-split partner permutes
# (~1.5 KiB) — against 256 CUs x 256 B/clk x 2.4 GHz (MI355X_MICROARCH.md §LDS).
LDS_PEAK_GBS = 256 * 256 * 2.4
SPECREG_LDS_BYTES = 4096 + 2 * 2 * 4096 + 1536


def valu_roofline(cfg, nw, C, kernel_ms):
    """roofline for the compute-bound §8f kernels:
      sampen — pair tests |x[j] - x[i]| < r, W (W - 1) / 2 per window-channel; the floor is
               2.5 lane-ops per test (half a v_pk_add_f32 for the fp32 difference, the
               compare, the match-bit insert of the match-word walk, order.hip
               sampen_cyclic);
      mode (order_kernel, sorting) — bitonic compare-exchanges, N log2 N (log2 N + 1) / 4
               per window-channel (N = the padded power of two); the floor is 4 lane-ops
               per compare-exchange (min, max and a select per key);
      median / percentile / IQR without mode (order_kernel's rank selection) — key
               compares of the bit-serial count search MODEL, N log2 N per rank searched
               (log2 N halving steps over all N keys; median and percentile search one
               rank, IQR two) — a model of the work, not a lower bound: the kernel's
               interpolated range search takes ~7.1 steps at N = 256 on average (DESIGN
               §5.5); 1 lane-op per compare (the ballot's v_cmp; its popcount
               is a scalar op issued beside it).
    achieved / peak in operations per second."""
    W = cfg["W"]
    feats = set(cfg["feats"])
    t = kernel_ms * 1e-3
    if feats == {"sampen"}:
        work, per, unit = nw * C * W * (W - 1) / 2.0, 2.5, "pair tests/s"
    elif feats and feats <= {"median", "percentile", "interquartile_range", "mode"}:
        N = 1 << max(6, (W - 1).bit_length())
        lg = N.bit_length() - 1
        if "mode" in feats:
            work, per, unit = nw * C * N * lg * (lg + 1) / 4.0, 4.0, "compare-exchanges/s"
        else:
            ranks = ("median" in feats) + ("percentile" in feats) + 2 * ("interquartile_range" in feats)
            work, per, unit = nw * C * ranks * N * lg, 1.0, "key compares/s (bit-search model)"
    else:
        return None
    peak = VALU_LANE_OPS / per
    return {"bound": "valu", "achieved": work / t, "peak": peak, "unit": unit,
            "frac": work / t / peak, "traffic": None, "work_per_launch": work,
            "lane_ops_per_unit_floor": per, "kernel_ms": kernel_ms}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--out-dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--windows", type=int, default=0, help="override windows per rank")
    ap.add_argument("--features", default="",
                    help="diagnostics: comma-separated feature names replacing the config's")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL on ROCm)")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: start the ranks, join a gloo group, print the world, "
                         "exit before any GPU call")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: one global record of nw windows on rank 0, scattered "
                         "to the ranks, features per rank, rows gathered back (SURVEY §8e)")
    ap.add_argument("--dry-run", action="store_true",
                    help="test hook for --strong on a CPU host (gloo): the scatter / gather "
                         "collectives on host tensors, no GPU and no feature compute")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch: N fresh rank processes, started before this process touches the GPU
        # (it only waits for them; rank 0 prints the JSON line to the inherited stdout)
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d (one process per GPU: launch with "
              "--nproc-per-node %d, or without WORLD_SIZE to self-launch)"
              % (args.gpus, world, args.gpus), file=sys.stderr)
        sys.exit(2)
    if args.launch_check:
        import torch.distributed as tdist
        if world > 1:
            tdist.init_process_group("gloo")
            ranks = [None] * world
            tdist.all_gather_object(ranks, int(os.environ.get("RANK", "0")))
            tdist.destroy_process_group()
        else:
            ranks = [0]
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": ranks}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run and not (args.strong and args.backend == "gloo"):
        ap.error("--dry-run is the CPU test hook of --strong --backend gloo")
    if args.dry_run:
        device = torch.device("cpu")
    else:
        # one process per GPU; (rehearsal only: more ranks than GPUs share devices round-robin)
        device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    if args.strong:
        run_strong(args, rank, world, device, dist)
        if dist:
            dist.destroy_process_group()
        return
    if CONFIGS[args.config].get("kind") == "filtfilt":
        run_filtfilt(args, rank, world, device, dist)
        if dist:
            dist.destroy_process_group()
        return

    from pymhealth_amd import engine

    cfg = dict(CONFIGS[args.config])
    workload = args.config
    if args.windows:
        cfg["nw"] = args.windows
    if args.features:
        cfg["feats"] = args.features.split(",")
    # an override makes it a diagnostic run: its line names what actually ran and never
    # carries a BASELINE metric or a config description it does not match
    diagnostic = (cfg["feats"] != CONFIGS[args.config]["feats"]
                  or cfg["nw"] != CONFIGS[args.config]["nw"])
    if diagnostic:
        workload = "diag-%s" % args.config
        cfg["desc"] = "%d x %d-sample windows, stride %d, %d channel(s), %s signal; features: %s" % (
            cfg["nw"], cfg["W"], cfg["S"], cfg["C"], cfg["signal"], ", ".join(cfg["feats"]))
    W, S, C, nw = cfg["W"], cfg["S"], cfg["C"], cfg["nw"]
    # weak scaling over one GLOBAL record: rank r owns global windows [r*nw, (r+1)*nw) and
    # generates exactly their samples (plus the (W - S) halo of overlapping windows) from
    # the counter-based generator, so N ranks compute what one GPU would on the N*nw-window
    # record, bit for bit (global window 0, on rank 0, keeps the serial row-0 numerics)
    w0 = rank * nw
    indexed = bool(cfg.get("indexed"))
    n = (nw - 1) * S + W + (IDX_JITTER if indexed else 0)
    x = synth_device(cfg, n, device, seed=1234, first_sample=w0 * S)
    ids = [FEATURE_IDS[f] for f in cfg["feats"]]
    out_dtype = torch.float32 if args.out_dtype == "f32" else torch.float64
    out = torch.empty((C, len(ids), nw), dtype=out_dtype, device=device)
    kw = dict(fs=cfg["fs"], band=cfg["band"], dom=cfg["dom"], out_dtype=out_dtype, out=out,
              first_window=w0, n_windows=nw, base_window=w0)
    f64 = cfg.get("dtype") == "f64"
    stream = torch.cuda.current_stream(device)
    if indexed:
        # this rank's windows: global boundaries w0 .. w0 + nw, relative to its first sample
        b = idx_boundaries(0, 0, S, xp=torch.arange(w0, w0 + nw + 1, dtype=torch.int64,
                                                    device=device)) - w0 * S
        idx = torch.stack([b[:-1], b[1:]]).contiguous()
        covered = int((b[-1] - b[0]).item())
        plan = engine.plan_name_indexed((C, 1 if C > 1 else 0, C), ids)

        def step():
            engine.indexed_window_features(x, idx, ids, out_dtype=out_dtype, out=out)
    else:
        plan = (engine.plan_name_f64((C, 1 if C > 1 else 0, C), W, S, ids, out_dtype) if f64
                else engine.plan_name((C, 1 if C > 1 else 0, C), W, S, ids, out_dtype))

        def step():
            engine.window_features(x, W, S, ids, **kw)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # the same steps followed by the feature-row gather to rank 0 over RCCL (SURVEY §8e:
    # "with and without the gather"); N = 1 has nothing to gather
    gather_elapsed = None
    if dist:
        from pymhealth_amd.distributed import gather_features
        gather_features(out, nw * world)               # warm the collective
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
            gather_features(out, nw * world)
        torch.cuda.synchronize()
        dist.barrier()
        gather_elapsed = time.perf_counter() - t1

    t = torch.tensor([elapsed, kernel_ms, gather_elapsed or 0.0], dtype=torch.float64,
                     device=device if args.backend == "nccl" else "cpu")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)     # the job ends when the slowest rank does
    elapsed, kernel_ms_max = float(t[0].item()), float(t[1].item())
    if gather_elapsed is not None:
        gather_elapsed = float(t[2].item())

    if indexed:   # every covered sample once + the feature rows
        bytes_launch = 4 * C * covered + nw * C * len(ids) * (4 if out_dtype == torch.float32 else 8)
    else:
        bytes_launch = engine.algorithmic_bytes(n, C, W, S, nw, len(ids), out_dtype,
                                                sample_bytes=8 if f64 else 4)
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    if rank == 0:
        windows_total = nw * world * args.steps
        res = {
            "metric": "windows/sec (256-sample fp32, 3-axis) at 1/2/4/8 GPUs; % HBM roofline"
            if args.config == "cfg2" and not diagnostic
            else "windows/sec (%s%s)" % ("diagnostic: " if diagnostic else "", cfg["desc"]),
            "value": windows_total / elapsed,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if f64 else "f32",
            "data": "synthetic (on-device generated %s signal)" % cfg["signal"],
            "config": {"workload": workload, "description": cfg["desc"],
                       "windows_per_gpu": nw, "wsize": W, "wstep": S, "channels": C,
                       "features": cfg["feats"], "out_dtype": args.out_dtype,
                       "kernel": plan, "parallelism": "window shards x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": load_traffic(workload, plan, nw, cfg["feats"]),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "kernel_ms": kernel_ms, "kernel_ms_max_over_ranks": kernel_ms_max},
            "cpu_baseline": None,
        }
        if gather_elapsed is not None:
            res["with_gather"] = {
                "value": windows_total / gather_elapsed,
                "ms_per_step": gather_elapsed * 1e3 / args.steps,
                "backend": args.backend,
                "note": "each step also gathers every rank's (C, F, nw) feature rows to rank "
                        "0 (distributed.gather_features, one %s gather)"
                        % ("RCCL" if args.backend == "nccl" else "gloo (host buffers)")}
        spectral = {"band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"}
        if spectral & set(cfg["feats"]):
            # secondary: rFFT work at 2.5 W log2 W flop per window-channel vs the
            # fp32 vector peak (MI355X_MICROARCH.md) — cfg5 is FFT/VALU-bound, not HBM-bound
            fft_flop = nw * C * 2.5 * W * np.log2(W)
            res["compute"] = {"fft_tflops": fft_flop / (kernel_ms * 1e-3) / 1e12,
                              "peak_tflops_fp32_vector": 157.3,
                              "frac": fft_flop / (kernel_ms * 1e-3) / 1e12 / 157.3,
                              "flop_per_window_channel": 2.5 * W * np.log2(W)}
            if plan.startswith("spectral_reg"):
                lds = nw * C * SPECREG_LDS_BYTES / (kernel_ms * 1e-3) / 1e9
                res["compute"].update({"lds_gbs": lds, "lds_peak_gbs": LDS_PEAK_GBS,
                                       "lds_frac": lds / LDS_PEAK_GBS,
                                       "lds_bytes_per_window": SPECREG_LDS_BYTES})
        tv = tile_valu_roofline(cfg, nw, C, kernel_ms, plan)
        if tv is not None:
            res["roofline_valu"] = tv
        valu = valu_roofline(cfg, nw, C, kernel_ms)
        if valu is not None:
            # the pairwise / sorting kernels are VALU-issue-bound, not HBM-bound: the headline
            # roofline becomes the work rate against the VALU peak; the HBM figures stay
            res["roofline_hbm"] = res["roofline"]
            res["roofline"] = valu
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
