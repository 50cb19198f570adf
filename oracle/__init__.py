"""CPU parity oracle for the sliding-window feature engine.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
`cpu_baseline` leg of bench.py, never by the product package `pymhealth_amd`.
See oracle/mhf_oracle.c for the reference file:line each model restates.
"""
from .oracle import (FEATURE_IDS, PSD_OPS, build, filtfilt, get_indices,  # noqa: F401
                     indexed_features, psd_features,
                     load, magnitude, num_windows, periodogram, window_features,
                     zc_threshold32, roll, pitch, gradient, zero_crossings, magnitude_dot,
                     find_peaks)
