"""ctypes binding of libmhfeat.so (include/mhfeat.h).

The product has exactly one compute path: the HIP kernels in this library. If the
library is missing, or no GPU is visible, every entry point raises — there is no
CPU fallback anywhere in ``pymhealth_amd``.
"""
import ctypes
import math
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# MHF_LIB: diagnostics only (A/B builds of the same sources, e.g. a cache-policy variant);
# honoured only with MHF_DIAGNOSTICS=1, like the library's own switches
LIB_PATH = ((os.environ.get("MHF_LIB") if os.environ.get("MHF_DIAGNOSTICS") == "1" else None)
            or os.path.join(HERE, "libmhfeat.so"))

# include/mhfeat.h `mhf_feature`
MHF_MEAN = 0
MHF_MEAN32 = 1
MHF_VAR = 2
MHF_VAR32 = 3
MHF_STD = 4
MHF_STD32 = 5
MHF_SKEWNESS = 6
MHF_KURTOSIS = 7
MHF_KURTOSIS_EXCESS = 8
MHF_RMS = 9
MHF_ZERO_CROSSINGS = 10
MHF_PEAK_COUNT = 11
MHF_DRANGE = 12
MHF_LINE_LENGTH = 13
MHF_BAND_POWER = 14
MHF_REL_BAND_POWER = 15
MHF_SPECTRAL_ENTROPY = 16
MHF_DOMINANT_FREQ = 17
MHF_COEFF_VAR = 18
MHF_HJORTH_MOBILITY = 19
MHF_HJORTH_COMPLEXITY = 20
MHF_RMSSD = 21
MHF_SDSD = 22
MHF_SSD = 23
MHF_PNNX = 24
MHF_CSI_SD1 = 25
MHF_CSI_SD2 = 26
MHF_LORENZ_CSI = 27
MHF_LORENZ_CVI = 28
MHF_LORENZ_MCSI = 29
MHF_MIN = 30
MHF_MAX = 31
MHF_MEDIAN = 32
MHF_ENTROPY = 33
MHF_IQR = 34
MHF_MODE = 35
MHF_PERCENTILE = 36
MHF_SAMPEN = 37
MHF_RQA_RR = 38
MHF_RQA_DET = 39
MHF_RQA_LAM = 40
MHF_RQA_ENT = 41
MHF_NUM_FEATURES = 42
ORDER_IDS = frozenset((MHF_MEDIAN, MHF_IQR, MHF_MODE, MHF_PERCENTILE, MHF_SAMPEN))
RQA_IDS = frozenset((MHF_RQA_RR, MHF_RQA_DET, MHF_RQA_LAM, MHF_RQA_ENT))
MAX_RQA_W = 8191             # mhfeat.hip: (2 W + 2) words of LDS per window
MAX_RQA_W_F64 = 5460         # float64 records: (3 W + 2) words
MAX_ORDER_SAMPLES = 16384   # engine_common.h kMaxOrderSamples (window length x channels)
CSI_IDS = frozenset((MHF_CSI_SD1, MHF_CSI_SD2, MHF_LORENZ_CSI, MHF_LORENZ_CVI,
                     MHF_LORENZ_MCSI))
CSI_FACTOR = 0.70710678118654746    # 1 / np.sqrt(2): csi_sd1/2's default (hrv.py:208,221)
SPECTRAL_IDS = frozenset((MHF_BAND_POWER, MHF_REL_BAND_POWER, MHF_SPECTRAL_ENTROPY,
                          MHF_DOMINANT_FREQ))

MHF_ABI_VERSION = 7   # include/mhfeat.h MHF_ABI_VERSION
MHF_OUT_F64 = 0
MHF_OUT_F32 = 1
MHF_NUMERICS_REFERENCE = 0
MHF_NUMERICS_EXACT_VAR = 1   # OR-ed in: bit-exact rows >= 1 of np.var / np.std on the tiles
MHF_BOUNDS_FLOAT_STARTS = 1
MHF_BOUNDS_FLOAT_ENDS = 2
# include/mhfeat.h `mhf_psd_op`
MHF_PSD_POWER_BAND = 0
MHF_PSD_REL_POWER_BAND = 1
MHF_PSD_PEAK_FREQUENCY = 2
MHF_PSD_PEAK_FREQUENCY_HRV = 3
MHF_PSD_ENTROPY = 4
MHF_PSD_NUM_OPS = 5
MHF_DTYPE_F32 = 0
MHF_DTYPE_F64 = 1
MHF_DTYPE_I32 = 2
MHF_DTYPE_I64 = 3
MHF_CMP_GREATER = 0
MHF_CMP_GREATER_EQUAL = 1
MHF_CMP_LESS = 2
MHF_CMP_LESS_EQUAL = 3
MHF_FFT_FORWARD = -1
MHF_FFT_BACKWARD = 1
MHF_ROLL = 0
MHF_PITCH = 1

ERRORS = {-1: ValueError, -2: NotImplementedError, -3: RuntimeError}

EXPORTS = ("mhf_version", "mhf_last_error", "mhf_num_windows", "mhf_window_features",
           "mhf_window_features_f64",
           "mhf_algorithmic_bytes", "mhf_plan_name", "mhf_plan_name_f64",
           "mhf_indexed_window_features",
           "mhf_indexed_window_features_f64",
           "mhf_window_bounds", "mhf_filtfilt", "mhf_magnitude", "mhf_psd_features",
           "mhf_orientation", "mhf_gradient", "mhf_zero_crossings", "mhf_magnitude_dot",
           "mhf_find_peaks_workspace", "mhf_find_peaks", "mhf_find_peaks_cmp", "mhf_minmax",
           "mhf_fft", "mhf_indexed_workspace", "mhf_filtfilt_workspace",
           "mhf_magnitude_dot_workspace", "mhf_minmax_workspace", "mhf_fft_workspace",
           "mhf_plan_name_indexed")


class Params(ctypes.Structure):
    """`mhf_params` (include/mhfeat.h)."""
    _fields_ = [("fs", ctypes.c_double), ("band_lo", ctypes.c_double),
                ("band_hi", ctypes.c_double), ("dom_lo", ctypes.c_double),
                ("dom_hi", ctypes.c_double), ("zc_threshold", ctypes.c_double),
                ("pnn_threshold", ctypes.c_double), ("csi_factor", ctypes.c_double),
                ("percentile_q", ctypes.c_double), ("sampen_m", ctypes.c_double),
                ("sampen_r", ctypes.c_double), ("sampen_sd", ctypes.c_double),
                ("rqa_radius", ctypes.c_double), ("rqa_minlen", ctypes.c_double)]


def make_params(fs=None, band=(None, None), dom=(None, None), zc_threshold=0.0,
                pnn_threshold=50.0, csi_factor=CSI_FACTOR, percentile_q=50.0, sampen_m=2,
                sampen_r=0.2, sampen_sd=None, rqa_radius=0.0, rqa_minlen=2):
    def nn(v):
        return math.nan if v is None else float(v)
    return Params(0.0 if fs is None else float(fs), nn(band[0]), nn(band[1]), nn(dom[0]),
                  nn(dom[1]), float(zc_threshold), float(pnn_threshold), float(csi_factor),
                  float(percentile_q), float(sampen_m), float(sampen_r), nn(sampen_sd),
                  float(rqa_radius), float(rqa_minlen))


_lock = threading.Lock()
_lib = None


def lib():
    """Load libmhfeat.so once (after torch, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "pymhealth_amd: %s is not built. Build it with `make -C %s` or "
                "`python -c 'import __graft_entry__ as g; g.build()'`."
                % (LIB_PATH, os.path.join(HERE, "csrc")))
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.mhf_version.restype = ctypes.c_int
        L.mhf_version.argtypes = []
        L.mhf_last_error.restype = ctypes.c_char_p
        L.mhf_last_error.argtypes = []
        L.mhf_num_windows.restype = i64
        L.mhf_num_windows.argtypes = [i64, i64, i64]
        L.mhf_algorithmic_bytes.restype = i64
        L.mhf_algorithmic_bytes.argtypes = [i64, i32, i64, i64, i64, i32, i32]
        L.mhf_plan_name.restype = ctypes.c_char_p
        L.mhf_plan_name.argtypes = [i32, i64, i64, i64, i64, vp, i32, i32]
        L.mhf_plan_name_f64.restype = ctypes.c_char_p
        L.mhf_plan_name_f64.argtypes = [i32, i64, i64, i64, i64, vp, i32, i32]
        L.mhf_window_features.restype = ctypes.c_int
        L.mhf_window_features.argtypes = [vp, i64, i32, i64, i64, i64, i64, i64, i64, vp, i32,
                                          ctypes.POINTER(Params), i32, i32, vp, i64, vp]
        L.mhf_window_features_f64.restype = ctypes.c_int
        L.mhf_window_features_f64.argtypes = L.mhf_window_features.argtypes
        L.mhf_indexed_window_features.restype = ctypes.c_int
        L.mhf_indexed_window_features.argtypes = [vp, i64, i32, i64, i64, vp, vp, i64, i64, vp,
                                                  i32, ctypes.POINTER(Params), i32, vp, i64, vp,
                                                  i64, vp]
        L.mhf_plan_name_indexed.restype = ctypes.c_char_p
        L.mhf_plan_name_indexed.argtypes = [i32, i64, i64, vp, i32, i32]
        L.mhf_indexed_workspace.restype = i64
        L.mhf_indexed_workspace.argtypes = [i64, i32, i32, vp, i32]
        L.mhf_indexed_window_features_f64.restype = ctypes.c_int
        L.mhf_indexed_window_features_f64.argtypes = L.mhf_indexed_window_features.argtypes
        L.mhf_window_bounds.restype = ctypes.c_int
        L.mhf_window_bounds.argtypes = [vp, i64, i64, i32, i64, i64, i64, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, vp, vp, vp]
        if L.mhf_version() != MHF_ABI_VERSION:
            raise ImportError("pymhealth_amd: %s has ABI %d, this package needs %d; rebuild it "
                              "(make -C %s)" % (LIB_PATH, L.mhf_version(), MHF_ABI_VERSION,
                                                os.path.join(HERE, "csrc")))
        L.mhf_filtfilt.restype = ctypes.c_int
        L.mhf_filtfilt.argtypes = [vp, i64, i32, i64, i64, vp, i32, vp, i32, vp, i32, vp, i64,
                                   i64, vp, i64, vp]
        L.mhf_filtfilt_workspace.restype = i64
        L.mhf_filtfilt_workspace.argtypes = [i64, i32, i32, i32]
        L.mhf_magnitude.restype = ctypes.c_int
        L.mhf_magnitude.argtypes = [vp, i64, i64, i64, vp, vp]
        L.mhf_orientation.restype = ctypes.c_int
        L.mhf_orientation.argtypes = [i32, vp, vp, vp, i64, i64, i32, vp, vp]
        L.mhf_gradient.restype = ctypes.c_int
        L.mhf_gradient.argtypes = [vp, i64, i64, i32, vp, vp]
        L.mhf_zero_crossings.restype = ctypes.c_int
        L.mhf_zero_crossings.argtypes = [vp, i64, i64, i32, ctypes.c_double, vp, vp]
        L.mhf_magnitude_dot.restype = ctypes.c_int
        L.mhf_magnitude_dot.argtypes = [vp, vp, vp, i64, i64, i32, vp, vp, i64, vp]
        L.mhf_magnitude_dot_workspace.restype = i64
        L.mhf_magnitude_dot_workspace.argtypes = [i64]
        L.mhf_find_peaks_workspace.restype = i64
        L.mhf_find_peaks_workspace.argtypes = [i64]
        L.mhf_find_peaks.restype = ctypes.c_int
        L.mhf_find_peaks.argtypes = [vp, i64, i64, i32, vp, vp, vp]
        L.mhf_find_peaks_cmp.restype = ctypes.c_int
        L.mhf_find_peaks_cmp.argtypes = [vp, i64, i64, i32, i32, vp, vp, vp]
        L.mhf_minmax.restype = ctypes.c_int
        L.mhf_minmax.argtypes = [vp, i64, i64, i32, vp, vp, i64, vp]
        L.mhf_minmax_workspace.restype = i64
        L.mhf_minmax_workspace.argtypes = [i64, i32]
        L.mhf_fft.restype = ctypes.c_int
        L.mhf_fft.argtypes = [vp, vp, i64, i64, i32, ctypes.c_double, vp, i64, vp]
        L.mhf_fft_workspace.restype = i64
        L.mhf_fft_workspace.argtypes = [i64, i64]
        L.mhf_psd_features.restype = ctypes.c_int
        L.mhf_psd_features.argtypes = [vp, i32, i64, i64, i64, vp, i32, vp, i32,
                                       ctypes.c_double, ctypes.c_double, vp, i64, vp]
        _lib = L
        return _lib


def workspace(nbytes, device, stream):
    """A caller-owned device workspace of ``nbytes`` (include/mhfeat.h: the library
    allocates nothing): a uint8 CUDA tensor from torch's caching allocator, tied to the
    ``stream`` (a raw hipStream_t handle) the library call runs on. When that is not the
    current stream the tensor records it (``record_stream``), so the allocator does not
    hand the bytes to another allocation until the library's kernels on that stream are
    done — the caller may drop the tensor right after the asynchronous call returns.

    A negative query result (arguments the library rejects) gives no workspace: the call
    itself then fails with the library's own ``mhf_last_error`` message.
    Returns (tensor or None, pointer, nbytes)."""
    import torch
    nbytes = int(nbytes)
    if nbytes <= 0:
        return None, None, 0
    t = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if int(stream) != torch.cuda.current_stream(device).cuda_stream:
        t.record_stream(torch.cuda.ExternalStream(int(stream), device=device))
    return t, ctypes.c_void_p(t.data_ptr()), nbytes


def cstream(stream, *tensors):
    """The launch argument for the raw hipStream_t ``stream`` (an int handle). When it is
    not the current stream of the current device: it first waits for the current stream
    (the wrappers stage inputs, outputs and dtype copies there, and the caller's side
    stream must not start before those are done), and ``tensors`` — the call's staged
    inputs and its outputs, allocated on the current stream — record the side stream, so
    the allocator does not hand their bytes to the current stream's next allocations
    while the library's kernels still read or write them."""
    import torch
    cur = torch.cuda.current_stream()
    if int(stream) != cur.cuda_stream:
        side = torch.cuda.ExternalStream(int(stream))
        side.wait_stream(cur)
        for t in tensors:
            if t is not None:
                t.record_stream(side)
    return ctypes.c_void_p(int(stream))


def join(stream):
    """After a launch on ``stream``: work the wrapper still does on the current stream
    (a dtype conversion or read-back of the outputs) waits for it."""
    import torch
    cur = torch.cuda.current_stream()
    if int(stream) != cur.cuda_stream:
        cur.wait_stream(torch.cuda.ExternalStream(int(stream)))


def check(rc):
    if rc != 0:
        msg = lib().mhf_last_error().decode(errors="replace")
        raise ERRORS.get(rc, RuntimeError)("libmhfeat: %s (code %d)" % (msg, rc))
