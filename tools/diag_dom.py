"""Diagnostic: W = 1024 dominant frequency must lie inside the requested range."""
import itertools
import os
import numpy as np
import torch
from pymhealth_amd import _lib
from pymhealth_amd.engine import window_features

nw, W, S = 300, 1024, 128
n = (nw - 1) * S + W
rng = np.random.default_rng(77)
x = (rng.standard_normal(n) * 0.3 + np.sin(np.arange(n) * 0.31) + 0.7).astype(np.float32)
xd = torch.from_numpy(x).cuda()
for mode, band, dom, feats in itertools.product(
        ["ring", "dma", "vgpr"], [(None, None), (0.5, 40.0), (0.5, 128.0), (20.0, 30.0)],
        [(2.0, 10.0), (0.5, 40.0)], [["dominant_frequency"], ["band_power", "dominant_frequency"]]):
    os.environ.pop("MHF_SPECREG_NORING", None)
    os.environ.pop("MHF_SPECREG_NODMA", None)
    if mode == "dma":
        os.environ["MHF_SPECREG_NORING"] = "1"
    if mode == "vgpr":
        os.environ["MHF_SPECREG_NODMA"] = "1"
    ids = [{"dominant_frequency": _lib.MHF_DOMINANT_FREQ, "band_power": _lib.MHF_BAND_POWER}[f] for f in feats]
    got = window_features(xd, W, S, ids, fs=256.0, band=band, dom=dom).cpu().numpy()
    d = got[0, feats.index("dominant_frequency")]
    bad = ~((d >= dom[0]) & (d < dom[1]))
    print(mode, band, dom, feats, "bad", int(bad.sum()), d[:4], flush=True)
