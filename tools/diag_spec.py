"""Per (channel, feature) max relative error of the engine vs the CPU oracle (diagnostic)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from pymhealth_amd.engine import window_features, plan_name  # noqa: E402

rng = np.random.default_rng(5)
n = 256 * 4000
t = np.arange(n) / 50.0
e = rng.standard_normal((n, 3))
x = np.stack([0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * e[:, 0],
              0.2 * np.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * e[:, 1],
              1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2) + 0.05 * e[:, 2]], 1).astype(np.float32)
names = ["band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"]
ids = [oracle.FEATURE_IDS[k] for k in names]
kw = dict(fs=50.0, band=(0.5, 4.0), dom=(0.5, 8.0))
print("plan", plan_name((3, 1, 3), 256, 256, ids), "force_generic", os.environ.get("MHF_FORCE_GENERIC"))
got = window_features(torch.from_numpy(x).cuda(), 256, 256, ids, **kw).cpu().numpy()
ref = oracle.window_features(x, 256, 256, names, **kw)
for c in range(3):
    for j, nm in enumerate(names):
        rel = np.abs(got[c, j] - ref[c, j]) / np.maximum(np.abs(ref[c, j]), 1e-30)
        print(c, nm, "max rel %.3g" % rel.max(), "p99 %.3g" % np.quantile(rel, 0.99),
              "n>1e-5", int((rel > 1e-5).sum()))
