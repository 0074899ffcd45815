"""Where the Harris kernel differs from the oracle (debug aid): error map summary."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sv_oracle as O  # noqa: E402
from stereovision_amd.engine import get_engine  # noqa: E402

e = get_engine(0)
for H, W in [(50, 70), (16, 64), (20, 130)]:
    g = np.random.default_rng(0).integers(0, 256, (H, W), dtype=np.uint8)
    got, exp = e.harris(g), O.harris(g)
    bad = np.abs(got - exp) > 1e-4
    print(H, W, "bad", int(bad.sum()), "of", bad.size)
    print(" bad rows", np.nonzero(bad.any(1))[0][:40])
    print(" bad cols", np.nonzero(bad.any(0))[0][:80])
    print(" got row 5", got[5, :6], "exp", exp[5, :6])
