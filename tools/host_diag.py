#!/usr/bin/env python3
"""Diagnostic (GPU box): which output path do consecutive create_depth_map calls take?

Per call: whether the host expansion ran (sv_host_profile 'expand' > 0 -> int16 medians +
host expansion; 0 -> registered outputs filled by DMA), the engine's recycling slots and the
reference counts `Engine.outputs` compares against."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from stereovision_amd import depth_map as DM  # noqa: E402
from stereovision_amd import engine as E  # noqa: E402
from stereovision_amd.synthetic import stereo_pair, to_bgr  # noqa: E402

H, W, D = int(sys.argv[1]) if len(sys.argv) > 1 else 1080, int(sys.argv[2]) if len(sys.argv) > 2 else 1920, 128
DM.NUM_DISP, DM.WINDOW_SIZE, DM.MIN_DISP = D, 9, 0
frames = []
for s in range(4):
    L, R, _ = stereo_pair(H, W, D, seed=900 + s)
    frames.append((to_bgr(L), to_bgr(R)))
eng = E.get_engine()
E.host_profile(enable=True, reset=True)
print("base refs", E._BASE_REFS)
for i in range(12):
    DM.create_depth_map(*frames[i % 4])
    hp = E.host_profile(reset=True)
    slots = {k: [[sys.getrefcount(a) for a in s] for s in v] for k, v in eng._recycle.items()}
    print(f"call {i}: expand {hp['expand']:.3f} ms  total {hp['total']:.3f} ms  registered "
          f"{len(getattr(eng, '_registered', {}))}  noreg {getattr(eng, '_noreg', False)}  slots {list(slots.values())}")
E.host_profile(enable=False)
