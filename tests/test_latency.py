"""First-call latency of the drop-ins against the reference's 0.5 s budget.

fused_depth_map.py:2591-2598 submits create_depth_map_stereo_scaled to a worker and
fused_depth_map.py:2671 waits `future.result(timeout=0.5)`; a timeout yields zero maps
(:2678-2695).  Importing the drop-in module warms the engine up on a background thread
(HIP initialisation, context, code objects, staging at the processing size: 1920x1080 at
PROCESSING_SCALE 0.33 = 633x356, D=96, window 5), so the FIRST frame of a fresh process
must come back inside the budget.  Measured in a fresh interpreter each time.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CODE = r"""
import json, sys, time
sys.path.insert(0, %(root)r)
t0 = time.perf_counter()
import numpy as np
from stereovision_amd import %(module)s as M
from stereovision_amd.synthetic import stereo_pair, to_bgr
t_import = time.perf_counter() - t0
L, R, _ = stereo_pair(%(H)d, %(W)d, %(D)d, seed=1)
bl, br = to_bgr(L), to_bgr(R)
t_ready = time.perf_counter() - t0
t1 = time.perf_counter()
out = %(call)s
t_first = time.perf_counter() - t1
t2 = time.perf_counter()
out2 = %(call)s
t_second = time.perf_counter() - t2
same = all(np.array_equal(a, b) for a, b in zip(out, out2))
print(json.dumps({"import_s": t_import, "ready_s": t_ready, "first_call_s": t_first,
                  "second_call_s": t_second, "same": bool(same),
                  "nonzero": bool(np.count_nonzero(out[1]))}))
"""


def _run(module, call, H, W, D):
    code = _CODE % {"root": ROOT, "module": module, "call": call, "H": H, "W": W, "D": D}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       cwd=ROOT, env=dict(os.environ, SV_WARMUP_AT_IMPORT="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(module, res)
    return res


def test_first_scaled_call_within_the_reference_timeout():
    res = _run("fused_depth_map", "M.create_depth_map_stereo_scaled(bl, br, 0, 96, 5)", 356, 633, 96)
    assert res["same"] and res["nonzero"]
    assert res["first_call_s"] < 0.5, res


def test_first_depth_map_call_latency():
    res = _run("depth_map", "M.create_depth_map(bl, br)", 480, 640, 320)
    assert res["same"] and res["nonzero"]
    assert res["first_call_s"] < 0.5, res
