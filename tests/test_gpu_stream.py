"""The stream kind of the SAD matcher (k_match_stream: persistent waves walking whole rows
through LDS pack rings, sv_match.hip) against the C oracle, bit-exact.

It serves SAD with 5 <= win <= 9 and 65 <= D <= 256 on 4-aligned images; the cases below
cover both lane-group widths (32: D <= 128, 64: D <= 256), every radius, shares that start
inside a row (prologue) or at a row start, bundles with a null group (odd row-quad counts),
partial row quads, row bands, frame batches, non-zero / negative / odd minimum disparities
(the right stream's gap phase), image borders on both sides, and A/B equality with the ring
kind (SV_STREAM=0 in a child process).  The stream kind is opt-in (SV_STREAM=1, read per
launch): every test here switches it on.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _stream_on(monkeypatch):
    monkeypatch.setenv("SV_STREAM", "1")


def _dev(engine, a):
    p = engine.dev_alloc(max(256, a.nbytes))
    engine.to_device(p, np.ascontiguousarray(a))
    return p


@pytest.mark.parametrize("H,W,D,win,minD", [
    (64, 320, 96, 5, 0), (61, 400, 128, 7, 0), (37, 256, 72, 9, 0), (120, 640, 128, 9, 0),
    (96, 512, 200, 9, 0), (45, 320, 256, 7, 0), (80, 480, 128, 9, 5), (50, 384, 100, 5, -7),
    (33, 300, 80, 9, 3), (8, 200, 68, 5, 0), (1080, 1920, 128, 9, 0), (200, 1024, 192, 9, 2)])
def test_stream_matches_oracle(engine, H, W, D, win, minD):
    L, R, _ = stereo_pair(H, W, D, seed=H * 7 + W + D, min_disp=max(0, minD))
    exp = C.disparity16(L, R, minD, D, win)
    got = engine.disparity(L, R, minD, D, win)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("nf,H,W,D,win", [(3, 45, 320, 128, 9), (16, 120, 640, 128, 9), (5, 66, 400, 160, 7)])
def test_stream_frame_batches(engine, nf, H, W, D, win):
    frames = [stereo_pair(H, W, D, seed=300 + f)[:2] for f in range(nf)]
    Ls = np.stack([f[0] for f in frames])
    Rs = np.stack([f[1] for f in frames])
    dL, dR = _dev(engine, Ls), _dev(engine, Rs)
    out = engine.dev_alloc(2 * nf * H * W)
    try:
        engine.disparity_batch_dev(dL, dR, nf, H, W, W, H * W, 0, D, win, "sad", out, W, H * W)
        engine.synchronize()
        got = engine.to_host(out, (nf, H, W), np.int16)
        for f, (L, R) in enumerate(frames):
            np.testing.assert_array_equal(got[f], C.disparity16(L, R, 0, D, win), err_msg=f"frame {f}")
    finally:
        for p in (dL, dR, out):
            engine.dev_free(p)


@pytest.mark.parametrize("row0,row1", [(0, 13), (5, 50), (17, 18), (40, 97)])
def test_stream_row_bands(engine, row0, row1):
    H, W, D, win = 97, 448, 128, 9
    L, R, _ = stereo_pair(H, W, D, seed=row0 * 100 + row1)
    exp = C.disparity16(L, R, 0, D, win, rows=(row0, row1))
    dL, dR = _dev(engine, L), _dev(engine, R)
    out = engine.dev_alloc(2 * H * W)
    try:
        engine.to_device(out, np.full((H, W), 1234, np.int16))
        engine.disparity_dev(dL, dR, H, W, W, 0, D, win, "sad", row0, row1, out, W)
        engine.synchronize()
        got = engine.to_host(out, (H, W), np.int16)
        np.testing.assert_array_equal(got[row0:row1], exp[row0:row1])
        assert (got[:row0] == 1234).all() and (got[row1:] == 1234).all(), "rows outside the band written"
    finally:
        for p in (dL, dR, out):
            engine.dev_free(p)


def test_stream_and_ring_kinds_agree():
    """The same maps from a child with SV_STREAM=0 (ring kind) and one with SV_STREAM=1."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r)\n"
            "from stereovision_amd.engine import get_engine\n"
            "from stereovision_amd.synthetic import stereo_pair\n"
            "L, R, _ = stereo_pair(270, 960, 128, seed=5)\n"
            "d = get_engine(0).disparity(L, R, 0, 128, 9)\n"
            "sys.stdout.buffer.write(d.tobytes())\n") % ROOT
    outs = []
    for flag in ("0", "1"):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120,
                           env=dict(os.environ, SV_STREAM=flag, SV_WARMUP_AT_IMPORT="0"))
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        outs.append(r.stdout)
    assert outs[0] == outs[1] and len(outs[0]) == 2 * 270 * 960
