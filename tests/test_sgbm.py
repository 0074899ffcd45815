"""SGBM-3WAY mode: the reference's own matcher
(cv2.StereoSGBM, MODE_SGBM_3WAY, depth_map.py:894-909) restated.

Oracle: oracle/sv_sgbm_oracle.py (OpenCV's published algorithm, one stripe; parity with
OpenCV itself unpinned — cv2 is absent).  GPU bar: the int16 x16 map bit-exact against
the oracle for every parameter path (int16/int32 path storage, uniqueness, sub-pixel,
left-right check, speckle filter, band borders, negative/positive min_disp).
"""
import numpy as np
import pytest

import sv_sgbm_oracle as SG
from stereovision_amd.synthetic import stereo_pair


# ---------------------------------------------------------------------------- CPU: oracle
def test_oracle_recovers_integer_shift():
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (40, 200), dtype=np.uint8)
    shift = 7
    L = base[:, :150].copy()                             # L(x) = R(x - shift)
    R = base[:, shift:shift + 150].copy()
    d = SG.sgbm(L, R, 0, 32, 5)
    inner = d[3:-3, 40:-3].astype(np.int32)
    assert (np.abs(inner - shift * 16) <= 1).mean() > 0.99      # sub-pixel within 1/16
    assert (inner == shift * 16).mean() > 0.9
    assert (d[:, :32] == -16).all()                     # band [X0, X1) only


def test_oracle_invalid_band_and_negative_min_disp():
    L, R, _ = stereo_pair(24, 90, 16, seed=2)
    d = SG.sgbm(L, R, -8, 16, 3)
    X0, X1 = max(-8 + 16, 0), 90 - 8
    assert (d[:, :X0] == -9 * 16).all() and (d[:, X1:] == -9 * 16).all()


def test_filter_speckles_known_answer():
    img = np.full((10, 12), 100, np.int16)
    img[2:4, 2:4] = 900                                  # 4-pixel island, differs by 800
    img[6:9, 5:11] = 80                                  # joins the background (|diff| 20)
    out = SG.filter_speckles(img, -16, 5, 512)
    assert (out[2:4, 2:4] == -16).all() and (out[6:9, 5:11] == 80).all() and out[0, 0] == 100
    out = SG.filter_speckles(img, -16, 3, 512)
    assert (out[2:4, 2:4] == 900).all()                  # 4 > maxSpeckleSize 3: kept


def test_oracle_quality_on_synthetic_pair():
    L, R, gt = stereo_pair(48, 200, 32, seed=3)
    d = SG.sgbm(L, R, 0, 32, 5)
    ok = d[:, 40:] >= 0
    assert ok.mean() > 0.8


# ---------------------------------------------------------------------------- GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("D,win,min_disp", [(16, 3, 0), (32, 5, 0), (48, 7, 0), (64, 9, 0),
                                            (96, 5, 0), (32, 11, -8), (16, 1, 5), (80, 7, 3)])
def test_gpu_sgbm_matches_oracle(engine, D, win, min_disp):
    L, R, _ = stereo_pair(53, 240, max(D, 16), seed=D + win, min_disp=max(0, min_disp))
    got = engine.sgbm(L, R, min_disp, D, win)
    exp = SG.sgbm(L, R, min_disp, D, win)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(disp12_max_diff=-1), dict(uniqueness_ratio=0),
                                dict(speckle_window_size=0), dict(P2=40000),
                                dict(P1=50, P2=10), dict(pre_filter_cap=31, speckle_range=2)])
def test_gpu_sgbm_parameter_paths(engine, kw):
    L, R, _ = stereo_pair(37, 200, 32, seed=11)
    got = engine.sgbm(L, R, 0, 32, 5, **kw)
    okw = {"disp12_max_diff": "disp12MaxDiff", "uniqueness_ratio": "uniquenessRatio",
           "speckle_window_size": "speckleWindowSize", "pre_filter_cap": "preFilterCap",
           "speckle_range": "speckleRange"}
    exp = SG.sgbm(L, R, 0, 32, 5, **{okw.get(k, k): v for k, v in kw.items()})
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
def test_gpu_sgbm_int32_paths_window15(engine):
    L, R, _ = stereo_pair(40, 180, 32, seed=5)
    np.testing.assert_array_equal(engine.sgbm(L, R, 0, 32, 15), SG.sgbm(L, R, 0, 32, 15))
    # D > 128: the vertical path fused with the WTA, on int32 path volumes
    L, R, _ = stereo_pair(19, 330, 192, seed=6)
    np.testing.assert_array_equal(engine.sgbm(L, R, 0, 192, 15), SG.sgbm(L, R, 0, 192, 15))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W", [(1, 40), (2, 33), (5, 17), (30, 20)])
def test_gpu_sgbm_ragged(engine, H, W):
    rng = np.random.default_rng(H * W)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    np.testing.assert_array_equal(engine.sgbm(L, R, 0, 16, 3), SG.sgbm(L, R, 0, 16, 3))


@pytest.mark.gpu
def test_gpu_sgbm_through_generic_entry_points(engine):
    """cost='sgbm' through sv_disparity / sv_depth_map: the reference's parameters."""
    import sv_oracle as O
    from stereovision_amd.synthetic import to_bgr
    L, R, _ = stereo_pair(45, 210, 48, seed=8)
    exp = SG.sgbm(L, R, 0, 48, 7)
    np.testing.assert_array_equal(engine.disparity(L, R, 0, 48, 7, "sgbm"), exp)
    depth, disp, norm = engine.depth_map(to_bgr(L), to_bgr(R), 0, 48, 7, 0.3, 2.0, cost="sgbm")
    e_disp = O.disparity_f32(exp)                        # /16 + medianBlur(5)
    np.testing.assert_array_equal(disp, e_disp)
    e_depth, e_norm = O.depth_post(e_disp, 0.3, 2.0, 0)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)
    with pytest.raises(Exception):
        engine.disparity_rows(L, R, 0, 48, 7, 5, 20, "sgbm")   # row bands: frames only


@pytest.mark.gpu
def test_gpu_sgbm_1080p_properties(engine):
    """Benchmark size: integer-shift scene recovered; invalid band exact."""
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, (1080, 1920 + 32), dtype=np.uint8).astype(np.int32)
    base = ((base + np.roll(base, 1, 1) + np.roll(base, 1, 0)) // 3).astype(np.uint8)
    L = np.ascontiguousarray(base[:, :1920])            # L(x) = R(x - 20)
    R = np.ascontiguousarray(base[:, 20:20 + 1920])
    d = engine.sgbm(L, R, 0, 128, 7)
    assert (d[:, :128] == -16).all()
    inner = d[10:-10, 140:-10].astype(np.int32)
    assert (np.abs(inner - 20 * 16) <= 1).mean() > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("deep", [None, "0", "2"])
@pytest.mark.parametrize("D,win", [(160, 5), (256, 7), (320, 7), (384, 3), (512, 5)])
def test_gpu_sgbm_wide_disparity_ranges(engine, monkeypatch, D, win, deep):
    """Every lane plan of the path kernels (DPL 12..32), incl. the reference's default
    NUM_DISP = 16*20 = 320 with WINDOW_SIZE = 7 (depth_map.py:31-33); both forms of the
    vertical path + WTA (SV_SGBM_DEEP, read per call: 0 = two waves per SIMD, 2 = one wave
    with the deeper prefetch; default = deep for small launches like these)."""
    if deep is not None:
        monkeypatch.setenv("SV_SGBM_DEEP", deep)
    L, R, _ = stereo_pair(21, D + 90, D, seed=D)
    np.testing.assert_array_equal(engine.sgbm(L, R, 0, D, win), SG.sgbm(L, R, 0, D, win))


def _speckle_scene(H, W, seed):
    """Regions of every size, many crossing the 32x32 tiles: random blobs of constant
    disparity on a smooth background, plus snakes and invalid pixels."""
    rng = np.random.default_rng(seed)
    img = (rng.integers(0, 3, (H, W)) + 40 * 16).astype(np.int16)          # background
    for _ in range(H * W // 300):
        y, x = int(rng.integers(0, H)), int(rng.integers(0, W))
        h, w = int(rng.integers(1, 14)), int(rng.integers(1, 14))
        img[y:y + h, x:x + w] = int(rng.integers(0, 128)) * 16
    for _ in range(H * W // 4000):                                          # 1-pixel snakes
        y, x = int(rng.integers(0, H)), int(rng.integers(0, W))
        v = int(rng.integers(0, 128)) * 16
        for _ in range(int(rng.integers(20, 200))):
            img[y, x] = v
            if rng.random() < 0.5:
                x = min(max(x + int(rng.integers(-1, 2)), 0), W - 1)
            else:
                y = min(max(y + int(rng.integers(-1, 2)), 0), H - 1)
    img[rng.random((H, W)) < 0.02] = -16                                    # invalid
    return img


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,maxsize,maxdiff", [(67, 130, 100, 32), (200, 301, 100, 512),
                                                 (96, 96, 5, 16), (150, 170, 1000, 64),
                                                 (1, 50, 3, 0), (40, 1, 3, 0)])
def test_gpu_filter_speckles_matches_oracle(engine, H, W, maxsize, maxdiff):
    """cv2.filterSpeckles restated (SG.filter_speckles) vs the union-find kernels: regions
    across tile borders, snakes, invalid pixels, tiny and huge size limits."""
    img = _speckle_scene(H, W, H * 7 + W)
    np.testing.assert_array_equal(engine.filter_speckles(img, -16, maxsize, maxdiff),
                                  SG.filter_speckles(img, -16, maxsize, maxdiff))


@pytest.mark.gpu
def test_gpu_filter_speckles_1080p_property(engine):
    """Benchmark size: a background that spans every tile stays, isolated small blocks on
    it go, blocks of more than maxsize pixels stay (the border-skip path)."""
    H, W = 1080, 1920
    img = np.full((H, W), 50 * 16, np.int16)
    exp = img.copy()
    for i, y in enumerate(range(5, H - 20, 40)):
        for j, x in enumerate(range(5, W - 20, 40)):
            s = 7 if (i + j) % 2 else 12                      # 49 px (speckle) / 144 px (kept)
            img[y + 20:y + 20 + s, x + 20:x + 20 + s] = (100 + (i * 7 + j) % 20) * 16
            if s == 12:
                exp[y + 20:y + 20 + s, x + 20:x + 20 + s] = img[y + 20, x + 20]
            else:
                exp[y + 20:y + 20 + s, x + 20:x + 20 + s] = -16
    np.testing.assert_array_equal(engine.filter_speckles(img, -16, 100, 32), exp)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,D,win", [(300, 120, 32, 9), (257, 96, 16, 3), (130, 72, 48, 15)])
def test_gpu_sgbm_tall_frames_row_bands(engine, H, W, D, win):
    """Tall frames: the window-row sums run in row bands of >= 64 rows (k_sgbm_vsum8), each
    band re-summing its first window; band seams must be invisible."""
    L, R, _ = stereo_pair(H, W, D, seed=H + W)
    np.testing.assert_array_equal(engine.sgbm(L, R, 0, D, win), SG.sgbm(L, R, 0, D, win))


@pytest.mark.gpu
@pytest.mark.parametrize("nf,H,W,D,win,minD", [(11, 37, 150, 32, 5, 0),     # fused R->L + WTA
                                                (9, 29, 133, 48, 15, -3),   # fused, int32 paths
                                                (3, 29, 133, 48, 15, -3),   # unfused, int32
                                                (2, 64, 200, 64, 9, 4),     # unfused
                                                (3, 23, 430, 320, 7, 0),    # unfused, vertical path + WTA fused
                                                (2, 17, 300, 160, 13, -2),  # unfused, vertical + WTA, int32
                                                (8, 16, 380, 320, 7, 0),    # DPL 20 (R->L fused when forced)
                                                (8, 12, 560, 512, 5, 0),    # DPL 32 (forced)
                                                (8, 21, 90, 16, 3, 0),      # fused, DPL 1
                                                (8, 19, 230, 128, 9, -2),   # fused, DPL 8
                                                (8, 14, 300, 192, 5, 0),    # DPL 12 (forced)
                                                (8, 13, 330, 256, 7, 3),    # DPL 16 (forced)
                                                (8, 11, 450, 384, 3, 0)])   # DPL 24 (forced)
@pytest.mark.parametrize("fused", ["auto", "1"])
def test_gpu_sgbm_frame_batch(engine, monkeypatch, fused, nf, H, W, D, win, minD):
    """Frame batches (every SGBM stage and the speckle filter over grid.z; batches of >= 8
    frames with D <= 128 fuse the R->L path with the WTA, D > 128 the vertical path; fused="1"
    forces the R->L fusion, SV_SGBM_FUSED read per call): each frame of a pitched, strided
    stack bit-exact against the oracle run on that frame alone."""
    if fused != "auto":
        monkeypatch.setenv("SV_SGBM_FUSED", fused)
    pitch, fs = W + 24, (H + 3) * (W + 24)
    Ls = np.zeros((nf, H + 3, pitch), np.uint8)
    Rs = np.zeros_like(Ls)
    for z in range(nf):
        L, R, _ = stereo_pair(H, W, D, seed=100 + z)
        if z % 3 == 2:   # flat / noise frames beside textured ones
            R = np.random.default_rng(z).integers(0, 256, (H, W), dtype=np.uint8)
        Ls[z, :H, :W], Rs[z, :H, :W] = L, R
    opitch, ofs = W + 8, H * (W + 8) + 40
    dL, dR = engine.dev_alloc(Ls.nbytes), engine.dev_alloc(Rs.nbytes)
    dO = engine.dev_alloc(nf * ofs * 2)
    try:
        engine.to_device(dL, Ls)
        engine.to_device(dR, Rs)
        engine.disparity_batch_dev(dL, dR, nf, H, W, pitch, fs, minD, D, win, "sgbm", dO, opitch, ofs)
        engine.synchronize()
        flat = engine.to_host(dO, (nf * ofs,), np.int16)
        for z in range(nf):
            got = flat[z * ofs:z * ofs + H * opitch].reshape(H, opitch)[:, :W]
            exp = SG.sgbm(Ls[z, :H, :W], Rs[z, :H, :W], minD, D, win)
            np.testing.assert_array_equal(got, exp, err_msg=f"frame {z}")
    finally:
        for p in (dL, dR, dO):
            engine.dev_free(p)
