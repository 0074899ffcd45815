"""Rectification stage: stereoRectify geometry, the
initUndistortRectifyMap / remap / resize oracles, and GPU parity of k_undistort_map,
k_remap and k_resize_linear through the C ABI.

Parity bar: maps, remapped and resized images bit-exact against the oracle
(oracle/sv_rectify_oracle.py).  Against OpenCV itself parity is unpinned (cv2 absent);
the CPU tests pin the oracle with known answers instead.
"""
import io
import json
import os
import pickle

import numpy as np
import pytest

import sv_rectify_oracle as RO
from stereovision_amd import calib


def _camera(fx=700.0, fy=702.0, cx=318.3, cy=241.7):
    return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])


def _stereo_setup(seed=0, size=(640, 480)):
    rng = np.random.default_rng(seed)
    K1 = _camera(700 + rng.normal() * 5, 702 + rng.normal() * 5,
                 size[0] / 2 + rng.normal() * 4, size[1] / 2 + rng.normal() * 4)
    K2 = _camera(698 + rng.normal() * 5, 699 + rng.normal() * 5,
                 size[0] / 2 + rng.normal() * 4, size[1] / 2 + rng.normal() * 4)
    D1 = np.array([[-0.12, 0.05, 0.001, -0.0008, -0.01]])
    D2 = np.array([[-0.10, 0.04, -0.0005, 0.0009, -0.008]])
    R = calib.rodrigues_to_matrix(rng.normal(size=3) * 0.02)
    T = np.array([[-0.08], [0.002 * rng.normal()], [0.001 * rng.normal()]])
    return K1, D1, K2, D2, R, T


# ---------------------------------------------------------------------------- CPU: oracle
def test_bilinear_fixed_point_forms_agree():
    """OpenCV's 2^15 table (with its saturated (0,0) entry) and the 10-bit form the kernel
    uses give the same byte for every fraction; exhaustive over v for the (0,0) entry."""
    tab = RO.bilinear_tab_i()
    assert tab[0].tolist() == [32767, 0, 0, 0]
    assert (tab[1:].sum(1) == 32768).all()
    rng = np.random.default_rng(1)
    v = rng.integers(0, 256, (4096, 4))
    v[:16] = [[255, 255, 255, 255], [0, 0, 0, 0], [255, 0, 0, 0], [0, 255, 255, 255]] * 4
    for f in range(1024):
        fx, fy = f & 31, f >> 5
        w = np.array([(32 - fy) * (32 - fx), (32 - fy) * fx, fy * (32 - fx), fy * fx])
        a = (v @ tab[f] + (1 << 14)) >> 15
        b = (v @ w + 512) >> 10
        np.testing.assert_array_equal(a, b)
    v0 = np.arange(256)
    for v3 in (0, 255):
        np.testing.assert_array_equal((v0 * 32767 + v3 * 0 + (1 << 14)) >> 15, v0)


def test_identity_calibration_gives_identity_maps():
    K = _camera()
    m1, m2, _, _ = RO.undistort_rectify_map(K, None, None, K, 65, 33)
    jj, ii = np.meshgrid(np.arange(65), np.arange(33))
    assert (m1[..., 0] == jj).all() and (m1[..., 1] == ii).all() and (m2 == 0).all()


def test_maps_follow_the_forward_distortion_model():
    K1, D1, K2, D2, R, T = _stereo_setup(3)
    R1, R2, P1, P2, Q, _, _ = calib.stereo_rectify(K1, D1, K2, D2, (160, 120), R, T, alpha=0)
    m1, m2, u, v = RO.undistort_rectify_map(K1, D1, R1, P1, 160, 120)
    jj, ii = np.meshgrid(np.arange(160.0), np.arange(120.0))
    ray = np.linalg.inv(P1[:, :3] @ R1) @ np.stack([jj.ravel(), ii.ravel(), np.ones(jj.size)])
    xd, yd = RO.distort_normalised(ray[0] / ray[2], ray[1] / ray[2], D1)
    np.testing.assert_allclose(u.ravel(), K1[0, 0] * xd + K1[0, 2], atol=1e-8)
    np.testing.assert_allclose(v.ravel(), K1[1, 1] * yd + K1[1, 2], atol=1e-8)
    iu = m1[..., 0].astype(np.int64) * 32 + (m2 & 31)
    iv = m1[..., 1].astype(np.int64) * 32 + (m2 >> 5)
    assert np.abs(iu - u * 32).max() <= 0.5 and np.abs(iv - v * 32).max() <= 0.5


def test_remap_oracle_integer_maps_are_a_gather():
    rng = np.random.default_rng(2)
    src = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    m1 = np.stack([rng.integers(-3, 33, (9, 11)), rng.integers(-3, 23, (9, 11))], -1).astype(np.int16)
    out = RO.remap_linear(src, m1, np.zeros((9, 11), np.uint16))
    x, y = m1[..., 0].astype(int), m1[..., 1].astype(int)
    ok = (x >= 0) & (x < 30) & (y >= 0) & (y < 20)
    exp = np.zeros((9, 11, 3), np.uint8)
    exp[ok] = src[y[ok], x[ok]]
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(out, RO.remap_linear(src, m1, np.zeros((9, 11), np.uint16), table="exact"))


def test_remap_oracle_half_pixel_is_rounded_mean():
    src = np.array([[10, 21], [30, 41]], np.uint8)
    m1 = np.zeros((1, 1, 2), np.int16)
    m2 = np.array([[16 * 32 + 16]], np.uint16)           # fx = fy = 1/2
    assert RO.remap_linear(src, m1, m2)[0, 0] == (10 + 21 + 30 + 41 + 2) // 4


def test_resize_oracle_known_answers():
    z = np.full((40, 60, 3), 77, np.uint8)
    for w, h in [(33, 17), (120, 90), (30, 20), (61, 41)]:
        assert (RO.resize_linear(z, w, h) == 77).all()
    a = np.arange(16, dtype=np.uint8).reshape(4, 4) * 10
    np.testing.assert_array_equal(RO.resize_linear(a, 2, 2),
                                  (a[0::2, 0::2].astype(int) + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2)
    ramp = np.tile(np.arange(0, 200, 2, dtype=np.uint8), (3, 1))      # 3 x 100, linear in x
    r = RO.resize_linear(ramp, 50, 3).astype(int)[0]
    # centre of output d at x = 2d + 0.5: (ramp[2d] + ramp[2d+1]) / 2 = 4d + 1 exactly
    np.testing.assert_array_equal(r, 4 * np.arange(50) + 1)


# ------------------------------------------------------------------- CPU: stereoRectify
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stereo_rectify_geometry(seed):
    K1, D1, K2, D2, R, T = _stereo_setup(seed)
    R1, R2, P1, P2, Q, roi1, roi2 = calib.stereo_rectify(K1, D1, K2, D2, (640, 480), R, T, alpha=0)
    for Rk in (R1, R2):
        np.testing.assert_allclose(Rk @ Rk.T, np.eye(3), atol=1e-12)
        assert np.linalg.det(Rk) > 0
    np.testing.assert_allclose(R2 @ R @ R1.T, np.eye(3), atol=1e-12)   # common orientation
    t = R2 @ T.ravel()
    assert abs(t[1]) < 1e-12 and abs(t[2]) < 1e-12 and t[0] < 0          # baseline along x
    assert P1[0, 0] == P1[1, 1] == P2[0, 0] == P2[1, 1]
    assert P1[1, 2] == P2[1, 2] and P1[0, 2] == P2[0, 2]                 # CALIB_ZERO_DISPARITY
    np.testing.assert_allclose(P2[0, 3], P2[0, 0] * t[0], rtol=1e-12)
    # random 3D points: equal rows in both rectified views; Q reprojects them
    rng = np.random.default_rng(seed)
    X = np.stack([rng.uniform(-1, 1, 50), rng.uniform(-0.7, 0.7, 50), rng.uniform(1, 5, 50)], 1)
    p1 = (P1 @ np.vstack([(R1 @ X.T), np.ones(50)]))
    p2 = (P2 @ np.vstack([(R1 @ X.T), np.ones(50)]))
    u1, v1 = p1[0] / p1[2], p1[1] / p1[2]
    u2, v2 = p2[0] / p2[2], p2[1] / p2[2]
    np.testing.assert_allclose(v1, v2, atol=1e-9)
    h = Q @ np.vstack([u1, v1, u1 - u2, np.ones(50)])
    np.testing.assert_allclose((h[:3] / h[3]).T, (R1 @ X.T).T, rtol=1e-9, atol=1e-9)
    for r in (roi1, roi2):
        assert r[0] >= 0 and r[1] >= 0 and r[0] + r[2] <= 640 and r[1] + r[3] <= 480 and r[2] > 300


def test_stereo_rectify_aligned_cameras_have_identity_rotations():
    K = _camera(700, 700, 320, 240)
    R1, R2, P1, P2, Q, _, _ = calib.stereo_rectify(K, None, K, None, (640, 480), np.eye(3),
                                                    np.array([-0.08, 0, 0]), alpha=0)
    np.testing.assert_allclose(R1, np.eye(3), atol=1e-15)
    np.testing.assert_allclose(R2, np.eye(3), atol=1e-15)
    assert P1[0, 0] >= 700.0                      # alpha = 0 crops (zooms in) only
    np.testing.assert_allclose(Q[3, 2], 1 / 0.08)


def test_rodrigues_round_trip():
    rng = np.random.default_rng(4)
    for _ in range(20):
        r = rng.normal(size=3)
        r *= rng.uniform(0.01, 3.0) / np.linalg.norm(r)      # |r| < pi: the unique vector
        np.testing.assert_allclose(calib.rodrigues_to_vector(calib.rodrigues_to_matrix(r)), r, atol=1e-9)
    np.testing.assert_allclose(calib.rodrigues_to_vector(np.eye(3)), 0)
    rpi = np.array([0, np.pi, 0])
    np.testing.assert_allclose(calib.rodrigues_to_matrix(calib.rodrigues_to_vector(calib.rodrigues_to_matrix(rpi))),
                               calib.rodrigues_to_matrix(rpi), atol=1e-9)


def _calib_dict(size=(160, 120), seed=0):
    K1, D1, K2, D2, R, T = _stereo_setup(seed, size)
    return {"ret": 0.3, "mtx_left": K1, "dist_left": D1, "mtx_right": K2, "dist_right": D2, "R": R,
            "T": T, "img_size": size, "num_valid_pairs": 12}


def test_calibration_file_formats(tmp_path):
    d = _calib_dict()
    p = tmp_path / "stereo_calibration_data.pkl"
    with open(p, "wb") as f:
        pickle.dump(d, f)
    got = calib.read_calibration(str(p))
    np.testing.assert_array_equal(got["mtx_left"], d["mtx_left"])
    assert tuple(got["img_size"]) == (160, 120)
    np.savez(tmp_path / "c.npz", **{k: np.asarray(v) for k, v in d.items()})
    np.testing.assert_array_equal(calib.read_calibration(str(tmp_path / "c.npz"))["R"], d["R"])
    with open(tmp_path / "c.json", "w") as f:
        json.dump({k: np.asarray(v).tolist() for k, v in d.items()}, f)
    np.testing.assert_array_equal(calib.read_calibration(str(tmp_path / "c.json"))["T"], d["T"])


def test_calibration_pickle_refuses_foreign_globals(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.getcwd, ())
    p = tmp_path / "evil.pkl"
    with open(p, "wb") as f:
        pickle.dump({"mtx_left": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        calib.read_calibration(str(p))


def test_loaders_missing_file_return_none(capsys):
    from stereovision_amd import rectify
    assert rectify.load_stereo_calibration("/nonexistent/x.pkl") is None
    assert rectify.load_stereo_calibration_with_scaling(0.5, "/nonexistent/x.pkl") is None
    l = np.zeros((4, 4, 3), np.uint8)
    a, b = rectify.apply_stereo_rectification(l, l, None)
    assert a is l and b is l


# ---------------------------------------------------------------------------- GPU parity
def _random_maps(H, W, sH, sW, seed):
    rng = np.random.default_rng(seed)
    m1 = np.stack([rng.integers(-3, sW + 3, (H, W)), rng.integers(-3, sH + 3, (H, W))], -1).astype(np.int16)
    m2 = rng.integers(0, 1 << 16, (H, W)).astype(np.uint16)      # high bits must be ignored
    return m1, m2


@pytest.mark.gpu
@pytest.mark.parametrize("size", [(640, 480), (633, 355), (97, 31)])
@pytest.mark.parametrize("seed", [0, 5])
def test_gpu_undistort_map_matches_oracle(engine, size, seed):
    W, H = size
    K1, D1, K2, D2, R, T = _stereo_setup(seed, size)
    R1, R2, P1, P2, Q, _, _ = calib.stereo_rectify(K1, D1, K2, D2, size, R, T, alpha=0)
    for K, D, Rk, P in ((K1, D1, R1, P1), (K2, D2, R2, P2)):
        m1, m2 = engine.init_undistort_rectify_map(K, D, Rk, P, W, H)
        e1, e2, _, _ = RO.undistort_rectify_map(K, D, Rk, P, W, H)
        np.testing.assert_array_equal(m1, e1)
        np.testing.assert_array_equal(m2, e2)


@pytest.mark.gpu
def test_gpu_undistort_map_distortion_models(engine):
    K = _camera()
    for D in ([0.1, -0.2, 0.01, 0.02],
              [-0.3, 0.1, 0.0, 0.001, 0.02, 0.01, -0.02, 0.03],
              [-0.2, 0.05, 0.001, 0.001, 0.0, 0.0, 0.0, 0.0, 0.001, -0.002, 0.003, 0.0005]):
        m1, m2 = engine.init_undistort_rectify_map(K, D, None, None, 200, 150)
        e1, e2, _, _ = RO.undistort_rectify_map(K, D, None, None, 200, 150)
        np.testing.assert_array_equal(m1, e1)
        np.testing.assert_array_equal(m2, e2)
    P34 = np.hstack([K, np.array([[-56.0], [0], [0]])])
    m1, m2 = engine.init_undistort_rectify_map(K, None, np.eye(3), P34, 64, 48)
    jj, ii = np.meshgrid(np.arange(64), np.arange(48))
    assert (m1[..., 0] == jj).all() and (m1[..., 1] == ii).all() and (m2 == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [1, 3])
@pytest.mark.parametrize("shape", [(48, 64, 40, 60), (31, 97, 29, 101), (7, 5, 9, 3), (1, 1, 1, 1)])
def test_gpu_remap_random_maps(engine, channels, shape):
    H, W, sH, sW = shape
    rng = np.random.default_rng(H * W + channels)
    src = rng.integers(0, 256, (sH, sW, channels) if channels == 3 else (sH, sW), dtype=np.uint8)
    m1, m2 = _random_maps(H, W, sH, sW, seed=H + W)
    np.testing.assert_array_equal(engine.remap(src, m1, m2), RO.remap_linear(src, m1, m2))
    np.testing.assert_array_equal(engine.remap(src, m1, None), RO.remap_linear(src, m1, np.zeros_like(m2)))


@pytest.mark.gpu
@pytest.mark.parametrize("size", [(640, 480), (633, 355)])
def test_gpu_rectify_pair_calibrated_maps(engine, size):
    from stereovision_amd.rectify import StereoRectifier
    from stereovision_amd.synthetic import stereo_pair, to_bgr
    W, H = size
    K1, D1, K2, D2, R, T = _stereo_setup(1, size)
    R1, R2, P1, P2, Q, _, _ = calib.stereo_rectify(K1, D1, K2, D2, size, R, T, alpha=0)
    rect = StereoRectifier.from_calibration(K1, D1, R1, P1, K2, D2, R2, P2, size, engine)
    L, Rr, _ = stereo_pair(H, W, 64, seed=2)
    for l, r in ((L, Rr), (to_bgr(L), to_bgr(Rr))):
        ol, orr = rect.rectify(l, r)
        lm1, lm2, rm1, rm2 = rect.host_maps()
        np.testing.assert_array_equal(ol, RO.remap_linear(l, lm1, lm2))
        np.testing.assert_array_equal(orr, RO.remap_linear(r, rm1, rm2))
    rect.close()


@pytest.mark.gpu
def test_gpu_remap_gray_out_batch(engine):
    """Device path: BGR frames -> rectified gray in one pass, a batch of frames per launch,
    unaligned source pitch."""
    rng = np.random.default_rng(9)
    nf, sH, sW, H, W = 3, 50, 70, 44, 68
    pitch = sW * 3 + 1
    frames = rng.integers(0, 256, (nf, sH, pitch), dtype=np.uint8)
    m1, m2 = _random_maps(H, W, sH, sW, 4)
    d_src = engine.dev_alloc(frames.nbytes)
    d_m1 = engine.dev_alloc(m1.nbytes)
    d_m2 = engine.dev_alloc(m2.nbytes)
    d_out = engine.dev_alloc(nf * H * W)
    try:
        engine.to_device(d_src, frames)
        engine.to_device(d_m1, m1)
        engine.to_device(d_m2, m2)
        engine.remap_dev(d_src, sH, sW, 3, pitch, d_m1, d_m2, H, W, d_out, W, gray_out=True,
                         n_frames=nf, src_frame_stride=sH * pitch, dst_frame_stride=H * W)
        got = engine.to_host(d_out, (nf, H, W), np.uint8)
    finally:
        for p in (d_src, d_m1, d_m2, d_out):
            engine.dev_free(p)
    for z in range(nf):
        bgr = np.ascontiguousarray(frames[z, :, :sW * 3].reshape(sH, sW, 3))
        np.testing.assert_array_equal(got[z], RO.remap_gray(bgr, m1, m2))


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", [((480, 640), (356, 633)), ((1080, 1920), (356, 633)),
                                     ((480, 640), (240, 320)), ((120, 160), (481, 639)),
                                     ((37, 53), (37, 29)), ((5, 3), (1, 1)), ((33, 47), (66, 94))])
@pytest.mark.parametrize("channels", [1, 3])
def test_gpu_resize_matches_oracle(engine, src, dst, channels):
    rng = np.random.default_rng(src[0] * 7 + dst[1] + channels)
    a = rng.integers(0, 256, src + ((3,) if channels == 3 else ()), dtype=np.uint8)
    np.testing.assert_array_equal(engine.resize(a, dst[1], dst[0]), RO.resize_linear(a, dst[1], dst[0]))


@pytest.mark.gpu
def test_gpu_dropin_loaders_and_rectification(tmp_path):
    from stereovision_amd import depth_map, fused_depth_map, rectify
    from stereovision_amd.synthetic import stereo_pair, to_bgr
    d = _calib_dict(size=(320, 240), seed=2)
    p = tmp_path / "stereo_calibration_data.pkl"
    with open(p, "wb") as f:
        pickle.dump(d, f)
    c = rectify.load_stereo_calibration(str(p))
    assert c is not None and c["img_size"] == (320, 240)
    assert c["left_map1"].shape == (240, 320, 2) and c["left_map1"].dtype == np.int16
    R1, R2, P1, P2, Q, roi1, roi2 = calib.stereo_rectify(d["mtx_left"], d["dist_left"], d["mtx_right"],
                                                          d["dist_right"], (320, 240), d["R"], d["T"], alpha=0)
    e1, e2, _, _ = RO.undistort_rectify_map(d["mtx_left"], d["dist_left"], R1, P1, 320, 240)
    np.testing.assert_array_equal(c["left_map1"], e1)
    np.testing.assert_array_equal(c["left_map2"], e2)
    L, R, _ = stereo_pair(240, 320, 32, seed=3)
    bl, br = to_bgr(L), to_bgr(R)
    ol, orr = depth_map.apply_stereo_rectification(bl, br, c)
    np.testing.assert_array_equal(ol, RO.remap_linear(bl, c["left_map1"], c["left_map2"]))
    np.testing.assert_array_equal(orr, RO.remap_linear(br, c["right_map1"], c["right_map2"]))
    # a frame at another size is resized to the calibration size first (depth_map.py:808-811)
    big = to_bgr(stereo_pair(480, 640, 32, seed=4)[0])
    ol2, _ = depth_map.apply_stereo_rectification(big, big, c)
    np.testing.assert_array_equal(ol2, RO.remap_linear(RO.resize_linear(big, 320, 240),
                                                       c["left_map1"], c["left_map2"]))
    # fused app: scaled calibration, maps at int(w*s) x int(h*s)
    cs = fused_depth_map.load_stereo_calibration_with_scaling(0.5, str(p))
    assert cs["img_size_proc"] == (160, 120) and cs["left_map1"].shape == (120, 160, 2)
    ol3, _ = fused_depth_map.apply_stereo_rectification(bl, br, cs)
    np.testing.assert_array_equal(ol3, RO.remap_linear(RO.resize_linear(bl, 160, 120),
                                                       cs["left_map1"], cs["left_map2"]))


@pytest.mark.gpu
@pytest.mark.parametrize("size", [(1920, 1080), (1001, 397)])
def test_gpu_remap_staged_tiles_and_fallback_blocks(engine, size):
    """k_remap stages each 64x16 output tile's source footprint in LDS when it fits and reads
    its taps from global memory otherwise.  Calibrated maps (small footprints: staged), a
    band of invalid map entries (huge footprints: those blocks fall back), ragged edge tiles,
    BGR and gray sources, the fused gray output over a batch — all bit-exact."""
    W, H = size
    K1, D1, K2, D2, R, T = _stereo_setup(4, size)
    R1, R2, P1, P2, Q, _, _ = calib.stereo_rectify(K1, D1, K2, D2, size, R, T, alpha=0)
    m1, m2, _, _ = RO.undistort_rectify_map(K1, D1, R1, P1, W, H)
    m1 = m1.copy()
    m1[H // 3:H // 3 + 5, W // 4:W // 4 + 70] = (-32768, 32767)     # invalid entries
    m1[-7:, -3:] = (W + 500, -400)                                  # far outside the image
    rng = np.random.default_rng(W)
    bgr = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    gray = np.ascontiguousarray(bgr[..., 1])
    np.testing.assert_array_equal(engine.remap(bgr, m1, m2), RO.remap_linear(bgr, m1, m2))
    np.testing.assert_array_equal(engine.remap(gray, m1, m2), RO.remap_linear(gray, m1, m2))
    nf = 2
    frames = np.stack([bgr, bgr[::-1].copy()])
    d_src = engine.dev_alloc(frames.nbytes)
    d_m1 = engine.dev_alloc(m1.nbytes)
    d_m2 = engine.dev_alloc(m2.nbytes)
    d_out = engine.dev_alloc(nf * H * W)
    try:
        engine.to_device(d_src, frames)
        engine.to_device(d_m1, np.ascontiguousarray(m1))
        engine.to_device(d_m2, np.ascontiguousarray(m2))
        engine.remap_dev(d_src, H, W, 3, 3 * W, d_m1, d_m2, H, W, d_out, W, gray_out=True,
                         n_frames=nf, src_frame_stride=3 * H * W, dst_frame_stride=H * W)
        got = engine.to_host(d_out, (nf, H, W), np.uint8)
    finally:
        for p in (d_src, d_m1, d_m2, d_out):
            engine.dev_free(p)
    for z in range(nf):
        np.testing.assert_array_equal(got[z], RO.remap_gray(frames[z], m1, m2))
