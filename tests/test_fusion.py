"""Reductions around the path: detect_camera_occlusion,
calibrate_midas_to_stereo, normalize_to_stereo_range.

The oracle is the reference's own NumPy code (oracle/sv_fusion_oracle.py).  Bar:
  * order statistics / percentiles / calibrated and normalised maps: bit-exact;
  * occlusion decision and scores: identical; metrics: mean/entropy exact, block and
    global std within rtol 1e-12 (NumPy's two-pass float sum vs the exact moments).
"""
import numpy as np
import pytest

import sv_fusion_oracle as FO
import sv_oracle as O
from stereovision_amd import fusion


class _HostSelect:
    """The select_count / select_ranks contract of the C ABI, on host arrays (to test the
    NumPy-percentile mirror without a GPU)."""

    def __init__(self):
        self.bufs = {}

    def put(self, a):
        k = len(self.bufs) + 1
        self.bufs[k] = np.ascontiguousarray(a, np.float32).ravel()
        return k

    def _sel(self, d_x, mode, d_mask, thr):
        x = self.bufs[d_x]
        if mode == fusion.SEL_POSITIVE:
            return x[x > 0], 0
        if mode == fusion.SEL_MASK_GT:
            x = x[self.bufs[d_mask] > np.float32(thr)]
        nan = int(np.isnan(x).sum())
        return x[~np.isnan(x)], nan

    def select_count(self, d_x, n, mode=0, d_mask=0, thr=0.0):
        s, nan = self._sel(d_x, mode, d_mask, thr)
        return s.size, nan

    def select_ranks(self, d_x, n, ranks, mode=0, d_mask=0, thr=0.0):
        s, _ = self._sel(d_x, mode, d_mask, thr)
        return np.sort(s)[np.asarray(ranks)]


def _arrays(seed):
    rng = np.random.default_rng(seed)
    yield rng.random(1001).astype(np.float32)
    yield (rng.normal(size=777) * 100).astype(np.float32)
    yield rng.integers(-5, 6, 500).astype(np.float32)                 # many ties
    yield np.array([3.5], np.float32)
    yield np.array([2.0, -0.0, 0.0, 1.0], np.float32)
    yield (rng.random(4099) * 1e-3).astype(np.float32)


@pytest.mark.parametrize("seed", [0, 1])
def test_percentile_mirror_matches_numpy(seed):
    eng = _HostSelect()
    for a in _arrays(seed):
        d = eng.put(a)
        for q in (0, 5, 10, 37.5, 50, 90, 95, 100, [10, 90], [5, 95], [0, 100]):
            got = fusion.percentile_dev(eng, d, a.size, q)
            exp = np.percentile(a, q)
            assert type(got) is type(exp) and np.asarray(got).dtype == np.asarray(exp).dtype
            np.testing.assert_array_equal(got, exp)
        pos = a[a > 0]
        if pos.size:
            np.testing.assert_array_equal(fusion.percentile_dev(eng, d, a.size, 5, fusion.SEL_POSITIVE),
                                          np.percentile(pos, 5))


def test_percentile_mirror_masks_and_nan():
    rng = np.random.default_rng(3)
    eng = _HostSelect()
    x = rng.normal(size=2000).astype(np.float32)
    conf = rng.random(2000).astype(np.float32)
    dx, dc = eng.put(x), eng.put(conf)
    np.testing.assert_array_equal(
        fusion.percentile_dev(eng, dx, x.size, [10, 90], fusion.SEL_MASK_GT, dc, 0.7),
        np.percentile(x[conf > 0.7], [10, 90]))
    x[17] = np.nan
    dn = eng.put(x)
    assert np.isnan(fusion.percentile_dev(eng, dn, x.size, 5)) and np.isnan(np.percentile(x, 5))


def _scene(H, W, seed, kind):
    rng = np.random.default_rng(seed)
    if kind == "texture":
        from stereovision_amd.synthetic import stereo_pair
        return stereo_pair(H, W, 32, seed)[0]
    if kind == "covered":          # a finger over the lens: dark, nearly flat
        return np.clip(20 + rng.normal(size=(H, W)) * 2, 0, 255).astype(np.uint8)
    if kind == "flat":
        return np.full((H, W), 128, np.uint8)
    return rng.integers(0, 256, (H, W), dtype=np.uint8)


@pytest.mark.parametrize("kinds", [("texture", "texture"), ("covered", "texture"),
                                   ("texture", "covered"), ("covered", "covered"),
                                   ("flat", "noise")])
def test_occlusion_metrics_from_moments(kinds):
    """Host half of the GPU path: metrics from exact moments vs the reference's NumPy."""
    H, W = 150, 250
    L, R = (_scene(H, W, i, k) for i, k in enumerate(kinds))
    mets = []
    for g in (L, R):
        bh, bw = max(1, H // 48), max(1, W // 48)
        bs = np.zeros((bh, bw), np.uint32)
        bq = np.zeros((bh, bw), np.uint32)
        for i in range(bh):
            for j in range(bw):
                blk = g[i * 48:min((i + 1) * 48, H), j * 48:min((j + 1) * 48, W)].astype(np.int64)
                bs[i, j], bq[i, j] = blk.sum(), (blk * blk).sum()
        hist = np.bincount(g.ravel(), minlength=256).astype(np.uint32)
        m = fusion.occlusion_metrics(bs, bq, hist, H, W)
        e = FO.occlusion_metrics(g)
        for k in ("std", "contrast"):
            np.testing.assert_allclose(m[k], e[k], rtol=1e-12)
        assert m["entropy"] == e["entropy"] and m["brightness"] == e["brightness"]
        assert m["low_var"] == e["low_var"]
        mets.append(m)
    assert fusion.occlusion_decision(*mets) == FO.detect_camera_occlusion(L, R)


def test_resize_f32_oracle_known_answers():
    z = np.full((30, 40), 2.5, np.float32)
    assert (FO.resize_linear_f32(z, 17, 11) == 2.5).all()
    a = np.arange(16, dtype=np.float32).reshape(4, 4)
    np.testing.assert_array_equal(FO.resize_linear_f32(a, 2, 2),
                                  np.array([[2.5, 4.5], [10.5, 12.5]], np.float32))


# ---------------------------------------------------------------------------- GPU parity
def _maps(H, W, seed, reliable=True):
    from stereovision_amd.synthetic import stereo_pair
    rng = np.random.default_rng(seed)
    d = (rng.integers(0, 64, (H, W)) + rng.random((H, W))).astype(np.float32)
    d[rng.random((H, W)) < 0.1] = -1.0                      # invalid pixels
    conf = (rng.random((H, W)) > (0.2 if reliable else 0.9995)).astype(np.float32)
    midas = (rng.random((H, W)) * 255).astype(np.float32)
    return d, conf, midas


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(480, 640), (47, 61), (1, 1), (96, 144), (1080, 1920)])
@pytest.mark.parametrize("channels", [1, 3])
def test_gpu_frame_stats_exact(engine, shape, channels):
    H, W = shape
    rng = np.random.default_rng(H + W + channels)
    a = rng.integers(0, 256, shape + ((3,) if channels == 3 else ()), dtype=np.uint8)
    b = rng.integers(0, 256, shape + ((3,) if channels == 3 else ()), dtype=np.uint8)
    bs, bq, hist = engine.frame_stats(a, b)
    for k, img in enumerate((a, b)):
        g = O.bgr_to_gray(img) if channels == 3 else img
        bh, bw = max(1, H // 48), max(1, W // 48)
        for i in range(bh):
            for j in range(bw):
                blk = g[i * 48:min((i + 1) * 48, H), j * 48:min((j + 1) * 48, W)].astype(np.int64)
                assert bs[k, i, j] == blk.sum() and bq[k, i, j] == (blk * blk).sum()
        np.testing.assert_array_equal(hist[k], np.bincount(g.ravel(), minlength=256))


@pytest.mark.gpu
@pytest.mark.parametrize("agg", ["0", "1", "2"])
def test_gpu_frame_stats_flat_and_mixed_regions(engine, agg):
    """The histogram adds' aggregation branches (SV_STATS_AGG, read at the first launch of a
    process: run in a child) on images built to hit each: flat tiles (one wave-uniform dword),
    tiles of 4-equal-byte dwords that differ across lanes, noisy-flat tiles (few distinct
    values), random tiles and ragged borders."""
    import subprocess, sys, os
    code = r"""
import sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
from stereovision_amd.engine import get_engine
rng = np.random.default_rng(5)
H, W = 250, 500
a = np.zeros((H, W), np.uint8)
a[:, :96] = 200                                            # flat tiles
a[:, 96:192] = np.repeat(rng.integers(0, 256, (H, 24), dtype=np.uint8), 4, axis=1)   # 4-equal dwords
a[:, 192:288] = 40 + rng.integers(0, 3, (H, 96), dtype=np.uint8)                     # noisy flat
a[:, 288:] = rng.integers(0, 256, (H, W - 288), dtype=np.uint8)                      # random
b = np.full((H, W), 7, np.uint8)
b[100:, 300:] = rng.integers(0, 256, (H - 100, W - 300), dtype=np.uint8)
bs, bq, hist = get_engine(0).frame_stats(a, b)
for k, g in enumerate((a, b)):
    assert np.array_equal(hist[k], np.bincount(g.ravel(), minlength=256)), k
    for i in range(H // 48):
        for j in range(W // 48):
            blk = g[i * 48:(i + 1) * 48, j * 48:(j + 1) * 48].astype(np.int64)
            assert bs[k, i, j] == blk.sum() and bq[k, i, j] == (blk * blk).sum(), (k, i, j)
print("ok")
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, SV_STATS_AGG=agg, SV_WARMUP_AT_IMPORT="0"))
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("nf,shape,channels,pair", [(8, (1080, 1920), 1, True), (3, (47, 61), 3, True),
                                                    (5, (480, 640), 1, False), (1, (96, 144), 1, True)])
def test_gpu_frame_stats_batch_equals_per_frame(engine, nf, shape, channels, pair):
    """sv_frame_stats_batch_dev: one launch over nf frames (pairs) == nf single calls."""
    H, W = shape
    rng = np.random.default_rng(nf * 1000 + H)
    ext = (3,) if channels == 3 else ()
    a = rng.integers(0, 256, (nf,) + shape + ext, dtype=np.uint8)
    b = rng.integers(0, 256, (nf,) + shape + ext, dtype=np.uint8)
    a[0] = 17                                         # a flat frame: one histogram bin
    fs = H * W * channels
    dA, dB = engine.dev_alloc(a.nbytes), engine.dev_alloc(b.nbytes)
    engine.to_device(dA, a)
    engine.to_device(dB, b)
    bh, bw = max(1, H // 48), max(1, W // 48)
    per = 2 if pair else 1
    nimg = nf * per
    dbs, dbq, dh = engine.dev_alloc(4 * nimg * bh * bw), engine.dev_alloc(4 * nimg * bh * bw), engine.dev_alloc(4 * nimg * 256)
    try:
        for _ in range(2):   # twice: the fold leaves the accumulators zeroed
            engine.frame_stats_batch_dev(dA, dB if pair else 0, nf, fs, H, W, channels, W * channels, dbs, dbq, dh)
            engine.synchronize()
        bs = engine.to_host(dbs, (nimg, bh, bw), np.uint32)
        bq = engine.to_host(dbq, (nimg, bh, bw), np.uint32)
        hist = engine.to_host(dh, (nimg, 256), np.uint32)
        for f in range(nf):
            e_bs, e_bq, e_h = engine.frame_stats(a[f], b[f]) if pair else engine.frame_stats(a[f])
            for k in range(per):
                z = f * per + k
                np.testing.assert_array_equal(bs[z], e_bs[k], err_msg=f"frame {f} image {k}")
                np.testing.assert_array_equal(bq[z], e_bq[k])
                np.testing.assert_array_equal(hist[z], e_h[k])
    finally:
        for p in (dA, dB, dbs, dbq, dh):
            engine.dev_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("kinds", [("texture", "texture"), ("covered", "texture"),
                                   ("texture", "covered"), ("covered", "covered"), ("flat", "noise")])
def test_gpu_detect_camera_occlusion(kinds):
    from stereovision_amd.synthetic import to_bgr
    L, R = (_scene(356, 633, i, k) for i, k in enumerate(kinds))
    for l, r in ((L, R), (to_bgr(L), to_bgr(R))):
        assert fusion.detect_camera_occlusion(l, r) == FO.detect_camera_occlusion(l, r)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 1000, 1 << 20, 1000003])
def test_gpu_select_ranks_exact(engine, n):
    rng = np.random.default_rng(n)
    x = (rng.normal(size=n) * 1e3).astype(np.float32)
    if n > 3:
        x[:n // 10] = x[0]                                   # ties
        x[n // 10] = -0.0
    d = engine.upload("t_x", x)
    s = np.sort(x)
    ranks = np.unique(np.array([0, n // 3, n // 2, n - 1]))
    np.testing.assert_array_equal(engine.select_ranks(d, n, ranks), s[ranks])
    assert engine.select_count(d, n, fusion.SEL_POSITIVE) == ((x > 0).sum(), 0)
    conf = rng.random(n).astype(np.float32)
    dc = engine.upload("t_c", conf)
    sm = np.sort(x[conf > np.float32(0.7)])
    if sm.size:
        np.testing.assert_array_equal(engine.select_ranks(d, n, [0, sm.size - 1], 2, dc, 0.7),
                                      sm[[0, sm.size - 1]])


@pytest.mark.gpu
@pytest.mark.parametrize("off", [1, 2, 3])
def test_gpu_select_unaligned_and_nan(engine, off):
    """Arrays not 16-byte aligned (the scalar path) and NaN counting, every mask mode."""
    n = 300001
    rng = np.random.default_rng(off)
    x = (rng.random(n) * 100 - 10).astype(np.float32)
    x[rng.integers(0, n, 50)] = np.nan
    conf = rng.random(n).astype(np.float32)
    d = engine.upload("t_x", x)
    dc = engine.upload("t_c", conf)
    xs, cs = x[off:], conf[off:]
    m = n - off
    assert engine.select_count(d + 4 * off, m) == ((~np.isnan(xs)).sum(), np.isnan(xs).sum())
    assert engine.select_count(d + 4 * off, m, fusion.SEL_POSITIVE) == ((xs > 0).sum(), 0)
    sel = cs > np.float32(0.7)
    assert engine.select_count(d + 4 * off, m, 2, dc + 4 * off, 0.7) == \
        ((sel & ~np.isnan(xs)).sum(), (sel & np.isnan(xs)).sum())
    pos = np.sort(xs[xs > 0])
    np.testing.assert_array_equal(engine.select_ranks(d + 4 * off, m, [0, pos.size // 2, pos.size - 1],
                                                      fusion.SEL_POSITIVE),
                                  pos[[0, pos.size // 2, pos.size - 1]])


@pytest.mark.gpu
@pytest.mark.parametrize("reliable", [True, False])
@pytest.mark.parametrize("shape", [(356, 633), (120, 160)])
def test_gpu_calibrate_and_normalize(reliable, shape):
    H, W = shape
    d, conf, midas = _maps(H, W, 7, reliable)
    np.testing.assert_array_equal(fusion.calibrate_midas_to_stereo(midas, d, conf),
                                  FO.calibrate_midas_to_stereo(midas, d, conf))
    np.testing.assert_array_equal(fusion.normalize_to_stereo_range(midas, d),
                                  FO.normalize_to_stereo_range(midas, d))
    # MiDaS at another resolution is resized first (fused_depth_map.py:1215-1217)
    small = np.ascontiguousarray(midas[::2, ::2][:H // 2 - 1, :W // 2 - 3])
    np.testing.assert_array_equal(fusion.calibrate_midas_to_stereo(small, d, conf),
                                  FO.calibrate_midas_to_stereo(small, d, conf))
    # no valid stereo pixels: the (0, 255) fallback range; a flat map: full_like
    neg = np.full((H, W), -1.0, np.float32)
    np.testing.assert_array_equal(fusion.normalize_to_stereo_range(midas, neg),
                                  FO.normalize_to_stereo_range(midas, neg))
    flat = np.full((H, W), 3.0, np.float32)
    np.testing.assert_array_equal(fusion.normalize_to_stereo_range(flat, d),
                                  FO.normalize_to_stereo_range(flat, d))
    assert fusion.calibrate_midas_to_stereo(None, d, conf) is None


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", [((120, 160), (356, 633)), ((480, 640), (240, 320)),
                                     ((37, 53), (19, 80))])
def test_gpu_resize_f32(engine, src, dst):
    rng = np.random.default_rng(src[0])
    a = (rng.random(src) * 255).astype(np.float32)
    d_a = engine.upload("rs_a", a)
    d_o = engine.scratch("rs_o", 4 * dst[0] * dst[1])
    engine.resize_f32_dev(d_a, src[0], src[1], d_o, dst[0], dst[1])
    got = engine.to_host(d_o, dst, np.float32)
    np.testing.assert_array_equal(got, FO.resize_linear_f32(a, dst[1], dst[0]))


@pytest.mark.gpu
@pytest.mark.parametrize("narr,n,mode", [(16, 1 << 18, 0), (3, 1000003, 1), (5, 4097, 2), (1, 777, 0)])
def test_gpu_select_batch_equals_single(engine, narr, n, mode):
    """sv_select_count_batch / sv_select_ranks_batch: per-array results == single calls."""
    rng = np.random.default_rng(narr * 31 + n)
    x = (rng.normal(size=(narr, n)) * 100).astype(np.float32)
    x[0, :7] = np.nan
    m = rng.random((narr, n)).astype(np.float32)
    dx, dm = engine.dev_alloc(x.nbytes), engine.dev_alloc(m.nbytes)
    engine.to_device(dx, x)
    engine.to_device(dm, m)
    try:
        sel, nan = engine.select_count_batch(dx, n, n, narr, mode, dm, n, 0.7)
        ranks = []
        for y in range(narr):
            s1, n1 = engine.select_count(dx + 4 * y * n, n, mode, dm + 4 * y * n, 0.7)
            assert (sel[y], nan[y]) == (s1, n1), y
            ranks.append([0, s1 // 3, s1 // 2, max(0, s1 - 1)])
        vals = engine.select_ranks_batch(dx, n, n, ranks, mode, dm, n, 0.7)
        for y in range(narr):
            single = engine.select_ranks(dx + 4 * y * n, n, ranks[y], mode, dm + 4 * y * n, 0.7)
            np.testing.assert_array_equal(vals[y], single, err_msg=f"array {y}")
            sel_y = x[y][(~np.isnan(x[y])) & ((x[y] > 0) if mode == 1 else (m[y] > 0.7) if mode == 2 else True)]
            np.testing.assert_array_equal(vals[y], np.sort(sel_y)[ranks[y]])
    finally:
        engine.dev_free(dx)
        engine.dev_free(dm)
