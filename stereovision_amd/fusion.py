"""Reductions on either side of the disparity path, on the GPU.

Drop-ins for fused_depth_map.py's
  detect_camera_occlusion(left, right, occlusion_threshold=0.45)          :131-301
  calibrate_midas_to_stereo(midas_depth, stereo_disparity, stereo_conf)   :1169-1257
  normalize_to_stereo_range(depth_map, stereo_disparity)                  :1503-1554
with the reference's arguments, return values and decisions.

* The occlusion statistics come from one ``k_frame_stats`` launch per pair: exact integer
  moments of every 48x48 block and the 256-bin histogram of each image.  np.mean and the
  entropy are then exact (the histogram is what cv2.calcHist returns and the entropy is
  the reference's NumPy expression over it); np.std is evaluated from the exact moments
  (sqrt((n*Q - S^2) / n^2)), i.e. the correctly rounded value, where NumPy's two-pass sum
  may differ in the last bits (tests: rtol 1e-12); the "std < 12" block test is done
  exactly on the integers.
* np.percentile is split the way NumPy computes it: the GPU finds the order statistics
  (``k_select_hist``, radix select with the reference's masks as predicates — the masked
  array is never built), and the interpolation runs here with NumPy's own dtype rules for
  the 'linear' method (scalar q on float32 -> float32 arithmetic, a list of q -> float64),
  so results are bit-identical to np.percentile.
* The elementwise epilogues run in ``k_affine_f32`` with the reference's precision.

Inputs are host NumPy arrays (as in the reference); ``*_dev`` variants take device
pointers for pipelines that keep the maps in HBM.
"""
from __future__ import annotations

import math

import numpy as np

from .engine import get_engine

SEL_ALL, SEL_POSITIVE, SEL_MASK_GT = 0, 1, 2
AFF_F32, AFF_F64, AFF_FILL = 0, 1, 2


# ----------------------------------------------------------------------------------------
# np.percentile from GPU order statistics
# ----------------------------------------------------------------------------------------
def percentile_dev(eng, d_x: int, n: int, q, mask_mode: int = SEL_ALL, d_mask: int = 0,
                   thr: float = 0.0, dtype=np.float32):
    """np.percentile(x[mask], q) (method 'linear') of a float32 device array."""
    sel, nans = eng.select_count(d_x, n, mask_mode, d_mask, thr)
    if sel + nans == 0:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")   # NumPy's error
    # numpy/lib/_function_base_impl.py: percentile -> _quantile (method 'linear')
    qa = np.asanyarray(np.true_divide(q, dtype(100)))
    if np.any(qa < 0) or np.any(qa > 1):
        raise ValueError("Percentiles must be in the range [0, 100]")
    cnt = sel + nans
    vi = np.asanyarray((cnt - 1) * qa)
    prev = np.asanyarray(np.floor(vi))
    nxt = np.asanyarray(prev + 1)
    above = vi >= cnt - 1
    if above.any():
        prev[above] = -1
        nxt[above] = -1
    below = vi < 0
    if below.any():
        prev[below] = 0
        nxt[below] = 0
    prev = prev.astype(np.intp)
    nxt = nxt.astype(np.intp)
    if nans:
        out = np.full(vi.shape, np.nan, dtype)
        return out[()] if out.ndim == 0 else out
    pr = np.where(prev < 0, cnt - 1, prev).ravel()
    nr = np.where(nxt < 0, cnt - 1, nxt).ravel()
    ranks = np.unique(np.concatenate([pr, nr]))
    vals = {}
    for i in range(0, ranks.size, 4):
        chunk = ranks[i:i + 4]
        for r, v in zip(chunk, eng.select_ranks(d_x, n, chunk, mask_mode, d_mask, thr)):
            vals[int(r)] = v
    previous = np.array([vals[int(r)] for r in pr], dtype).reshape(vi.shape)
    nextv = np.array([vals[int(r)] for r in nr], dtype).reshape(vi.shape)
    gamma = np.asanyarray(vi - prev)
    gamma = np.asanyarray(gamma, dtype=vi.dtype)
    # _lerp
    diff_b_a = np.subtract(nextv, previous)
    res = np.asanyarray(np.add(previous, diff_b_a * gamma))
    np.subtract(nextv, diff_b_a * (1 - gamma), out=res, where=gamma >= 0.5, casting="unsafe",
                dtype=type(res.dtype))
    if res.ndim == 0:
        res = res[()]
    return res


def percentile(x: np.ndarray, q, positive: bool = False):
    """np.percentile(x[x > 0] if positive else x, q) of a float32 host array, on the GPU."""
    x = np.ascontiguousarray(x)
    if x.dtype != np.float32:
        raise TypeError(f"percentile: float32 maps only, got {x.dtype}")
    eng = get_engine()
    d_x = eng.upload("pct_x", x)
    return percentile_dev(eng, d_x, x.size, q, SEL_POSITIVE if positive else SEL_ALL)


# ----------------------------------------------------------------------------------------
# detect_camera_occlusion   fused_depth_map.py:131-301
# ----------------------------------------------------------------------------------------
def _std_from_moments(n: int, s: int, q: int) -> float:
    return math.sqrt((n * q - s * s) / (n * n))


def occlusion_metrics(block_sum, block_sq, hist, H: int, W: int) -> dict:
    """The five per-camera metrics of detect_camera_occlusion from exact moments."""
    bh, bw = block_sum.shape
    bsize = 48
    hs = [min((i + 1) * bsize, H) - i * bsize for i in range(bh)]
    ws = [min((j + 1) * bsize, W) - j * bsize for j in range(bw)]
    stds, low = [], 0
    for i in range(bh):
        for j in range(bw):
            n = hs[i] * ws[j]
            s, q = int(block_sum[i, j]), int(block_sq[i, j])
            stds.append(_std_from_moments(n, s, q))
            low += (n * q - s * s) < 144 * n * n          # np.std(block) < 12, exactly
    avg_std = np.mean(stds) if stds else 0
    low_var_ratio = low / max(len(stds), 1)
    h = hist.astype(np.int64)
    N = int(h.sum())
    levels = np.arange(256, dtype=np.int64)
    S = int((h * levels).sum())
    Q = int((h * levels * levels).sum())
    contrast = np.float64(_std_from_moments(N, S, Q))
    # compute_entropy (fused_depth_map.py:230-241) on cv2.calcHist's float32 counts
    hf = hist.astype(np.float32).flatten() + 1e-10
    hf = hf / hf.sum()
    entropy = -np.sum(hf * np.log2(hf + 1e-10))
    brightness = np.float64(S) / N                        # np.mean(gray): exact integer sum
    return {"std": avg_std, "low_var": low_var_ratio, "contrast": contrast, "entropy": entropy,
            "brightness": brightness}


def occlusion_decision(L: dict, R: dict, occlusion_threshold: float = 0.45):
    """The scoring and decision block of fused_depth_map.py:243-301, verbatim."""
    STD_THRESHOLD = 28.0
    LOW_VAR_THRESHOLD = 0.55
    CONTRAST_RATIO = 2.2
    ENTROPY_RATIO = 1.6
    BRIGHTNESS_DIFF = 45.0
    ls = rs = 0.0
    if L["std"] < STD_THRESHOLD * 0.8:
        ls += 0.35
    if L["low_var"] > LOW_VAR_THRESHOLD:
        ls += 0.35
    if L["contrast"] < R["contrast"] / CONTRAST_RATIO and R["contrast"] > 15:
        ls += 0.25
    if L["entropy"] < R["entropy"] / ENTROPY_RATIO and R["entropy"] > 5.0:
        ls += 0.25
    if abs(L["brightness"] - R["brightness"]) > BRIGHTNESS_DIFF and L["brightness"] < 80:
        ls += 0.2
    if R["std"] < STD_THRESHOLD * 0.8:
        rs += 0.35
    if R["low_var"] > LOW_VAR_THRESHOLD:
        rs += 0.35
    if R["contrast"] < L["contrast"] / CONTRAST_RATIO and L["contrast"] > 15:
        rs += 0.25
    if R["entropy"] < L["entropy"] / ENTROPY_RATIO and L["entropy"] > 5.0:
        rs += 0.25
    if abs(R["brightness"] - L["brightness"]) > BRIGHTNESS_DIFF and R["brightness"] < 80:
        rs += 0.2
    if ls > occlusion_threshold and rs < occlusion_threshold * 0.6:
        result = "left"
    elif rs > occlusion_threshold and ls < occlusion_threshold * 0.6:
        result = "right"
    elif ls > occlusion_threshold and rs > occlusion_threshold:
        result = "both"
    else:
        result = "none"
    return result, ls, rs


def detect_camera_occlusion(left_img, right_img, occlusion_threshold=0.45):
    """fused_depth_map.py:131-301 -> (result, left_score, right_score)."""
    left_img = np.asarray(left_img)
    right_img = np.asarray(right_img)
    if left_img.dtype != np.uint8 or right_img.dtype != np.uint8:
        raise TypeError("detect_camera_occlusion: uint8 frames only")
    eng = get_engine()
    if left_img.shape == right_img.shape:
        bs, bq, hist = eng.frame_stats(left_img, right_img)
    else:
        a = eng.frame_stats(left_img)
        b = eng.frame_stats(right_img)
        bs, bq, hist = [a[0][0], b[0][0]], [a[1][0], b[1][0]], [a[2][0], b[2][0]]
    mets = [occlusion_metrics(bs[k], bq[k], hist[k], *(im.shape[:2]))
            for k, im in enumerate((left_img, right_img))]
    return occlusion_decision(mets[0], mets[1], occlusion_threshold)


# ----------------------------------------------------------------------------------------
# calibrate_midas_to_stereo / normalize_to_stereo_range   :1169-1257, :1503-1554
# ----------------------------------------------------------------------------------------
def _f32_map(a, name):
    a = np.ascontiguousarray(a)
    if a.dtype != np.float32:
        raise TypeError(f"{name}: float32 maps only, got {a.dtype}")
    return a


def _affine(eng, d_x: int, shape, mode: int, **kw) -> np.ndarray:
    n = int(np.prod(shape))
    d_out = eng.scratch("aff_out", 4 * n)
    eng.affine_f32_dev(d_x, n, mode, d_out, **kw)
    return eng.to_host(d_out, shape, np.float32)


def calibrate_midas_to_stereo(midas_depth, stereo_disparity, stereo_confidence):
    """fused_depth_map.py:1169-1257 (percentile calibration of a relative depth map to the
    stereo disparity range) with the reductions and the epilogue on the GPU."""
    if midas_depth is None or stereo_disparity is None:
        return None
    eng = get_engine()
    sd = _f32_map(stereo_disparity, "stereo_disparity")
    md = _f32_map(midas_depth, "midas_depth")
    H, W = sd.shape[:2]
    d_md = eng.upload("cal_midas", md)
    if md.shape != sd.shape:   # cv2.resize(..., INTER_LINEAR) (:1215-1217)
        d_rs = eng.scratch("cal_midas_rs", 4 * H * W)
        eng.resize_f32_dev(d_md, md.shape[0], md.shape[1], d_rs, H, W)
        d_md = d_rs
    n = H * W
    d_sd = eng.upload("cal_disp", sd)
    d_cf = eng.upload("cal_conf", _f32_map(stereo_confidence, "stereo_confidence"))
    sel, nans = eng.select_count(d_sd, n, SEL_MASK_GT, d_cf, 0.7)
    if sel + nans < 100:                       # np.sum(reliable_mask) < 100
        midas_min = percentile_dev(eng, d_md, n, 5)
        midas_max = percentile_dev(eng, d_md, n, 95)
        stereo_min = percentile_dev(eng, d_sd, n, 5)
        stereo_max = percentile_dev(eng, d_sd, n, 95)
        if (midas_max - midas_min) < 1e-6:
            c = np.full((1,), (stereo_min + stereo_max) / 2.0, np.float32)[0]
            return _affine(eng, d_md, (H, W), AFF_FILL, fc=c)
        den = midas_max - midas_min + 1e-8
        rng = stereo_max - stereo_min
        return _affine(eng, d_md, (H, W), AFF_F32, fa=midas_min, fb=den, fc=stereo_min, fd=rng)
    stereo_min, stereo_max = percentile_dev(eng, d_sd, n, [10, 90], SEL_MASK_GT, d_cf, 0.7)
    midas_min, midas_max = percentile_dev(eng, d_md, n, [10, 90], SEL_MASK_GT, d_cf, 0.7)
    if (midas_max - midas_min) < 1e-6:
        scale = 1.0
    else:
        scale = (stereo_max - stereo_min) / (midas_max - midas_min + 1e-8)
    offset = stereo_min - midas_min * scale
    return _affine(eng, d_md, (H, W), AFF_F64, ds=float(scale), doff=float(offset))


def normalize_to_stereo_range(depth_map, stereo_disparity):
    """fused_depth_map.py:1503-1554 with the reductions and the epilogue on the GPU."""
    if depth_map is None or stereo_disparity is None:
        return None
    eng = get_engine()
    sd = _f32_map(stereo_disparity, "stereo_disparity")
    dm = _f32_map(depth_map, "depth_map")
    d_sd = eng.upload("nrm_disp", sd)
    d_dm = eng.upload("nrm_depth", dm)
    sel, _ = eng.select_count(d_sd, sd.size, SEL_POSITIVE)
    if sel > 0:                                # np.any(stereo_valid)
        stereo_min = percentile_dev(eng, d_sd, sd.size, 5, SEL_POSITIVE)
        stereo_max = percentile_dev(eng, d_sd, sd.size, 95, SEL_POSITIVE)
    else:
        stereo_min, stereo_max = 0, 255
    d_min = percentile_dev(eng, d_dm, dm.size, 5)
    d_max = percentile_dev(eng, d_dm, dm.size, 95)
    if (d_max - d_min) < 1e-6:
        c = np.full((1,), (stereo_min + stereo_max) / 2.0, np.float32)[0]
        return _affine(eng, d_dm, dm.shape, AFF_FILL, fc=c)
    den = d_max - d_min + 1e-8
    rng = np.float32(stereo_max - stereo_min)
    return _affine(eng, d_dm, dm.shape, AFF_F32, fa=d_min, fb=den, fc=np.float32(stereo_min), fd=rng)
