"""Device-side multi-GPU paths of the C ABI, torch-free.

* sv_multi_gpu_dev, SV_SHARD_FRAMES (C4 from one process): every context computes create_depth_map
  for its resident frames and all outputs are gathered onto ctxs[0]'s device.
* sv_multi_gpu_dev, SV_SHARD_ROWS (C5 from one process): one frame row-tiled over the contexts, the
  bands gathered onto ctxs[0]'s device into the full frame.
* sv_comm_* (RCCL loaded with dlopen): a communicator per process (init_rank) and a group
  (init_all) on the devices this box has.
* the one-process-per-GPU launch of bench.py (torch.distributed.run starts the workers; the
  workers never import torch): ranks sharing this box's GPU fall back to the file store.
* the context scratch is ordered across streams (two parameter sets alternating on two
  streams of one context).

On a 1-GPU box the 8 "devices" are 8 contexts on device 0 (own stream and buffers each; the
gather degenerates to device copies); on an 8-GPU node the same tests spread them out.
Bar: bit-exact against the C oracle frame by frame.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd.engine import (POST_DEPTH, POST_NONE, POST_SCALED, Communicator, Engine,
                                     device_count, depth_map_rows_map, depth_map_rows_multi,
                                     multi_gpu_depth_map_dev, multi_gpu_m16_dev, multi_gpu_map_dev)
from stereovision_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle(L, R, D, win, cost="sad", lo=0.3, hi=2.0):
    d16 = C.disparity16(L, R, 0, D, win, {"sad": 0, "ssd": 1, "hog": 2}[cost])
    disp = C.median5_f32(d16)
    depth, norm = C.depth_post(disp, lo, hi)
    return disp, depth, norm


@pytest.fixture(scope="module")
def ctxs(engine):
    nd = max(1, device_count())
    extra = [Engine(k % nd) for k in range(1, 8)]
    yield [engine] + extra
    for e in extra:
        e.close()


def _upload(e, a):
    p = e.dev_alloc(a.nbytes)
    e.to_device(p, np.ascontiguousarray(a))
    return p


@pytest.mark.parametrize("ndev,counts,cost,win", [(8, [2, 1, 0, 3, 1, 1, 2, 1], "sad", 9),
                                                   (3, [1, 2, 1], "sad", 11),
                                                   (2, [2, 2], "hog", 7),
                                                   (1, [3], "ssd", 5)])
def test_multi_gpu_depth_map_dev_gathers_every_frame(ctxs, ndev, counts, cost, win):
    H, W, D = 45, 320, 64
    es = ctxs[:ndev]
    total = sum(counts)
    frames = [stereo_pair(H, W, D, seed=700 + f)[:2] for f in range(total)]
    dLs, dRs, f0 = [], [], 0
    for e, n in zip(es, counts):
        Ls = np.stack([frames[f0 + z][0] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        Rs = np.stack([frames[f0 + z][1] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        dLs.append(_upload(e, Ls))
        dRs.append(_upload(e, Rs))
        f0 += n
    root = es[0]
    n = H * W
    o_depth, o_disp, o_norm = root.dev_alloc(4 * n * total), root.dev_alloc(4 * n * total), root.dev_alloc(n * total)
    try:
        for _ in range(2):   # twice: the second call reuses every context's scratch
            multi_gpu_depth_map_dev(es, None, dLs, dRs, counts, H, W, W, H * W, 0, D, win, 0.3, 2.0,
                                    o_depth, o_disp, o_norm, cost=cost)
            root.synchronize()
        depth = root.to_host(o_depth, (total, H, W), np.float32)
        disp = root.to_host(o_disp, (total, H, W), np.float32)
        norm = root.to_host(o_norm, (total, H, W), np.uint8)
        for f, (L, R) in enumerate(frames):
            e_disp, e_depth, e_norm = _oracle(L, R, D, win, cost)
            np.testing.assert_array_equal(disp[f], e_disp, err_msg=f"frame {f}")
            np.testing.assert_array_equal(depth[f], e_depth, err_msg=f"frame {f}")
            np.testing.assert_array_equal(norm[f], e_norm, err_msg=f"frame {f}")
    finally:
        for e, a, b in zip(es, dLs, dRs):
            e.dev_free(a)
            e.dev_free(b)
        for p in (o_depth, o_disp, o_norm):
            root.dev_free(p)


@pytest.mark.parametrize("ndev,counts,cost,win", [(8, [2, 1, 0, 3, 1, 1, 2, 1], "sad", 9),
                                                   (3, [0, 2, 1], "hog", 7), (2, [1, 2], "ssd", 5),
                                                   (1, [2], "sad", 11)])
def test_multi_gpu_m16_dev_gathers_int16_medians(ctxs, ndev, counts, cost, win):
    """sv_multi_gpu_dev gather-only (out.med16): only the int16 x16 medians cross (2 B/px); they equal the C
    oracle's median map x 16 frame by frame, in context order."""
    H, W, D = 37, 300, 64
    es = ctxs[:ndev]
    total = sum(counts)
    frames = [stereo_pair(H, W, D, seed=900 + f)[:2] for f in range(total)]
    dLs, dRs, f0 = [], [], 0
    for e, n in zip(es, counts):
        Ls = np.stack([frames[f0 + z][0] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        Rs = np.stack([frames[f0 + z][1] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        dLs.append(_upload(e, Ls))
        dRs.append(_upload(e, Rs))
        f0 += n
    root = es[0]
    d_m16 = root.dev_alloc(2 * H * W * total)
    try:
        for _ in range(2):
            multi_gpu_m16_dev(es, None, dLs, dRs, counts, H, W, W, H * W, 0, D, win, d_m16, cost=cost)
            root.synchronize()
        m16 = root.to_host(d_m16, (total, H, W), np.int16)
        for f, (L, R) in enumerate(frames):
            e_disp = _oracle(L, R, D, win, cost)[0]
            np.testing.assert_array_equal(m16[f], (e_disp * 16).astype(np.int16), err_msg=f"frame {f}")
    finally:
        for e, a, b in zip(es, dLs, dRs):
            e.dev_free(a)
            e.dev_free(b)
        root.dev_free(d_m16)


@pytest.mark.parametrize("ndev,counts,cost,win,mind", [(8, [2, 1, 0, 3, 1, 1, 2, 1], "sad", 9, 0),
                                                        (3, [1, 0, 2], "hog", 7, 3), (2, [2, 1], "ssd", 5, -7),
                                                        (1, [2], "sad", 11, 0)])
def test_multi_gpu_map_dev_gathers_u8_indices(ctxs, ndev, counts, cost, win, mind):
    """sv_multi_gpu_dev gather-only (out.d8): the one-process C4 gather at 1 B/px — every frame's u8
    disparity index d - min_disp + 1 lands on ctxs[0]'s device in context order and encodes
    the C oracle's median map exactly (d8 + min_disp - 1)."""
    H, W, D = 37, 300, 48
    es = ctxs[:ndev]
    total = sum(counts)
    frames = [stereo_pair(H, W, D, seed=1300 + f)[:2] for f in range(total)]
    dLs, dRs, f0 = [], [], 0
    for e, n in zip(es, counts):
        Ls = np.stack([frames[f0 + z][0] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        Rs = np.stack([frames[f0 + z][1] for z in range(n)]) if n else np.zeros((1, H, W), np.uint8)
        dLs.append(_upload(e, Ls))
        dRs.append(_upload(e, Rs))
        f0 += n
    root = es[0]
    d_map = root.dev_alloc(H * W * total)
    try:
        for _ in range(2):
            multi_gpu_map_dev(es, None, dLs, dRs, counts, H, W, W, H * W, mind, D, win, d_map, fmt="d8",
                              cost=cost)
        root.synchronize()
        d8 = root.to_host(d_map, (total, H, W), np.uint8)
        for f, (L, R) in enumerate(frames):
            d16 = C.disparity16(L, R, mind, D, win, {"sad": 0, "ssd": 1, "hog": 2}[cost])
            np.testing.assert_array_equal(d8[f].astype(np.float32) + np.float32(mind - 1), C.median5_f32(d16),
                                          err_msg=f"frame {f}")
    finally:
        for e, a, b in zip(es, dLs, dRs):
            e.dev_free(a)
            e.dev_free(b)
        root.dev_free(d_map)


def test_back_to_back_gathers_without_sync(ctxs):
    """two enqueue-only C4 calls with peer-copy gathers, no synchronisation in
    between.  The peers' copies of call 2 into the root's receive buffer must wait until call
    1's expansion on the root stream has read it; both calls' outputs stay bit-exact (also the
    rows forms, which share the receive buffer)."""
    H, W, D, win = 41, 256, 64, 9
    es = ctxs[:4]
    n = H * W
    root = es[0]
    sets = []
    for c in range(2):
        fr = [stereo_pair(H, W, D, seed=1500 + 10 * c + k)[:2] for k in range(len(es))]
        sets.append((fr, [_upload(e, f[0]) for e, f in zip(es, fr)], [_upload(e, f[1]) for e, f in zip(es, fr)]))
    outs = [[root.dev_alloc(4 * n * len(es)), root.dev_alloc(4 * n * len(es)), root.dev_alloc(n * len(es))]
            for _ in range(2)]
    rows_out = [[root.dev_alloc(4 * n), root.dev_alloc(4 * n), root.dev_alloc(n)] for _ in range(2)]
    try:
        for rep in range(3):
            for c in range(2):
                _, dLs, dRs = sets[c]
                multi_gpu_depth_map_dev(es, None, dLs, dRs, [1] * len(es), H, W, W, n, 0, D, win, 0.3, 2.0,
                                        *outs[c])
            for c in range(2):
                _, dLs, dRs = sets[c]
                depth_map_rows_multi(es, None, dLs, dRs, H, W, W, 0, D, win, 0.3, 2.0, *rows_out[c])
            root.synchronize()
            for c in range(2):
                fr = sets[c][0]
                for k, (L, R) in enumerate(fr):
                    e_disp, e_depth, e_norm = _oracle(L, R, D, win)
                    np.testing.assert_array_equal(root.to_host(outs[c][1] + 4 * n * k, (H, W), np.float32), e_disp)
                    np.testing.assert_array_equal(root.to_host(outs[c][0] + 4 * n * k, (H, W), np.float32), e_depth)
                    np.testing.assert_array_equal(root.to_host(outs[c][2] + n * k, (H, W), np.uint8), e_norm)
                # rows form: every context holds its own frame, so band k is frame k's rows
                got = root.to_host(rows_out[c][1], (H, W), np.float32)
                for k in range(len(es)):   # band k comes from context k's frame
                    r0, r1 = H * k // len(es), H * (k + 1) // len(es)
                    np.testing.assert_array_equal(got[r0:r1], _oracle(*fr[k], D, win)[0][r0:r1])
    finally:
        for _, dLs, dRs in sets:
            for e, a, b in zip(es, dLs, dRs):
                e.dev_free(a)
                e.dev_free(b)
        for o in outs + rows_out:
            for p in o:
                root.dev_free(p)


@pytest.mark.parametrize("ndev,H,cost,win,fmt,scatter", [(8, 131, "sad", 9, "d8", True), (3, 29, "sad", 15, "m16", True),
                                                         (4, 57, "hog", 5, "d8", False), (2, 64, "ssd", 7, "m16", False),
                                                         (1, 40, "sad", 9, "d8", True), (8, 131, "sad", 9, "d8", "host"),
                                                         (3, 29, "ssd", 15, "m16", "host"), (1, 40, "hog", 7, "d8", "host")])
def test_depth_map_rows_map_gather_only(ctxs, ndev, H, cost, win, fmt, scatter):
    """sv_multi_gpu_dev (SV_SHARD_ROWS), gather-only: the root receives only the full-frame map
    (int16 x16 / u8 indices): its own band from its median epilogue, the peers' bands gathered;
    nothing is expanded.  Twice (the second call reuses scratch), with the frame on every
    context, scattered from the root (SV_INPUTS_SCATTER) or uploaded by every context from
    host memory (SV_INPUTS_HOST)."""
    W, D = 400, 64
    L, R, _ = stereo_pair(H, W, D, seed=ndev * 31 + H)
    es = ctxs[:ndev]
    root = es[0]
    el = 1 if fmt == "d8" else 2
    if scatter == "host":
        dL, dR = np.ascontiguousarray(L), np.ascontiguousarray(R)
        srcs = []
    elif scatter:
        dL, dR = _upload(root, L), _upload(root, R)
        srcs = [(root, dL), (root, dR)]
    else:
        dL, dR = [_upload(e, L) for e in es], [_upload(e, R) for e in es]
        srcs = list(zip(es, dL)) + list(zip(es, dR))
    d_map = root.dev_alloc(el * H * W)
    try:
        for _ in range(2):
            depth_map_rows_map(es, None, dL, dR, H, W, W, 0, D, win, d_map, fmt=fmt, scatter=scatter, cost=cost)
        root.synchronize()
        e_disp = _oracle(L, R, D, win, cost)[0]
        if fmt == "d8":
            got = root.to_host(d_map, (H, W), np.uint8).astype(np.float32) - np.float32(1)
        else:
            got = root.to_host(d_map, (H, W), np.int16).astype(np.float32) / np.float32(16)
        np.testing.assert_array_equal(got, e_disp)
    finally:
        for e, p in srcs:
            e.dev_free(p)
        root.dev_free(d_map)


@pytest.mark.parametrize("fmt", ["d8", "m16"])
def test_gather_only_maps_with_empty_shares(ctxs, fmt):
    """Edge cases of the gather-only forms: a root with no frames of its own, peers with none,
    and a row tiling with more contexts than rows (empty bands), all bit-exact."""
    H, W, D, win = 5, 96, 16, 3
    L, R, _ = stereo_pair(H, W, D, seed=77)
    el = 1 if fmt == "d8" else 2
    root = ctxs[0]
    e_disp = _oracle(L, R, D, win)[0]
    dL = [_upload(e, L) for e in ctxs]
    dR = [_upload(e, R) for e in ctxs]
    d_map = root.dev_alloc(el * H * W * 2)
    try:
        counts = [0, 1, 0, 0, 0, 0, 1, 0]            # frame 0 from context 1, frame 1 from 6
        multi_gpu_map_dev(ctxs, None, dL, dR, counts, H, W, W, H * W, 0, D, win, d_map, fmt=fmt)
        root.synchronize()
        if fmt == "d8":
            got = root.to_host(d_map, (2, H, W), np.uint8).astype(np.float32) - np.float32(1)
        else:
            got = root.to_host(d_map, (2, H, W), np.int16).astype(np.float32) / np.float32(16)
        np.testing.assert_array_equal(got[0], e_disp)
        np.testing.assert_array_equal(got[1], e_disp)
        for scatter in (False, True):                # 8 contexts, 5 rows: 3 empty bands
            depth_map_rows_map(ctxs, None, dL[0] if scatter else dL, dR[0] if scatter else dR, H, W, W, 0,
                               D, win, d_map, fmt=fmt, scatter=scatter)
            root.synchronize()
            if fmt == "d8":
                got = root.to_host(d_map, (H, W), np.uint8).astype(np.float32) - np.float32(1)
            else:
                got = root.to_host(d_map, (H, W), np.int16).astype(np.float32) / np.float32(16)
            np.testing.assert_array_equal(got, e_disp)
    finally:
        for e, a, b in zip(ctxs, dL, dR):
            e.dev_free(a)
            e.dev_free(b)
        root.dev_free(d_map)


def test_median_map_dev_rows_and_formats(engine):
    """sv_median_rows_dev (out.med16 / out.d8): a row band's median written only as a map (int16 x16 / u8 indices)
    at full-frame offsets, rows outside the band untouched; num_disp > 255 refused for u8."""
    from stereovision_amd.engine import SVError
    H, W, D, win, md = 50, 210, 40, 7, -4
    L, R, _ = stereo_pair(H, W, D, seed=5)
    e, n = engine, H * W
    dL, dR, d16 = _upload(e, L), _upload(e, R), e.dev_alloc(2 * n)
    m16, d8 = e.dev_alloc(2 * n), e.dev_alloc(n)
    try:
        e.to_device(m16, np.full(n, 0x7777, np.int16))
        e.to_device(d8, np.full(n, 0xAB, np.uint8))
        e.disparity_dev(dL, dR, H, W, W, md, D, win, "sad", 0, H, d16, W)
        e.median_map_dev(d16, H, W, 9, 33, m16, "m16", min_disp=md, num_disp=D)
        e.median_map_dev(d16, H, W, 9, 33, d8, "d8", min_disp=md, num_disp=D)
        e.synchronize()
        exp = C.median5_f32(C.disparity16(L, R, md, D, win, 0))
        g16 = e.to_host(m16, (H, W), np.int16)
        g8 = e.to_host(d8, (H, W), np.uint8)
        np.testing.assert_array_equal(g16[9:33].astype(np.float32) / np.float32(16), exp[9:33])
        np.testing.assert_array_equal(g8[9:33].astype(np.float32) + np.float32(md - 1), exp[9:33])
        assert (g16[:9] == 0x7777).all() and (g16[33:] == 0x7777).all()
        assert (g8[:9] == 0xAB).all() and (g8[33:] == 0xAB).all()
        with pytest.raises(SVError):
            e.median_map_dev(d16, H, W, 0, H, d8, "d8", min_disp=0, num_disp=256)
    finally:
        for p in (dL, dR, d16, m16, d8):
            e.dev_free(p)


def test_depth_map_batch_d8_dev_indices(engine):
    """sv_depth_map_batch_dev with out.d8: u8 disparity indices d - min_disp + 1 beside the f32 outputs
    (whole-pixel disparities: d8 + min_disp - 1 == the f32 disparity exactly, 0 = invalid), for
    SAD, SSD and HOG, a negative min_disp and num_disp 255; SGBM and num_disp > 255 refused."""
    from stereovision_amd.engine import SVError
    for cost, D, win, mind in (("sad", 64, 9, 0), ("ssd", 48, 7, -5), ("hog", 32, 9, 3), ("sad", 255, 7, 0)):
        nf, H, W = 2, 40, 330
        L = np.stack([stereo_pair(H, W, D, seed=s)[0] for s in range(nf)])
        R = np.stack([stereo_pair(H, W, D, seed=s)[1] for s in range(nf)])
        n = H * W
        dL, dR = engine.dev_alloc(L.nbytes), engine.dev_alloc(R.nbytes)
        bufs = [engine.dev_alloc(4 * n * nf), engine.dev_alloc(4 * n * nf), engine.dev_alloc(n * nf),
                engine.dev_alloc(n * nf)]
        try:
            engine.to_device(dL, L)
            engine.to_device(dR, R)
            engine.depth_map_batch_dev(dL, dR, nf, H, W, W, n, mind, D, win, 0.3, 2.0, bufs[0], bufs[1],
                                       bufs[2], cost=cost, d_d8=bufs[3])
            engine.synchronize()
            disp = engine.to_host(bufs[1], (nf, H, W), np.float32)
            d8 = engine.to_host(bufs[3], (nf, H, W), np.uint8)
            np.testing.assert_array_equal(d8.astype(np.float32) + np.float32(mind - 1), disp)
            for z in range(nf):
                exp = C.disparity16(L[z], R[z], mind, D, win, {"sad": 0, "ssd": 1, "hog": 2}[cost])
                assert (exp % 16 == 0).all()
        finally:
            for p in [dL, dR] + bufs:
                engine.dev_free(p)
    p = engine.dev_alloc(64 * 64 * 4)
    try:
        for cost, D in (("sgbm", 64), ("sad", 256)):
            with pytest.raises(SVError):
                engine.depth_map_batch_dev(p, p, 1, 8, 8, 8, 64, 0, D, 5, 0.3, 2.0, p, p, p, cost=cost, d_d8=p)
    finally:
        engine.dev_free(p)


@pytest.mark.parametrize("mode", [POST_DEPTH, POST_SCALED, POST_NONE])
def test_post_m16_dev_equals_median_epilogue(engine, mode):
    """sv_post_m16_dev over the int16 x16 medians reproduces the median kernel's own
    epilogue byte for byte (the root's expansion of gathered maps), including a ragged
    pixel count and an output offset that defeats the 16-byte vector path."""
    H, W, D, win, md = 41, 203, 48, 7, -3
    L, R, _ = stereo_pair(H, W, D, seed=77)
    e, n = engine, H * W
    dL, dR = _upload(e, L), _upload(e, R)
    bufs = [e.dev_alloc(4 * n + 64) for _ in range(6)] + [e.dev_alloc(n + 64), e.dev_alloc(n + 64),
                                                          e.dev_alloc(2 * n + 64), e.dev_alloc(2 * n)]
    disp_a, a_a, b_a, disp_b, a_b, b_b, u_a, u_b, m16, d16 = bufs
    try:
        e.disparity_dev(dL, dR, H, W, W, md, D, win, "sad", 0, H, d16, W)
        kw = dict(min_depth=0.3, max_depth=2.0, min_disp_global=md, min_disp=md, num_disp=D)
        scaled = mode == POST_SCALED
        e.median_post_m16_dev(d16, H, W, 0, H, mode, d_disparity=disp_a,
                              d_out_a=a_a if mode else 0, d_out_u8=u_a if mode else 0,
                              d_out_b=b_a if scaled else 0, d_med16=m16, **kw)
        for off in (0, 4):   # element offset 4: 16-B f32 stores misaligned -> scalar path
            e.post_m16_dev(m16 + 2 * off, n - off, mode, d_disparity=disp_b + 4 * off,
                           d_out_a=(a_b + 4 * off) if mode else 0, d_out_u8=(u_b + off) if mode else 0,
                           d_out_b=(b_b + 4 * off) if scaled else 0, **kw)
            e.synchronize()
            got = e.to_host(disp_b, (n,), np.float32)[off:]
            np.testing.assert_array_equal(got, e.to_host(disp_a, (n,), np.float32)[off:])
            if mode:
                np.testing.assert_array_equal(e.to_host(a_b, (n,), np.float32)[off:],
                                              e.to_host(a_a, (n,), np.float32)[off:])
                np.testing.assert_array_equal(e.to_host(u_b, (n,), np.uint8)[off:],
                                              e.to_host(u_a, (n,), np.uint8)[off:])
            if scaled:
                np.testing.assert_array_equal(e.to_host(b_b, (n,), np.float32)[off:],
                                              e.to_host(b_a, (n,), np.float32)[off:])
        np.testing.assert_array_equal(e.to_host(m16, (n,), np.int16).astype(np.float32) / np.float32(16),
                                      e.to_host(disp_a, (n,), np.float32))
    finally:
        for p in (dL, dR, *bufs):
            e.dev_free(p)


def _rows_multi(es, comms, L, R, D, win, cost="sad"):
    H, W = L.shape
    dLs = [_upload(e, L) for e in es]
    dRs = [_upload(e, R) for e in es]
    root = es[0]
    n = H * W
    o = [root.dev_alloc(4 * n), root.dev_alloc(4 * n), root.dev_alloc(n)]
    try:
        depth_map_rows_multi(es, comms, dLs, dRs, H, W, W, 0, D, win, 0.3, 2.0, o[0], o[1], o[2],
                             cost=cost)
        root.synchronize()
        return (root.to_host(o[1], (H, W), np.float32), root.to_host(o[0], (H, W), np.float32),
                root.to_host(o[2], (H, W), np.uint8))
    finally:
        for e, a, b in zip(es, dLs, dRs):
            e.dev_free(a)
            e.dev_free(b)
        for p in o:
            root.dev_free(p)


def test_rows_host_inputs_full_outputs(ctxs):
    """SV_INPUTS_HOST with create_depth_map's outputs on the root (the peers' int16 bands
    expanded there): every context uploads its own band rows; bit-exact against the oracle."""
    H, W, D, win = 83, 330, 48, 11
    L, R, _ = stereo_pair(H, W, D, seed=123)
    root = ctxs[0]
    n = H * W
    outs = [root.dev_alloc(4 * n), root.dev_alloc(4 * n), root.dev_alloc(n)]
    try:
        for nd in (8, 3):
            depth_map_rows_multi(ctxs[:nd], None, L, R, H, W, W, 0, D, win, 0.3, 2.0, outs[0], outs[1], outs[2],
                                 scatter="host")
            root.synchronize()
            e_disp, e_depth, e_norm = _oracle(L, R, D, win)
            np.testing.assert_array_equal(root.to_host(outs[1], (H, W), np.float32), e_disp)
            np.testing.assert_array_equal(root.to_host(outs[0], (H, W), np.float32), e_depth)
            np.testing.assert_array_equal(root.to_host(outs[2], (H, W), np.uint8), e_norm)
    finally:
        for p in outs:
            root.dev_free(p)


def test_batch_stages_apart_equal_the_fused_call(ctxs):
    """sv_depth_map_batch_dev with SV_STAGE_MATCH on one context and SV_STAGE_MEDIAN on another
    (the bench's split schedule: the two launches of consecutive batches on two streams) gives
    the same outputs as SV_STAGE_ALL, for SAD and SSD; a separate stage needs d_disp16."""
    from stereovision_amd.engine import STAGE_MATCH, STAGE_MEDIAN, SVError, map_out, POST_DEPTH
    ea, eb = ctxs[0], ctxs[1]
    for cost, D, win in (("sad", 64, 9), ("ssd", 48, 7)):
        nf, H, W = 3, 44, 300
        L = np.stack([stereo_pair(H, W, D, seed=40 + s)[0] for s in range(nf)])
        R = np.stack([stereo_pair(H, W, D, seed=40 + s)[1] for s in range(nf)])
        n = H * W
        dL, dR = _upload(ea, L), _upload(ea, R)
        d16 = ea.dev_alloc(2 * n * nf)
        a = [ea.dev_alloc(4 * n * nf), ea.dev_alloc(4 * n * nf), ea.dev_alloc(n * nf)]
        b = [ea.dev_alloc(4 * n * nf), ea.dev_alloc(4 * n * nf), ea.dev_alloc(n * nf), ea.dev_alloc(2 * n * nf)]
        try:
            ea.depth_map_batch_dev(dL, dR, nf, H, W, W, n, 0, D, win, 0.3, 2.0, a[0], a[1], a[2], cost=cost)
            ea.depth_map_batch_ex(dL, dR, nf, H, W, W, n, 0, D, win, cost, STAGE_MATCH, d16, None)
            ea.event_record(0, ea.stream)
            ea.stream_wait_event(0, eb.stream)
            out = map_out(POST_DEPTH, b[1], b[0], b[2], med16=b[3], min_depth=0.3, max_depth=2.0,
                          min_disp_global=0)
            eb.depth_map_batch_ex(0, 0, nf, H, W, W, n, 0, D, win, cost, STAGE_MEDIAN, d16, out, stream=eb.stream)
            eb.synchronize()
            ea.synchronize()
            for x, y, dt in ((a[0], b[0], np.float32), (a[1], b[1], np.float32), (a[2], b[2], np.uint8)):
                np.testing.assert_array_equal(ea.to_host(x, (nf, H, W), dt), ea.to_host(y, (nf, H, W), dt))
            m16 = ea.to_host(b[3], (nf, H, W), np.int16)
            np.testing.assert_array_equal(m16.astype(np.float32) / np.float32(16),
                                          ea.to_host(a[1], (nf, H, W), np.float32))
            for z in range(nf):
                np.testing.assert_array_equal(ea.to_host(a[1] + 4 * n * z, (H, W), np.float32),
                                              _oracle(L[z], R[z], D, win, cost)[0])
            with pytest.raises(SVError):
                ea.depth_map_batch_ex(dL, dR, nf, H, W, W, n, 0, D, win, cost, STAGE_MATCH, 0, None)
        finally:
            for p in [dL, dR, d16] + a + b:
                ea.dev_free(p)


def test_median_rows_refuses_d8_for_sgbm_maps(engine):
    """u8 indices are whole-pixel disparities; an SGBM (sub-pixel) map is refused."""
    from stereovision_amd.engine import SVError
    H, W = 16, 64
    d16, d8 = engine.dev_alloc(2 * H * W), engine.dev_alloc(H * W)
    try:
        engine.to_device(d16, np.zeros((H, W), np.int16))
        engine.median_map_dev(d16, H, W, 0, H, d8, "d8", min_disp=0, num_disp=16, cost="sad")
        with pytest.raises(SVError):
            engine.median_map_dev(d16, H, W, 0, H, d8, "d8", min_disp=0, num_disp=16, cost="sgbm")
    finally:
        engine.dev_free(d16)
        engine.dev_free(d8)


@pytest.mark.parametrize("ndev,H,cost,win", [(8, 131, "sad", 9), (3, 29, "sad", 15),
                                               (8, 17, "hog", 5), (2, 64, "ssd", 7), (1, 40, "sad", 9)])
def test_depth_map_rows_multi_reassembles_bit_exactly(ctxs, ndev, H, cost, win):
    W, D = 400, 64
    L, R, _ = stereo_pair(H, W, D, seed=ndev * 100 + H)
    disp, depth, norm = _rows_multi(ctxs[:ndev], None, L, R, D, win, cost)
    e_disp, e_depth, e_norm = _oracle(L, R, D, win, cost)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


def test_c5_row_tiled_over_8_contexts_gathered_on_device_0(ctxs):
    """C5 (3840x2160, D=256, 15x15): 8 bands, gathered onto the first context's device."""
    L, R, _ = stereo_pair(2160, 3840, 256, seed=56)
    disp, depth, norm = _rows_multi(ctxs, None, L, R, 256, 15)
    e_disp, e_depth, e_norm = _oracle(L, R, 256, 15)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


def _rows_scatter(es, comms, L, R, D, win, cost="sad"):
    """sv_multi_gpu_dev with SV_INPUTS_SCATTER: the frame on es[0]'s device only; bands + halos scattered."""
    from stereovision_amd.engine import depth_map_rows_scatter
    H, W = L.shape
    root = es[0]
    dL, dR = _upload(root, L), _upload(root, R)
    n = H * W
    o = [root.dev_alloc(4 * n), root.dev_alloc(4 * n), root.dev_alloc(n)]
    try:
        depth_map_rows_scatter(es, comms, dL, dR, H, W, W, 0, D, win, 0.3, 2.0, o[0], o[1], o[2],
                               cost=cost)
        root.synchronize()
        return (root.to_host(o[1], (H, W), np.float32), root.to_host(o[0], (H, W), np.float32),
                root.to_host(o[2], (H, W), np.uint8))
    finally:
        root.dev_free(dL)
        root.dev_free(dR)
        for p in o:
            root.dev_free(p)


@pytest.mark.parametrize("ndev,H,cost,win", [(8, 131, "sad", 9), (3, 29, "sad", 15),
                                               (8, 57, "hog", 5), (2, 64, "ssd", 7), (1, 40, "sad", 9),
                                               (4, 96, "sad", 11), (8, 300, "hog", 15)])
def test_depth_map_rows_scatter_band_only_inputs(ctxs, ndev, H, cost, win):
    """Band-only inputs: context k > 0 holds just the input rows of its band (+ halos), in a
    scratch buffer whose spare rows hold the PREVIOUS call's frame (first call: a different
    frame), so any read outside the band's rows would break bit-exactness."""
    W, D = 400, 64
    Lx, Rx, _ = stereo_pair(H, W, D, seed=ndev * 100 + H + 1)
    _rows_scatter(ctxs[:ndev], None, Lx, Rx, D, win, cost)          # leaves stale rows behind
    L, R, _ = stereo_pair(H, W, D, seed=ndev * 100 + H)
    disp, depth, norm = _rows_scatter(ctxs[:ndev], None, L, R, D, win, cost)
    e_disp, e_depth, e_norm = _oracle(L, R, D, win, cost)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


def test_c5_row_tiled_band_inputs_over_8_contexts(ctxs):
    """C5 (3840x2160, D=256, 15x15) with band-only inputs scattered from the first context."""
    L, R, _ = stereo_pair(2160, 3840, 256, seed=57)
    disp, depth, norm = _rows_scatter(ctxs, None, L, R, 256, 15)
    e_disp, e_depth, e_norm = _oracle(L, R, 256, 15)
    np.testing.assert_array_equal(disp, e_disp)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(norm, e_norm)


def test_rccl_group_scatter_band_inputs(ctxs):
    """The scatter + gather of SV_INPUTS_SCATTER as RCCL groups over this box's
    distinct devices."""
    nd = max(1, device_count())
    devs = list(range(min(nd, 8)))
    comms = Communicator.init_all(devs)
    es = [next(e for e in ctxs if e.device == d) for d in devs]
    try:
        L, R, _ = stereo_pair(97, 350, 64, seed=19)
        disp, depth, norm = _rows_scatter(es, comms, L, R, 64, 9)
        e_disp, e_depth, e_norm = _oracle(L, R, 64, 9)
        np.testing.assert_array_equal(disp, e_disp)
        np.testing.assert_array_equal(depth, e_depth)
        np.testing.assert_array_equal(norm, e_norm)
    finally:
        for c in comms:
            c.close()


def test_multi_device_argument_checks(ctxs):
    from stereovision_amd.engine import SVError
    H, W = 16, 64
    z = np.zeros((H, W), np.uint8)
    d = _upload(ctxs[0], z)
    try:
        with pytest.raises(SVError):      # the same context twice
            depth_map_rows_multi([ctxs[0], ctxs[0]], None, [d, d], [d, d], H, W, W, 0, 16, 5, 0.3,
                                 2.0, d, d, d)
        with pytest.raises(SVError):      # SGBM cannot be row-tiled
            depth_map_rows_multi(ctxs[:2], None, [d, d], [d, d], H, W, W, 0, 16, 5, 0.3, 2.0, d, d,
                                 d, cost="sgbm")
    finally:
        ctxs[0].dev_free(d)


# ---- RCCL communicators --------------------------------------------------------------------
def test_rccl_single_rank_communicator(engine):
    assert Communicator.available()
    uid = Communicator.unique_id()
    assert len(uid) == 128
    c = Communicator.init_rank(0, 1, 0, uid)
    try:
        assert (c.rank, c.nranks, c.device) == (0, 1, 0)
        c.barrier()
        assert c.allreduce_max(3.25) == 3.25
        # gatherv on one rank: the root's own block is a device copy into place
        src = np.arange(1000, dtype=np.uint8)
        d_src, d_dst = _upload(engine, src), engine.dev_alloc(3000)
        engine.to_device(d_dst, np.zeros(3000, np.uint8))
        c.gatherv(d_src, 1000, d_dst, [1500], [1000])
        c.synchronize()
        out = engine.to_host(d_dst, (3000,), np.uint8)
        np.testing.assert_array_equal(out[1500:2500], src)
        assert not out[:1500].any() and not out[2500:].any()
        engine.dev_free(d_src)
        engine.dev_free(d_dst)
    finally:
        c.close()


def test_rccl_group_on_distinct_devices_rows_and_frames(ctxs):
    """ncclCommInitAll over this box's distinct devices; the gathers of both multi-device
    entry points then run as RCCL send/recv groups."""
    nd = max(1, device_count())
    devs = list(range(min(nd, 8)))
    comms = Communicator.init_all(devs)
    es = [next(e for e in ctxs if e.device == d) for d in devs]
    try:
        L, R, _ = stereo_pair(97, 350, 64, seed=9)
        disp, depth, norm = _rows_multi(es, comms, L, R, 64, 9)
        e_disp, e_depth, e_norm = _oracle(L, R, 64, 9)
        np.testing.assert_array_equal(disp, e_disp)
        np.testing.assert_array_equal(depth, e_depth)
        np.testing.assert_array_equal(norm, e_norm)
    finally:
        for c in comms:
            c.close()


# ---- the one-process-per-GPU launch ------------------------------------------------------------
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode,root_outputs,fmt,bands", [("frames", "m16", "auto", "scatter"),
                                                         ("frames", "m16", "i16", "scatter"),
                                                         ("frames", "full", "auto", "scatter"),
                                                         ("rowtile", "m16", "auto", "scatter"),
                                                         ("rowtile", "m16", "i16", "scatter"),
                                                         ("rowtile", "full", "auto", "scatter"),
                                                         ("rowtile", "m16", "auto", "host"),
                                                         ("rowtile", "full", "auto", "host")])
def test_bench_under_torch_distributed_run_two_ranks(mode, root_outputs, fmt, bands):
    """The driver's N>1 launch: torch.distributed.run starts 2 bench.py workers (torch-free).
    On a 1-GPU box both ranks share the GPU, so the group falls back to the file store (RCCL
    refuses two ranks on one device); on a multi-GPU box it is RCCL.  The gather is on by
    default (u8 disparity indices where exact, else int16 x16); rank 0 checks every rank's
    gathered maps (frames) / the reassembled frame from band-only inputs (rowtile) against the
    C oracle: `verified` must be true."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--height", "96", "--width", "400", "--num-disp", "64",
           "--frames", "2", "--batch", "2", "--mode", mode, "--no-live-pmc", "--no-aux",
           "--no-host-path", "--no-cpu-baseline", "--hang-timeout", "90", "--root-outputs", root_outputs,
           "--gather-format", fmt, "--band-inputs", bands]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["scaling"] == ("strong" if mode == "rowtile" else "weak")
    assert res["verified"] is True, res["verify"]
    d = res["distributed"]
    assert d["gather"] is True and d["process_model"] == "one process per GPU"
    if device_count() == 1:
        assert d["backend"] == "host" and d["rccl_ranks"] == 0 and "share a GPU" in d["rccl_reason"]
    else:
        assert d["backend"] == "rccl" and d["rccl_ranks"] == 2
    checked = res["verify"]["checked"]
    if mode == "frames":     # both ranks' first and last frame, from rank 0's gathered stacks
        assert sum("gathered on rank 0" in c for c in checked) == 4, checked
        full = root_outputs == "full"
        u8 = fmt == "auto" and not full   # D = 64: u8 indices are exact
        assert d["gather_format"] == ("u8 disparity index" if u8 else "int16 x16")
        assert d["gather_bytes_per_step"] == (1 if u8 else 2) * 96 * 400 * 2 * 1   # B/px, B frames, 1 peer
        assert d["root_outputs"] == root_outputs
        assert sum("expanded on rank 0" in c for c in checked) == (2 if full else 0), checked
        assert (d["root_expand_us_per_step"] is not None) == full
    elif root_outputs == "full":
        assert checked == ["full frame gathered on rank 0"]
        assert d["root_expand_us_per_step"] is not None
    else:    # gather-only row tiling: the map only, nothing expanded on rank 0
        assert checked == [f"full-frame map gathered on rank 0 ({d['gather_format']})"], checked
        assert d["gather_format"] == ("u8 disparity index" if fmt == "auto" else "int16 x16")
        assert d["root_expand_us_per_step"] is None


@pytest.mark.parametrize("ngpu,mode,root_outputs,fmt,bands", [(2, "frames", "m16", "auto", "scatter"),
                                                              (3, "frames", "full", "auto", "scatter"),
                                                              (3, "frames", "m16", "i16", "scatter"),
                                                              (4, "rowtile", "m16", "auto", "scatter"),
                                                              (3, "rowtile", "m16", "i16", "scatter"),
                                                              (2, "rowtile", "full", "auto", "scatter"),
                                                              (8, "rowtile", "m16", "auto", "host"),
                                                              (3, "rowtile", "full", "auto", "host")])
def test_bench_one_process_rehearsal(ngpu, mode, root_outputs, fmt, bands):
    """`bench.py --gpus N` without a launcher (ONE process drives N GPUs: the gather lanes, two
    context sets, sv_multi_gpu_dev in all its shard / input / output forms) on N logical GPUs of this box (--rehearse: contexts of the
    visible devices, gathers as device copies): runs end to end and every gathered map of the
    last step is bit-exact against the C oracle; the line reports the gather traffic — u8
    indices (1 B/px) by default, int16 x16 (2 B/px) with --gather-format i16 or full outputs."""
    H, W, B = 96, 400, 2
    cmd = [sys.executable, "bench.py", "--gpus", str(ngpu), "--rehearse", "--steps", "3",
           "--warmup", "1", "--height", str(H), "--width", str(W), "--num-disp", "64",
           "--frames", "4", "--batch", str(B), "--mode", mode, "--root-outputs", root_outputs,
           "--gather-format", fmt, "--band-inputs", bands,
           "--no-live-pmc", "--no-aux", "--no-host-path", "--no-cpu-baseline", "--hang-timeout", "90"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == ngpu and res["verified"] is True, res["verify"]
    d = res["distributed"]
    assert d["process_model"] == "one process, all devices" and d["gather"] is True
    assert d["root_outputs"] == root_outputs
    u8 = root_outputs == "m16" and fmt == "auto"
    assert d["gather_format"] == ("u8 disparity index" if u8 else "int16 x16")
    assert (d["root_expand_us_per_step"] is not None) == (root_outputs == "full")
    checked = res["verify"]["checked"]
    if mode == "frames":
        assert len(checked) == 2 * ngpu, checked
        assert d["gather_bytes_per_step"] == (1 if u8 else 2) * H * W * B * (ngpu - 1)
    else:
        band0 = H // ngpu
        assert d["gather_bytes_per_step"] == (1 if u8 else 2) * (H - band0) * W
        assert len(checked) == 1 and "gathered on device 0" in checked[0], checked


def test_bench_rccl_init_failure_falls_back_to_peer_copies():
    """when ncclCommInitAll fails, the one-process N-GPU bench gathers with
    hipMemcpyPeerAsync instead of exiting, names the fallback (backend "peer", rccl_reason) and
    still verifies its gathered maps (SV_RCCL_INIT_FAIL=1 forces the failure)."""
    import json
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--rehearse", "--steps", "3", "--warmup", "1",
           "--height", "96", "--width", "400", "--num-disp", "64", "--frames", "2", "--batch", "2",
           "--no-live-pmc", "--no-aux", "--no-host-path", "--no-cpu-baseline", "--hang-timeout", "90"]
    env = dict(os.environ, SV_RCCL_INIT_FAIL="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    d = res["distributed"]
    assert res["verified"] is True, res["verify"]
    assert d["backend"] == "peer" and d["rccl_ranks"] == 0
    assert "ncclCommInitAll failed" in d["rccl_reason"] and "SV_RCCL_INIT_FAIL" in d["rccl_reason"]
    # --require-rccl: the same failure ends the run
    r = subprocess.run(cmd + ["--require-rccl"], cwd=ROOT, capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode != 0 and "require-rccl" in (r.stdout + r.stderr)


def test_bench_single_gpu_verifies_its_timed_outputs():
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--height", "120",
           "--width", "400", "--num-disp", "64", "--frames", "4", "--batch", "2", "--no-live-pmc",
           "--no-aux", "--no-host-path", "--no-cpu-baseline", "--harris"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["verified"] is True and res["distributed"] is None
    assert len(res["verify"]["checked"]) == 4     # frames 0 and B-1: maps + Harris each


# ---- cross-stream ordering of the context scratch -----------------------------------
def test_two_parameter_sets_alternating_on_two_streams(engine):
    """One context, its post table and int16 scratch used from two streams with two
    parameter sets in turn: every result matches its own parameter set."""
    other = Engine(0)
    try:
        H, W, D, win = 540, 960, 64, 9
        L, R, _ = stereo_pair(H, W, D, seed=77)
        n = H * W
        dL, dR = _upload(engine, L), _upload(engine, R)
        outs = [[engine.dev_alloc(4 * n), engine.dev_alloc(4 * n), engine.dev_alloc(n)] for _ in range(6)]
        params = [(0.3, 2.0), (0.1, 0.9)]
        streams = [engine.stream, other.stream]
        exp = [_oracle(L, R, D, win, "sad", lo, hi) for lo, hi in params]
        for i, o in enumerate(outs):
            lo, hi = params[i % 2]
            engine.depth_map_dev(dL, dR, H, W, W, 0, D, win, lo, hi, o[0], o[1], o[2],
                                 stream=streams[(i // 2) % 2] if i % 3 else streams[i % 2])
        engine.synchronize()
        other.synchronize()
        for i, o in enumerate(outs):
            e_disp, e_depth, e_norm = exp[i % 2]
            np.testing.assert_array_equal(engine.to_host(o[1], (H, W), np.float32), e_disp, err_msg=str(i))
            np.testing.assert_array_equal(engine.to_host(o[0], (H, W), np.float32), e_depth, err_msg=str(i))
            np.testing.assert_array_equal(engine.to_host(o[2], (H, W), np.uint8), e_norm, err_msg=str(i))
        for o in outs:
            for p in o:
                engine.dev_free(p)
        engine.dev_free(dL)
        engine.dev_free(dR)
    finally:
        other.close()


def test_hog_band_only_inputs_both_histogram_kernels():
    """band-only inputs with cost=HOG through both histogram kernels (the
    column-run form and the 64x16 tile form, SV_HOG_STRIP=0, each in a child): a band buffer holds only
    the input rows [in0, in1) plus SV_BAND_MARGIN poisoned rows either side, the band's last
    16-row tile starts at its last disparity row ((h1 - h0 - 1) % 16 == 0 for rank 1), and the
    band's disparity rows equal the full-frame oracle's."""
    from stereovision_amd.distributed import band_layout
    H, W, D, win, world = 87, 300, 48, 7, 3
    assert (band_layout(H, 1, world, win)["h1"] - band_layout(H, 1, world, win)["h0"] - 1) % 16 == 0
    code = ("import sys, numpy as np; sys.path.insert(0, %r)\n"
            "from stereovision_amd.engine import get_engine, BAND_MARGIN\n"
            "from stereovision_amd.distributed import band_layout\n"
            "from stereovision_amd.synthetic import stereo_pair\n"
            "e = get_engine(0)\n"
            "H, W, D, win, world = %d, %d, %d, %d, %d\n"
            "L, R, _ = stereo_pair(H, W, D, seed=515)\n"
            "for k in range(world):\n"
            "    b = band_layout(H, k, world, win)\n"
            "    rows = b['in1'] - b['in0']\n"
            "    bufs, ptrs = [], []\n"
            "    for img in (L, R):\n"
            "        band = np.full((rows + 2 * BAND_MARGIN, W), 255, np.uint8)\n"
            "        band[BAND_MARGIN:BAND_MARGIN + rows] = img[b['in0']:b['in1']]\n"
            "        p = e.dev_alloc(band.nbytes); e.to_device(p, band); bufs.append(p)\n"
            "        ptrs.append(p + (BAND_MARGIN - b['in0']) * W)\n"
            "    out = e.dev_alloc(2 * H * W)\n"
            "    e.disparity_dev(ptrs[0], ptrs[1], H, W, W, 0, D, win, 'hog', b['h0'], b['h1'], out, W)\n"
            "    d = e.to_host(out, (H, W), np.int16)[b['h0']:b['h1']]\n"
            "    sys.stdout.buffer.write(d.tobytes())\n"
            "    for p in bufs + [out]: e.dev_free(p)\n") % (ROOT, H, W, D, win, world)
    L, R, _ = stereo_pair(H, W, D, seed=515)
    exp = C.disparity16(L, R, 0, D, win, 2)
    for strip in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120,
                           env=dict(os.environ, SV_HOG_STRIP=strip, SV_WARMUP_AT_IMPORT="0"))
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        off = 0
        for k in range(world):
            b = band_layout(H, k, world, win)
            n = (b["h1"] - b["h0"]) * W * 2
            got = np.frombuffer(r.stdout[off:off + n], np.int16).reshape(-1, W)
            off += n
            np.testing.assert_array_equal(got, exp[b["h0"]:b["h1"]], err_msg=f"strip={strip} rank {k}")
