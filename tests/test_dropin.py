"""CPU tests of the drop-in host logic (reference interface, error convention, preamble).
A fake engine stands in for the GPU only to exercise the host-side control flow; every
numeric result of the real path is checked on the GPU in test_gpu_parity.py."""
import numpy as np
import pytest

import sv_oracle as O
from stereovision_amd import depth_map as DM
from stereovision_amd import fused_depth_map as FDM
from stereovision_amd import colormap, preamble
from stereovision_amd.engine import EngineUnavailable, SVError
from stereovision_amd.synthetic import stereo_pair, to_bgr


class OracleEngine:
    """Routes the drop-in's engine calls to the CPU oracle (test double, CPU tests only)."""

    def depth_map(self, gl, gr, min_disp, num_disp, win, min_depth, max_depth,
                  min_disp_global=None, cost="sad"):
        return O.create_depth_map(gl, gr, min_disp, num_disp, win, min_depth, max_depth)

    def stereo_scaled(self, gl, gr, min_disp, num_disp, win, cost="sad"):
        dn, disp, du, cf = O.create_depth_map_stereo_scaled(gl, gr, min_disp, num_disp, win)
        return dn, disp, du, cf

    def depth_map_color(self, gl, gr, min_disp, num_disp, win, min_depth, max_depth, cmap_bgr,
                        min_disp_global=None, cost="sad"):
        depth, disp, norm = self.depth_map(gl, gr, min_disp, num_disp, win, min_depth, max_depth)
        return depth, disp, np.asarray(cmap_bgr)[norm]

    def stereo_scaled_color(self, gl, gr, min_disp, num_disp, win, cmap_bgr, cost="sad"):
        dn, disp, du, cf = self.stereo_scaled(gl, gr, min_disp, num_disp, win)
        return dn, disp, np.asarray(cmap_bgr)[du], cf

    def gray(self, bgr):
        return O.bgr_to_gray(bgr)


class FailingEngine(OracleEngine):
    def depth_map(self, *a, **k):
        raise SVError("sv_depth_map", -5, "injected")

    def stereo_scaled(self, *a, **k):
        raise SVError("sv_stereo_scaled", -5, "injected")

    depth_map_color = depth_map
    stereo_scaled_color = stereo_scaled


def test_reference_globals_and_signatures():
    import inspect
    assert (DM.MIN_DISP, DM.NUM_DISP, DM.WINDOW_SIZE) == (0, 320, 7)       # depth_map.py:31-33
    assert FDM.PROCESSING_SCALE == 0.33                                    # fused_depth_map.py:39
    assert list(inspect.signature(DM.create_depth_map).parameters) == \
        ["left_img", "right_img", "stereo_calib", "min_depth", "max_depth"]
    assert list(inspect.signature(FDM.create_depth_map_stereo_scaled).parameters) == \
        ["left_img", "right_img", "min_disp", "num_disp", "window_size"]
    assert FDM.scaled_stereo_params() == (96, 5)


def test_missing_gpu_is_loud_not_zeros(monkeypatch):
    def boom(*a, **k):
        raise EngineUnavailable("no GPU")
    monkeypatch.setattr(DM, "get_engine", boom)
    monkeypatch.setattr(FDM, "get_engine", boom)
    L = np.zeros((8, 8, 3), np.uint8)
    with pytest.raises(EngineUnavailable):
        DM.create_depth_map(L, L)
    with pytest.raises(EngineUnavailable):
        FDM.create_depth_map_stereo_scaled(L, L, 0, 16, 5)


def test_create_depth_map_host_flow(monkeypatch):
    monkeypatch.setattr(DM, "get_engine", lambda: OracleEngine())
    monkeypatch.setattr(DM, "NUM_DISP", 32)
    monkeypatch.setattr(DM, "WINDOW_SIZE", 5)
    L, R, _ = stereo_pair(30, 100, 32, seed=1)
    depth, disp, cmap = DM.create_depth_map(to_bgr(L), to_bgr(R), None, 0.2, 4.0)
    e_depth, e_disp, e_norm = O.create_depth_map(L, R, 0, 32, 5, 0.2, 4.0)
    np.testing.assert_array_equal(depth, e_depth)
    np.testing.assert_array_equal(disp, e_disp)
    assert cmap.shape == (30, 100, 3) and cmap.dtype == np.uint8
    np.testing.assert_array_equal(cmap, colormap.table("turbo")[e_norm])
    assert depth.dtype == np.float32 and disp.dtype == np.float32


def test_per_frame_errors_return_zeros(monkeypatch, capsys):
    monkeypatch.setattr(DM, "get_engine", lambda: FailingEngine())
    monkeypatch.setattr(FDM, "get_engine", lambda: FailingEngine())
    L = np.zeros((10, 12, 3), np.uint8)
    depth, disp, cmap = DM.create_depth_map(L, L)
    assert depth.shape == (10, 12) and not depth.any() and not disp.any()
    assert cmap.shape == (10, 12, 3)
    dn, d, c, conf = FDM.create_depth_map_stereo_scaled(L, L, 0, 16, 5)
    for a in (dn, d, conf):
        assert a.shape == (10, 12) and a.dtype == np.float32 and not a.any()
    assert "injected" in capsys.readouterr().out


def test_scaled_host_flow(monkeypatch):
    monkeypatch.setattr(FDM, "get_engine", lambda: OracleEngine())
    L, R, _ = stereo_pair(24, 120, 48, seed=2)
    dn, disp, cmap, conf = FDM.create_depth_map_stereo_scaled(to_bgr(L), to_bgr(R), 0, 48, 5)
    e = O.create_depth_map_stereo_scaled(L, R, 0, 48, 5)
    np.testing.assert_array_equal(dn, e[0])
    np.testing.assert_array_equal(disp, e[1])
    np.testing.assert_array_equal(conf, e[3])
    assert cmap.shape == (24, 120, 3)


def test_mixed_gray_and_bgr_inputs(monkeypatch):
    monkeypatch.setattr(DM, "get_engine", lambda: OracleEngine())
    monkeypatch.setattr(DM, "NUM_DISP", 16)
    L, R, _ = stereo_pair(20, 60, 16, seed=3)
    a = DM.create_depth_map(to_bgr(L), R)
    b = DM.create_depth_map(L, R)
    np.testing.assert_array_equal(a[1], b[1])


def test_preamble_non_uint8_inputs_follow_reference():
    f = np.array([[[10.6, 20.2, 300.0]]], np.float32)
    g = preamble.to_engine_image(f)
    exp = np.uint8(np.clip(np.float32(10.6) * np.float32(0.114) + np.float32(20.2) * np.float32(0.587)
                           + np.float32(300.0) * np.float32(0.299), 0, 255))
    assert g.dtype == np.uint8 and g[0, 0] == exp
    u = np.zeros((4, 4, 3), np.uint8)
    assert preamble.to_engine_image(u) is u
    with pytest.raises(ValueError):
        preamble.to_engine_image(np.zeros((4, 4, 4), np.uint8))


def test_ensure_same_size_passthrough():
    a = np.zeros((10, 20), np.uint8)
    x, y = preamble.ensure_same_size(a, a)
    assert x is a and y is a
    with pytest.raises(TypeError):          # no host resize path: uint8 frames go to the GPU
        preamble.resize_linear(np.zeros((4, 4), np.float32), 2, 2)


def test_colormaps():
    u = np.arange(256, dtype=np.uint8).reshape(16, 16)
    for name in ("turbo", "jet"):
        c = colormap.apply(u, name)
        assert c.shape == (16, 16, 3) and c.dtype == np.uint8
        np.testing.assert_array_equal(c, colormap.table(name)[u])
    jet = colormap.apply(np.array([[0, 255]], np.uint8), "jet")
    assert jet[0, 0, 0] > jet[0, 0, 2] and jet[0, 1, 2] > jet[0, 1, 0]   # blue -> red (BGR)
