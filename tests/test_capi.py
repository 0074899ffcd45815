"""CPU checks of the C-ABI boundary: header <-> binding <-> exported symbols, host-only
entry points (no compute without a GPU), and the loud failure when no GPU is visible."""
import ctypes
import os
import re

import pytest

from stereovision_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "stereovision_amd.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sv_\w+)\s*\(", text)))


def test_header_declares_exactly_the_bound_symbols():
    assert header_functions() == sorted(E.EXPORTED)


def test_library_builds_and_exports_every_declared_symbol():
    if not os.path.exists(E.LIB_PATH):
        pytest.skip("libsvhip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(E.LIB_PATH)
    missing = [s for s in header_functions() if not hasattr(lib, s)]
    assert not missing, missing
    out = os.popen(f"nm -D --defined-only {E.LIB_PATH}").read()
    exported = set(re.findall(r"\bT (sv_\w+)", out))
    assert set(header_functions()) <= exported


def test_library_targets_gfx950():
    if not os.path.exists(E.LIB_PATH):
        pytest.skip("libsvhip.so not built")
    blob = open(E.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_version_and_plan_without_gpu():
    lib = E.load_library()
    assert lib.sv_version() == 1
    assert E.plan(128, 9) == {"dpl": 8, "lpg": 16, "lds_bytes": E.plan(128, 9)["lds_bytes"]}
    assert E.plan(64, 9)["dpl"] == 4 and E.plan(64, 9)["lpg"] == 16
    assert E.plan(96, 5)["dpl"] == 6
    assert E.plan(256, 15)["lpg"] == 32
    assert E.plan(320, 7)["lpg"] == 64
    assert E.plan(128, 9)["lds_bytes"] <= 160 * 1024
    for D, win, cost in [(128, 9, "sad"), (256, 15, "ssd"), (64, 3, "hog"), (512, 15, "sad")]:
        assert E.plan(D, win, cost)["lds_bytes"] <= 160 * 1024


@pytest.mark.parametrize("D,win,cost", [(0, 9, "sad"), (600, 9, "sad"), (64, 8, "sad"),
                                         (64, 17, "sad"), (64, 9, 7)])
def test_plan_rejects_bad_parameters(D, win, cost):
    with pytest.raises(E.SVError) as ei:
        E.plan(D, win, cost)
    assert ei.value.code == -22
    assert E.last_error()


def test_key_range_is_checked():
    with pytest.raises(E.SVError) as ei:
        E.plan(512, 15, "ssd")      # 15*15*255^2 << 9 overflows the 32-bit argmin key
    assert ei.value.code == -34


def test_key_range_with_padding_disparities():
    # D=256 fills the (8 x 32) lane plan exactly: (cmax << 8) fits
    assert E.plan(256, 15, "ssd")["dpl"] * E.plan(256, 15, "ssd")["lpg"] == 256
    # D=200 leaves padding disparities whose keys start at (cmax + 1) << 8: overflows
    with pytest.raises(E.SVError) as ei:
        E.plan(200, 15, "ssd")
    assert ei.value.code == -34
    E.plan(200, 15, "sad")


def test_engine_fails_loudly_without_gpu():
    if E.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(E.EngineUnavailable):
        E.Engine(0)


def test_missing_library_is_loud(tmp_path):
    with pytest.raises(E.EngineUnavailable):
        E.load_library(str(tmp_path / "nope.so"))


def test_null_context_is_rejected_not_crashing():
    lib = E.load_library()
    assert lib.sv_synchronize(None) == -22
    assert lib.sv_profile_reset(None) == -22
    assert "null context" in E.last_error()
