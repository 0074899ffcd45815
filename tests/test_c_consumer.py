"""A C program as the consumer of the drop-in boundary (include/stereovision_amd.h).

examples/depth_map_c.c creates a context, runs sv_depth_map on a synthetic pair with a known
shift and checks the disparity map in C.  CPU: the header compiles as strict C99 and the
example compiles and links against libsvhip.so.  GPU: the binary runs (no Python or
PyTorch in the process) and every interior pixel recovers the shift.
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "stereovision_amd", "lib")
SRC = os.path.join(ROOT, "examples", "depth_map_c.c")
BIN = os.path.join(ROOT, "examples", "depth_map_c")


def _build(out):
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
           "-L", LIB_DIR, "-lsvhip", f"-Wl,-rpath,{LIB_DIR}", "-o", out]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=120)


def test_header_is_strict_c99(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = tmp_path / "hdr.c"
    src.write_text('#include "stereovision_amd.h"\nint main(void) { return sv_version() > 0 ? 0 : 1; }\n')
    r = subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I",
                        os.path.join(ROOT, "include"), "-c", str(src), "-o", str(tmp_path / "hdr.o")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def test_c_example_compiles_and_links(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    if not os.path.exists(os.path.join(LIB_DIR, "libsvhip.so")):
        pytest.skip("libsvhip.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    r = _build(str(tmp_path / "depth_map_c"))
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("480", "640", "64", "9", "5"), ("1080", "1920", "128", "9", "20"),
                                  ("97", "333", "48", "11", "3")])
def test_c_example_runs_bit_exact_shift(args, tmp_path):
    exe = BIN
    if not os.path.exists(exe):
        exe = str(tmp_path / "depth_map_c")
        r = _build(exe)
        assert r.returncode == 0, r.stderr
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatched"] == 0 and res["checked"] > 0 and res["rc"] == 0
