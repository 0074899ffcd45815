"""bench.py's kernel-busy figure (CPU): the union of a kernel's dispatch intervals in a
rocprofv3 kernel trace, so overlapping launches of two lanes are not double counted."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

HEAD = ('"Kind","Agent_Id","Queue_Id","Stream_Id","Thread_Id","Dispatch_Id","Kernel_Id","Kernel_Name",'
        '"Correlation_Id","Start_Timestamp","End_Timestamp"\n')


def _trace(tmp_path, spans, name="sv::k_match_ring<4, 32, true, false, false>(sv::MatchParams)"):
    d = tmp_path / "trace" / "host"
    d.mkdir(parents=True)
    rows = [HEAD]
    for i, (a, b) in enumerate(spans):
        rows.append(f'"KERNEL_DISPATCH","Agent 2",1,1,1,{i},7,"{name}",{i},{a},{b}\n')
        rows.append(f'"KERNEL_DISPATCH","Agent 2",1,1,1,{i},8,"k_median_i16<0>(short const*)",{i},{b},{b + 50}\n')
    (d / "trace_kernel_trace.csv").write_text("".join(rows))
    return str(tmp_path)


def test_busy_is_the_union_of_overlapping_launches(tmp_path):
    # 8 launches, two lanes: each 1000 ns long, lane 1 starting 500 ns after lane 0, so the
    # union of every pair is 1500 ns; the first quarter (2 launches) is warm-up
    spans = []
    for k in range(4):
        t = 10_000 * k
        spans += [(t, t + 1000), (t + 500, t + 1500)]
    r = bench.kernel_busy(_trace(tmp_path, spans), "k_match")
    assert r["busy_launches"] == 6
    assert r["busy_us_per_launch"] == round(3 * 1500 / 6 / 1e3, 2)
    assert r["busy_overlap"] == round(6000 / 4500, 3)


def test_busy_of_serial_launches_is_their_duration(tmp_path):
    spans = [(2000 * k, 2000 * k + 700) for k in range(8)]
    r = bench.kernel_busy(_trace(tmp_path, spans), "k_match")
    assert r["busy_us_per_launch"] == 0.7 and r["busy_overlap"] == 1.0


def test_busy_needs_a_trace(tmp_path):
    assert bench.kernel_busy(str(tmp_path), "k_match") == {}
