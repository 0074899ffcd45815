"""The comparator networks k_median_i16 runs (stereovision_amd/csrc/sv_median_net.h, written
by gen_median_net.py), checked on the CPU as the kernel composes them: per column pair SEL16H
over the 4 common sorted columns, per window MRG14 with its own column, then the unique-row
merge -> medianBlur(5)'s median of 25 (cv2.medianBlur, depth_map.py:912).  0-1 principle
over every sorted-column binary input, plus random integer windows."""
import itertools
import os
import random
import re

HDR = os.path.join(os.path.dirname(__file__), "..", "stereovision_amd", "csrc", "sv_median_net.h")


def _arr(src, name):
    m = re.search(name + r"\[[^\]]*\](?:\[\d+\])?\s*=\s*\{(.*?)\};", src, re.S)
    assert m, name
    body = m.group(1)
    if "{" in body:
        return [tuple(int(x) for x in t.split(",")) for t in re.findall(r"\{([^{}]*)\}", body)]
    return [int(x) for x in body.split(",") if x.strip()]


SRC = open(HDR).read()
SEL16H, SEL16H_OUT = _arr(SRC, "SV_SEL16H_NET"), _arr(SRC, "SV_SEL16H_OUT")
MRG14, MRG14_OUT = _arr(SRC, "SV_MRG14_NET"), _arr(SRC, "SV_MRG14_OUT")
SORT4 = _arr(SRC, "SV_SORT4_NET")


def _run(net, v):
    v = list(v)
    for a, b, use in net:
        lo, hi = min(v[a], v[b]), max(v[a], v[b])
        if use & 1:
            v[a] = lo
        if use & 2:
            v[b] = hi
    return v


def _sort4(v):
    v = list(v)
    for a, b in SORT4:
        if v[a] > v[b]:
            v[a], v[b] = v[b], v[a]
    return v


def test_sel16h_zero_one_over_sorted_columns():
    for ks in itertools.product(range(5), repeat=4):   # ones per sorted column of 4
        v = [1 if i >= 4 - ks[c] else 0 for c in range(4) for i in range(4)]
        out = [_run(SEL16H, v)[o] for o in SEL16H_OUT]
        assert out == sorted(v)[3:13], ks


def test_mrg14_zero_one_over_sorted_inputs():
    for ka in range(11):
        for kc in range(5):
            v = [1 if i >= 10 - ka else 0 for i in range(10)] + [1 if i >= 4 - kc else 0 for i in range(4)]
            out = [_run(MRG14, v)[o] for o in MRG14_OUT]
            assert out == sorted(v)[4:10], (ka, kc)


def _pair_medians(grid):
    """medians of the windows at columns 0..4 and 1..5 of a 5x6 block, as the kernel does"""
    shared = [_sort4([grid[i][j] for i in range(1, 5)]) for j in range(6)]
    common = [shared[1 + c][i] for c in range(4) for i in range(4)]
    a = [_run(SEL16H, common)[o] for o in SEL16H_OUT]
    sc = _sort4(grid[0][1:5])
    out = []
    for w, own in ((0, shared[0]), (1, shared[5])):
        z = _run(MRG14, a + own)
        c = [z[o] for o in MRG14_OUT]
        u = sc + [grid[0][5 if w else 0]]
        for k in range(3, -1, -1):   # insertion of u[4]
            if u[k] > u[k + 1]:
                u[k], u[k + 1] = u[k + 1], u[k]
        out.append(min([c[5]] + [max(c[i], u[4 - i]) for i in range(5)]))
    return out


def test_pair_form_is_the_median_of_25_random_windows():
    rng = random.Random(7)
    for t in range(3000):
        lo, hi = (-40, 40) if t % 2 else (-3, 3)   # many ties in half the cases
        grid = [[rng.randint(lo, hi) for _ in range(6)] for _ in range(5)]
        m0, m1 = _pair_medians(grid)
        assert m0 == sorted(v for row in grid for v in row[0:5])[12]
        assert m1 == sorted(v for row in grid for v in row[1:6])[12]
