"""Generates sv_median_net.h: a comparator network selecting the median of 25 values.

Construction: Batcher's odd-even merge sort on 32 wires with wires 25..31 fixed at +inf,
constant-folded (comparators touching a +inf wire become no-ops or wire relabelings),
then pruned backwards to the comparators that can influence output wire 12.
Verification: the 0-1 principle for selection networks — the network returns the k-th
smallest of every input iff it does so for all 2^25 binary inputs — checked here
exhaustively (bit-sliced), plus random integer inputs.

Usage: python gen_median_net.py  (rewrites sv_median_net.h next to this file)
"""
from __future__ import annotations

import itertools
import os
import random


def batcher_pairs(n: int):
    pairs = []
    p = 1
    while p < n:
        k = p
        while k >= 1:
            for j in range(k % p, n - k, 2 * k):
                for i in range(min(k, n - j - k)):
                    if (i + j) // (2 * p) == (i + j + k) // (2 * p):
                        pairs.append((i + j, i + j + k))
            k //= 2
        p *= 2
    return pairs


def build(n_real: int = 25, n: int = 32, k: int = 12):
    # wire -> current label; constant-fold the +inf pads
    inf = [i >= n_real for i in range(n)]
    ops = []
    for a, b in batcher_pairs(n):
        if inf[a] and inf[b]:
            continue
        if inf[b]:          # min(real, inf) stays at a: no-op
            continue
        if inf[a]:          # pad moves to b, real value moves to a: relabel
            ops.append(("swap", a, b))
            inf[a], inf[b] = inf[b], inf[a]
            continue
        ops.append(("cmp", a, b))
    # resolve swaps by tracking a permutation of physical slots
    slot = list(range(n))   # logical wire -> physical slot
    cmps = []
    for op, a, b in ops:
        if op == "swap":
            slot[a], slot[b] = slot[b], slot[a]
        else:
            cmps.append((slot[a], slot[b]))
    out_slot = slot[k]
    # backward liveness pruning
    live = {out_slot}
    kept = []
    for a, b in reversed(cmps):
        need_a, need_b = a in live, b in live
        if need_a or need_b:
            # bit0: the min (to a) is consumed later, bit1: the max (to b) is consumed
            kept.append((a, b, int(need_a) | (int(need_b) << 1)))
            live.add(a)
            live.add(b)
    kept.reverse()
    assert all(s < n_real for s in live), "pruned network must only read real inputs"
    return kept, out_slot


def run(net, out_slot, vals):
    v = list(vals) + [None] * (32 - len(vals))
    for a, b, _ in net:
        x, y = v[a], v[b]
        v[a], v[b] = (x, y) if x <= y else (y, x)
    return v[out_slot]


def verify01(net, out_slot, n_real=25):
    # bit-sliced over 2^25 inputs: word w holds inputs (w<<6 .. w<<6|63) for wires 0..5;
    # wires 6..24 are enumerated by the outer loop over 2^19 values.
    low = []
    for i in range(6):
        m = 0
        for t in range(64):
            if (t >> i) & 1:
                m |= 1 << t
        low.append(m)
    full = (1 << 64) - 1
    for hi in range(1 << (n_real - 6)):
        v = low + [full if (hi >> (i - 6)) & 1 else 0 for i in range(6, n_real)] + [full] * 7
        for a, b, _ in net:
            x, y = v[a], v[b]
            v[a], v[b] = x & y, x | y
        res = v[out_slot]
        # expected: median bit = 1 iff at least 13 of the 25 inputs are 1
        ones_hi = bin(hi).count("1")
        need = 13 - ones_hi
        exp = 0
        for t in range(64):
            if bin(t).count("1") >= need:
                exp |= 1 << t
        if res != exp:
            return False
    return True


def build_sel(n_real: int, n: int, lo_pads: int, ranks: list[int]):
    """Batcher on n wires: `lo_pads` -inf pads below the real inputs (wires lo_pads ..
    lo_pads+n_real-1), +inf pads above; constant-folded, pruned to the wires that end up
    holding the given ranks (0-indexed among the real inputs), returned in rank order."""
    order = {"-": 0, "r": 1, "+": 2}
    kind = ["-"] * lo_pads + ["r"] * n_real + ["+"] * (n - lo_pads - n_real)
    ops = []
    for a, b in batcher_pairs(n):
        if kind[a] == "r" and kind[b] == "r":
            ops.append(("cmp", a, b))
        elif order[kind[a]] > order[kind[b]]:
            ops.append(("swap", a, b))
            kind[a], kind[b] = kind[b], kind[a]
    slot = list(range(n))
    cmps = []
    for op, a, b in ops:
        if op == "swap":
            slot[a], slot[b] = slot[b], slot[a]
        else:
            cmps.append((slot[a], slot[b]))
    outs = [slot[lo_pads + k] for k in ranks]
    live = set(outs)
    kept = []
    for a, b in reversed(cmps):
        need_a, need_b = a in live, b in live
        if need_a or need_b:
            kept.append((a, b, int(need_a) | (int(need_b) << 1)))
            live.add(a)
            live.add(b)
    kept.reverse()
    assert all(lo_pads <= w < lo_pads + n_real for w in live), "network reads a pad wire"
    # renumber real wires to 0..n_real-1
    net = [(a - lo_pads, b - lo_pads, u) for a, b, u in kept]
    return net, [o - lo_pads for o in outs]


def run_sel(net, outs, vals):
    v = list(vals)
    for a, b, _ in net:
        x, y = v[a], v[b]
        v[a], v[b] = (x, y) if x <= y else (y, x)
    return [v[o] for o in outs]


def verify01_sel(net, outs, n_real, ranks):
    """0-1 principle: output j must equal the ranks[j]-th smallest for all 2^n_real
    binary inputs (bit-sliced, 64 inputs per word)."""
    low = []
    for i in range(6):
        m = 0
        for t in range(64):
            if (t >> i) & 1:
                m |= 1 << t
        low.append(m)
    full = (1 << 64) - 1
    popc = [bin(t).count("1") for t in range(64)]
    for hi in range(1 << (n_real - 6)):
        v = low + [full if (hi >> (i - 6)) & 1 else 0 for i in range(6, n_real)]
        for a, b, _ in net:
            x, y = v[a], v[b]
            v[a], v[b] = x & y, x | y
        ones_hi = bin(hi).count("1")
        for o, k in zip(outs, ranks):
            # k-th smallest (0-indexed) is 1 iff the number of zeros <= k
            exp = 0
            for t in range(64):
                zeros = n_real - ones_hi - popc[t]
                if zeros <= k:
                    exp |= 1 << t
            if v[o] != exp:
                return False
    return True


# optimal 5-comparator sorting network for 4 inputs
SORT4 = [(0, 1), (2, 3), (0, 2), (1, 3), (1, 2)]


def sorted_column_inputs():
    """Bit-sliced 0-1 inputs of the 20 shared values v[i*5+j] (row i of the 4, column j of
    the 5) whose columns are sorted (v[j] <= v[5+j] <= v[10+j] <= v[15+j]): 5^5 = 3125 cases,
    one bit each.  Thresholding an integer input with sorted columns gives one of these, and
    min/max networks commute with thresholding, so a network that selects the right ranks
    for all of them selects them for every integer input with sorted columns."""
    import itertools
    cases = list(itertools.product(range(5), repeat=5))   # ones per column
    wires = [0] * 20
    for t, ks in enumerate(cases):
        for j, k in enumerate(ks):
            for i in range(4 - k, 4):
                wires[i * 5 + j] |= 1 << t
    return cases, wires


def build_sel20s(ranks, seeds=range(8)):
    """Ranks of the 20 shared values when each column of 4 arrives sorted (the columns are
    sorted once in LDS and shared by the 5 windows that read them).  Start: Batcher on 32
    wires with the 5 columns on its first five 4-wire blocks (+inf pads above), so its
    first two levels are exactly the column sorts; then drop comparators greedily (seeded
    order) while the outputs stay correct on every sorted-column 0-1 input; the cheapest
    seed (min/max op count after liveness pruning) wins."""
    import random
    cases, w0 = sorted_column_inputs()
    exp = []
    for k in ranks:
        m = 0
        for t, ks in enumerate(cases):
            if 20 - sum(ks) <= k:
                m |= 1 << t
        exp.append(m)
    base, outs = build_sel(20, 32, 0, ranks)
    v_of = {w: (w % 4) * 5 + (w // 4) for w in range(20)}   # Batcher wire -> v index
    net0 = [(v_of[a], v_of[b]) for a, b, _ in base]
    outs = [v_of[o] for o in outs]

    def ok(net):
        v = list(w0)
        for a, b in net:
            v[a], v[b] = v[a] & v[b], v[a] | v[b]
        return all(v[o] == e for o, e in zip(outs, exp))

    def liveness(net):
        live, kept, ops = set(outs), [], 0
        for a, b in reversed(net):
            na, nb = a in live, b in live
            if na or nb:
                kept.append((a, b, int(na) | (int(nb) << 1)))
                ops += 2 if na and nb else 1
                live.update((a, b))
        kept.reverse()
        return ops, kept

    assert ok(net0)
    best = None
    for seed in seeds:
        rng = random.Random(seed)
        net = list(net0)
        order = list(range(len(net)))
        rng.shuffle(order)
        drop = set()
        for i in order:
            if ok([c for k, c in enumerate(net) if k not in drop and k != i]):
                drop.add(i)
        ops, kept = liveness([c for k, c in enumerate(net) if k not in drop])
        if best is None or ops < best[0]:
            best = (ops, kept)
    assert ok([(a, b) for a, b, _ in best[1]])
    return best[1], outs, best[0]


def greedy_prune(net0, outs, w0, exp, seeds=range(16)):
    """Drop comparators of `net0` greedily (seeded orders) while every output wire still
    equals its expected bit-sliced 0-1 word; the cheapest seed after liveness pruning wins."""
    def ok(net):
        v = list(w0)
        for a, b in net:
            v[a], v[b] = v[a] & v[b], v[a] | v[b]
        return all(v[o] == e for o, e in zip(outs, exp))

    def liveness(net):
        live, kept, ops = set(outs), [], 0
        for a, b in reversed(net):
            na, nb = a in live, b in live
            if na or nb:
                kept.append((a, b, int(na) | (int(nb) << 1)))
                ops += 2 if na and nb else 1
                live.update((a, b))
        kept.reverse()
        return ops, kept

    assert ok(net0)
    best = None
    for seed in seeds:
        rng = random.Random(seed)
        order = list(range(len(net0)))
        rng.shuffle(order)
        drop = set()
        for i in order:
            if ok([c for k, c in enumerate(net0) if k not in drop and k != i]):
                drop.add(i)
        ops, kept = liveness([c for k, c in enumerate(net0) if k not in drop])
        if best is None or ops < best[0]:
            best = (ops, kept)
    assert ok([(a, b) for a, b, _ in best[1]])
    return best[1], best[0]


def build_sel16h():
    """Horizontal sharing (two adjacent windows x, x+1 of a row pair): their 20 shared values
    hold 4 common sorted columns (16 values).  The 13th of 25 has common rank 3..12 (9 values
    are outside the common 16), so the pair first takes sorted ranks 3..12 of the 16 (v[c*4+i],
    column c, rank i), once."""
    ranks = list(range(3, 13))
    base, outs = build_sel(16, 16, 0, ranks)
    cases = list(itertools.product(range(5), repeat=4))
    w0 = [0] * 16
    for t, ks in enumerate(cases):
        for c, k in enumerate(ks):
            for i in range(4 - k, 4):
                w0[c * 4 + i] |= 1 << t
    exp = [sum(1 << t for t, ks in enumerate(cases) if 16 - sum(ks) <= k) for k in ranks]
    net, ops = greedy_prune([(a, b) for a, b, _ in base], outs, w0, exp)
    return net, outs, ops


def build_merge10_4():
    """Per window: merge the pair's sorted ranks 3..12 (wires 0..9) with the window's own
    sorted column (wires 10..13) -> sorted ranks 4..9 of the 14 (the 5 unique-row values
    remain), i.e. the same 6 candidates SEL20S yields."""
    ranks = list(range(4, 10))
    base, outs = build_sel(14, 16, 0, ranks)
    cases = [(ka, kc) for ka in range(11) for kc in range(5)]
    w0 = [0] * 14
    for t, (ka, kc) in enumerate(cases):
        for i in range(10 - ka, 10):
            w0[i] |= 1 << t
        for i in range(4 - kc, 4):
            w0[10 + i] |= 1 << t
    exp = [sum(1 << t for t, (ka, kc) in enumerate(cases) if 14 - ka - kc <= k) for k in ranks]
    net, ops = greedy_prune([(a, b) for a, b, _ in base], outs, w0, exp)
    return net, outs, ops


# optimal 9-comparator sorting network for 5 inputs (Knuth, TAOCP 5.3.4)
SORT5 = [(0, 1), (3, 4), (2, 4), (2, 3), (1, 4), (0, 3), (0, 2), (1, 3), (1, 2)]


def main(check: bool = True):
    net, out_slot = build()
    rng = random.Random(0)
    for _ in range(2000):
        vals = [rng.randint(-40, 40) for _ in range(25)]
        assert run(net, out_slot, vals) == sorted(vals)[12]
    if check:
        assert verify01(net, out_slot), "0-1 principle check failed"
    # SEL20: sorted ranks 7..12 of 20 values (the shared 4x5 rows of two vertically
    # adjacent 5x5 windows: the 13th of 25 lies in ranks 7..12 of the shared 20 or among
    # the 5 rows unique to the window -> median = 6th of (6 sorted + 5 sorted))
    ranks = list(range(7, 13))
    sel, sel_out = build_sel(20, 32, 6, ranks)
    for _ in range(2000):
        vals = [rng.randint(-40, 40) for _ in range(20)]
        assert run_sel(sel, sel_out, vals) == sorted(vals)[7:13]
    for _ in range(2000):
        vals = [rng.randint(-9, 9) for _ in range(5)]
        v = list(vals)
        for a, b in SORT5:
            if v[a] > v[b]:
                v[a], v[b] = v[b], v[a]
        assert v == sorted(vals)
    if check:
        assert verify01_sel(sel, sel_out, 20, ranks), "SEL20 0-1 check failed"
    # SEL20S: the same ranks when every column of 4 is pre-sorted (k_median_i16)
    sels, sels_out, sels_ops = build_sel20s(ranks)
    for _ in range(4000):
        vals = [rng.randint(-40, 40) for _ in range(20)]
        cols = [sorted(vals[j::5]) for j in range(5)]
        srt = [cols[j][i] for i in range(4) for j in range(5)]
        assert run_sel(sels, sels_out, srt) == sorted(vals)[7:13]
    # horizontal pair form: SEL16H once per pair of windows + MERGE10_4 per window
    selh, selh_out, selh_ops = build_sel16h()
    mrg, mrg_out, mrg_ops = build_merge10_4()
    for _ in range(4000):
        vals = [rng.randint(-40, 40) for _ in range(25)]   # window: rows 0..4, columns 0..4
        grid = [vals[5 * i:5 * i + 5] for i in range(5)]
        shared = [sorted(grid[i][j] for i in range(1, 5)) for j in range(5)]   # 4 shared rows
        common = [shared[j][i] for j in range(1, 5) for i in range(4)]
        a = run_sel(selh, selh_out, common)
        c = run_sel(mrg, mrg_out, a + shared[0])
        u = sorted(grid[0])
        r = min([c[5]] + [max(c[i], u[4 - i]) for i in range(5)])
        assert r == sorted(vals)[12]
    here = os.path.dirname(os.path.abspath(__file__))
    lines = [
        "// Generated by gen_median_net.py — do not edit.",
        f"// Median-of-25 selection network: {len(net)} comparators (pruned Batcher odd-even",
        "// merge sort, 32 wires with 7 +inf pads constant-folded). Verified exhaustively",
        "// with the 0-1 principle over all 2^25 binary inputs.",
        "#pragma once",
        f"#define SV_MED25_NCMP {len(net)}",
        f"#define SV_MED25_OUT {out_slot}",
        f"// {sum(1 for c in net if c[2] == 3)} full comparators + "
        f"{sum(1 for c in net if c[2] != 3)} half (min-only / max-only) comparators",
        "// entry {a, b, use}: use bit0 -> wire a := min(a, b); bit1 -> wire b := max(a, b)",
        "static constexpr unsigned char SV_MED25_NET[SV_MED25_NCMP][3] = {",
    ]
    for a, b, u in net:
        lines.append(f"  {{{a}, {b}, {u}}},")
    lines.append("};")
    lines += [
        "",
        f"// Ranks 7..12 (sorted) of 20 values: {len(sel)} comparators ({sum(2 if c[2] == 3 else 1 for c in sel)}",
        "// min/max ops), pruned Batcher on 32 wires (6 -inf + 6 +inf pads folded). Verified",
        "// exhaustively with the 0-1 principle over all 2^20 binary inputs.",
        f"#define SV_SEL20_NCMP {len(sel)}",
        "static constexpr unsigned char SV_SEL20_OUT[6] = {" + ", ".join(map(str, sel_out)) + "};",
        "static constexpr unsigned char SV_SEL20_NET[SV_SEL20_NCMP][3] = {",
    ]
    for a, b, u in sel:
        lines.append(f"  {{{a}, {b}, {u}}},")
    lines.append("};")
    lines += [
        "",
        f"// Ranks 7..12 (sorted) of 20 values v[i*5+j] whose 5 columns (i = 0..3) arrive",
        f"// sorted: {len(sels)} comparators ({sels_ops} min/max ops), Batcher on 32 wires",
        "// (columns on its first five 4-wire blocks) greedily pruned; verified over every",
        "// sorted-column 0-1 input (0-1 principle restricted to sorted columns).",
        f"#define SV_SEL20S_NCMP {len(sels)}",
        "static constexpr unsigned char SV_SEL20S_OUT[6] = {" + ", ".join(map(str, sels_out)) + "};",
        "static constexpr unsigned char SV_SEL20S_NET[SV_SEL20S_NCMP][3] = {",
    ]
    for a, b, u in sels:
        lines.append(f"  {{{a}, {b}, {u}}},")
    lines.append("};")
    lines += [
        "",
        "// Horizontal pair form (two adjacent windows share 4 sorted columns): sorted ranks 3..12",
        f"// of the 16 common values v[c*4+i] (column c, rank i): {len(selh)} comparators ({selh_ops} ops),",
        "// Batcher on 16 wires greedily pruned, verified over every sorted-column 0-1 input.",
        f"#define SV_SEL16H_NCMP {len(selh)}",
        "static constexpr unsigned char SV_SEL16H_OUT[10] = {" + ", ".join(map(str, selh_out)) + "};",
        "static constexpr unsigned char SV_SEL16H_NET[SV_SEL16H_NCMP][3] = {",
    ]
    for a, b, u in selh:
        lines.append(f"  {{{a}, {b}, {u}}},")
    lines.append("};")
    lines += [
        "",
        "// Per window: sorted ranks 4..9 of (SEL16H's 10 on wires 0..9 + the window's own sorted",
        f"// column on wires 10..13): {len(mrg)} comparators ({mrg_ops} ops), verified over every sorted",
        "// 0-1 input pair; the window's median is then min(C5, min_i max(C_i, U_(4-i))) as for SEL20S.",
        f"#define SV_MRG14_NCMP {len(mrg)}",
        "static constexpr unsigned char SV_MRG14_OUT[6] = {" + ", ".join(map(str, mrg_out)) + "};",
        "static constexpr unsigned char SV_MRG14_NET[SV_MRG14_NCMP][3] = {",
    ]
    for a, b, u in mrg:
        lines.append(f"  {{{a}, {b}, {u}}},")
    lines.append("};")
    lines += ["", "// optimal 5-comparator sort of 4 values",
              "static constexpr unsigned char SV_SORT4_NET[5][2] = {" +
              ", ".join(f"{{{a}, {b}}}" for a, b in SORT4) + "};"]
    lines += ["", "// optimal 9-comparator sort of 5 values",
              "static constexpr unsigned char SV_SORT5_NET[9][2] = {" +
              ", ".join(f"{{{a}, {b}}}" for a, b in SORT5) + "};"]
    with open(os.path.join(here, "sv_median_net.h"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"{len(net)} comparators, output wire {out_slot}; SEL20 {len(sel)} comparators; "
          f"SEL20S {len(sels)} comparators ({sels_ops} ops); SEL16H {len(selh)} ({selh_ops} ops); "
          f"MRG14 {len(mrg)} ({mrg_ops} ops)")


if __name__ == "__main__":
    main()
