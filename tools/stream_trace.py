#!/usr/bin/env python3
"""Per-wave timing of k_match_stream launches (SV_STREAM_TRACE=<file> diagnostic).

Usage: python tools/stream_trace.py <file>   (the LAST launch in the file is analysed)
Clocks are s_memrealtime ticks (100 MHz)."""
import sys

import numpy as np


def main():
    raw = np.fromfile(sys.argv[1], np.uint64)
    i, launches = 0, []
    while i + 2 <= raw.size:
        waves, total = int(raw[i]), int(raw[i + 1])
        rec = raw[i + 2:i + 2 + 4 * waves].reshape(waves, 4)
        launches.append((waves, total, rec))
        i += 2 + 4 * waves
    waves, total, rec = launches[-1]
    t0 = rec[:, 0].astype(np.int64)
    t1 = rec[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0   # us
    d = e - s
    hw = rec[:, 2].astype(np.int64)
    xcc = rec[:, 3].astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    print(f"launches {len(launches)}, waves {waves}, bodies {total}")
    print(f"start spread {s.max():.1f} us; end min/median/max {e.min():.1f} / {np.median(e):.1f} / {e.max():.1f} us")
    print(f"duration min/median/max {d.min():.1f} / {np.median(d):.1f} / {d.max():.1f} us")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  XCC {x}: waves {m.sum():4d}  duration mean {d[m].mean():.1f}  end max {e[m].max():.1f}")
    key = xcc * 1000 + se * 100 + cu
    per_cu = {k: (key == k).sum() for k in np.unique(key)}
    counts = np.bincount(list(per_cu.values()))
    print("waves per CU histogram:", {i: int(c) for i, c in enumerate(counts) if c})
    slow = np.argsort(d)[-5:]
    for w in slow:
        print(f"  slow wave {w}: xcc {xcc[w]} se {se[w]} cu {cu[w]} simd {simd[w]} start {s[w]:.1f} dur {d[w]:.1f}")


if __name__ == "__main__":
    main()
