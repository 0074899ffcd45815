#!/usr/bin/env python3
"""Instruction counts of one kernel in a hipcc -S listing (ISA inspection aid).

Usage: python tools/isa_count.py <file.s> <symbol-substring> [op ...]
"""
import re
import sys

OPS = ["v_sad_u8", "v_sad_hi_u8", "v_mad_i32_i24", "v_sub_u32", "v_add_u32", "v_min3_u32",
       "v_min_u32", "ds_read_b128", "ds_read_b64", "ds_write_b128", "v_mov_b32", "v_cndmask_b32",
       "s_waitcnt", "s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccnz", "s_cbranch_execz"]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    ops = sys.argv[3:] or OPS
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and sym in l)
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^_Z\w*:", lines[i])), len(lines))
    body = "\n".join(lines[start:end])
    print(lines[start].split(":")[0])
    for op in ops:
        n = len(re.findall(r"\b" + op + r"\b", body))
        print(f"  {op:18s} {n}")
    meta = "\n".join(lines)
    name = lines[start].split(":")[0]
    m = re.search(r"\.name:\s+" + re.escape(name) + r"[\s\S]*?\.vgpr_count:\s+(\d+)", meta)
    if m:
        print("  vgpr_count", m.group(1))


if __name__ == "__main__":
    main()
