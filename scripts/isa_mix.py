#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc `-S` gfx950 assembly file.

    python scripts/isa_mix.py stencil.s <symbol-substring> [--loop | --loops]

Prints VGPR/SGPR counts and the opcode histogram of the whole kernel, or with
--loop of its largest basic-block loop (the label with the most instructions
before the branch that jumps back to it) -- the stream kernels' row loop.
--loops lists every loop (back edge) with its VALU, f64-add, DPP, 64-bit move,
barrier, load and store counts: the pipeline kernels' two stages each have one
steady row loop (the one with the global loads, and the one with the buffer
stores) besides their warm-up loops.
Used to count VALU issue slots per level-row (docs/PERF.md).
"""
import collections
import re
import sys


def kernel_lines(path, needle):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and l.endswith(":") and needle in l and not l.startswith(".") and "@" not in l.split(":")[0]:
            start = i
        elif start is None and re.match(r"^_Z\S*:", l) and needle in l:
            start = i
        elif start is not None and l.strip().startswith("s_endpgm"):
            return lines[start:i + 1], lines[i:i + 400]
    raise SystemExit(f"kernel {needle!r} not found")


def ops(body):
    out = []
    for l in body:
        t = l.split(";")[0].strip()
        if not t or t.startswith((".", "//")) or t.endswith(":"):
            continue
        out.append(t.split()[0])
    return out


def largest_loop(body):
    labels = {}
    best = (0, None, None)
    for i, l in enumerate(body):
        t = l.split(";")[0].strip()
        if t.endswith(":") and t.startswith(".LBB"):
            labels[t[:-1]] = i
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)", t) or re.match(r"s_branch\s+(\.LBB\S+)", t)
        if m and m.group(1) in labels:
            j = labels[m.group(1)]
            n = len(ops(body[j:i + 1]))
            if n > best[0]:
                best = (n, j, i)
    return best


def all_loops(body):
    labels, out = {}, []
    for i, l in enumerate(body):
        t = l.split(";")[0].strip()
        if t.endswith(":") and t.startswith(".LBB"):
            labels[t[:-1]] = i
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)", t) or re.match(r"s_branch\s+(\.LBB\S+)", t)
        if m and m.group(1) in labels:
            j = labels[m.group(1)]
            c = collections.Counter(ops(body[j:i + 1]))
            out.append((m.group(1), j, i, sum(c.values()), sum(v for k, v in c.items() if k.startswith("v_")),
                        c["v_add_f64"], c["v_pk_add_f32"], c["v_mov_b32_dpp"], c["v_mov_b64_e32"] + c["v_mov_b64"],
                        c["s_barrier"], c["global_load_dwordx4"], c["ds_write_b128"], c["ds_read_b128"],
                        c["buffer_store_dwordx4"]))
    return out


def main():
    path, needle = sys.argv[1], sys.argv[2]
    body, meta = kernel_lines(path, needle)
    for l in meta:
        if re.search(r"\.(vgpr_count|sgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count):", l):
            print(l.strip())
        if "NumVgprs:" in l or "ScratchSize:" in l or "Occupancy:" in l:
            print(l.strip())
    sel = body
    if "--loops" in sys.argv:
        print("label start end ops valu add_f64 pk_add_f32 dpp mov64 barrier gload ds_write ds_read buf_store")
        for row in sorted(all_loops(body), key=lambda r: r[1]):
            print(*row)
        return
    if "--loop" in sys.argv:
        n, j, i = largest_loop(body)
        print(f"largest loop: {n} instructions (lines {j}..{i})")
        sel = body[j:i + 1]
    c = collections.Counter(ops(sel))
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"v_* total {valu}")
    for k, v in c.most_common():
        print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
