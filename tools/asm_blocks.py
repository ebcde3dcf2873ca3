"""Dev tool: per-basic-block instruction counts of one kernel in the device assembly
(make asm -> mobile-env-gan_amd/lib/mev_step-gfx950.s), to compare instruction streams of
variants without a GPU.
usage: python tools/asm_blocks.py SYMBOL_SUBSTRING [--loop]
  --loop: only the blocks of the kernel's largest loop (the first back-edge spanning the most
  lines), which for the rollout kernels is the step loop.
Columns: V = VALU, S = SALU (branches listed separately), D = LDS, M = global / buffer."""
import os
import re
import sys

ASM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd", "lib",
                   "mev_step-gfx950.s")


def kernel_range(lines, sub):
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", ln) and sub in ln.split(":")[0]:
            start = i
        elif start is not None and "s_endpgm" in ln:
            return start, i + 1
    raise SystemExit(f"no kernel matching {sub}")


def main():
    sub = sys.argv[1]
    lines = open(ASM).read().split("\n")
    s, e = kernel_range(lines, sub)
    labels = {}
    for i in range(s, e):
        m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
        if m:
            labels[m.group(1)] = i
    if "--loop" in sys.argv:
        best = None
        for i in range(s, e):
            m = re.search(r"(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)", lines[i])
            if m and m.group(2) in labels and labels[m.group(2)] < i:
                span = (labels[m.group(2)], i + 1)
                if best is None or span[1] - span[0] > best[1] - best[0]:
                    best = span
        s, e = best
    order, cnt, blk = [], {}, None
    for i in range(s, e):
        ln = lines[i].strip()
        m = re.match(r"^(\.LBB\d+_\d+):", ln) or re.match(r"^; (%bb\.\d+):", ln)
        if m:
            blk = (m.group(1), i + 1)
            order.append(blk)
            cnt[blk] = [0, 0, 0, 0, []]
            continue
        if blk is None or not ln or ln.startswith((";", ".")):
            continue
        op = ln.split()[0]
        c = cnt[blk]
        if op.startswith("v_"):
            c[0] += 1
        elif op.startswith("s_"):
            if "branch" in op:
                c[4].append(ln.replace("s_cbranch_", "").replace("s_branch", "br"))
            elif op not in ("s_nop", "s_waitcnt"):
                c[1] += 1
        elif op.startswith("ds_"):
            c[2] += 1
        elif op.startswith(("global_", "buffer_")):
            c[3] += 1
    tot = [0, 0]
    for b in order:
        c = cnt[b]
        tot[0] += c[0]
        tot[1] += c[1]
        print(f"{b[0]:14s} L{b[1]:7d} V{c[0]:4d} S{c[1]:3d} D{c[2]:2d} M{c[3]:2d}  " + " | ".join(c[4]))
    print("total V", tot[0], "S", tot[1])


if __name__ == "__main__":
    main()
