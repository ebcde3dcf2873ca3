#!/usr/bin/env python3
"""Dev tool: one kernel's device assembly out of `make asm` output, with its VGPR / SGPR counts.

python tools/kasm.py <mangled-name-substring> [out.s]   (default out: /tmp/kernel.s)"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(ROOT, "mobile-env-gan_amd", "lib", "mev_step-gfx950.s")


def main():
    want, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "/tmp/kernel.s")
    s = open(ASM).read()
    lines = s.split("\n")
    names = [m.group(1) for m in (re.match(r"^(_Z\S+):", l) for l in lines) if m and want in m.group(1)]
    if len(names) != 1:
        sys.exit(f"{len(names)} kernels match {want!r}: {names[:8]}")
    name = names[0]
    st = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    open(out, "w").write("\n".join(lines[st:en + 1]))
    i = s.find(".name:           " + name + "\n")
    j0 = s.rfind("  - .agpr_count", 0, i) if i >= 0 else -1
    j1 = s.find("  - .agpr_count", i) if i >= 0 else -1
    meta = s[j0:(j1 if j1 > 0 else len(s))] if i >= 0 else ""
    vg = re.search(r"\.vgpr_count:\s+(\d+)", meta)
    sg = re.search(r"\.sgpr_count:\s+(\d+)", meta)
    body = lines[st:en + 1]
    nv = sum(1 for l in body if l.strip().startswith("v_"))
    ns = sum(1 for l in body if l.strip().startswith("s_"))
    print(f"{name}\n  lines {len(body)}  static VALU {nv}  SALU {ns}  "
          f"vgpr {vg.group(1) if vg else '?'}  sgpr {sg.group(1) if sg else '?'}  -> {out}")


if __name__ == "__main__":
    main()
