"""Static check of the gfx950 buffer-store data hazard in libmev's device assembly.

A MUBUF store of more than 8 bytes (buffer_store_dwordx3 / x4) needs a wait state before a
VALU instruction may overwrite its data registers. LLVM inserts it only when the store's
scalar offset is NOT a register (GCNHazardRecognizer::createsVALUHazard); with an SGPR soffset
it assumes no hazard -- and on gfx950 the overwrite then corrupted obs rows (round 1: other
values in a few rows, ~1 run in 4 at 40,000 envs). The kernels therefore pass the constant 0
as soffset for every wide buffer store (mev_step.hip, flush_pending). This check fails if any
wide buffer store in the generated assembly takes an SGPR soffset.

python tools/check_store_hazard.py [file.s]   (default: builds `make asm` and checks it)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mobile-env-gan_amd", "csrc")
ASM = os.path.join(ROOT, "mobile-env-gan_amd", "lib", "mev_step-gfx950.s")

_WIDE = re.compile(r"^\s*(buffer_store_dwordx[34]|buffer_store_b(?:96|128))\s+(.*)$")
_SGPR = re.compile(r"^(s\d+|s\[\d+:\d+\]|ttmp\d+|m0|vcc(_lo|_hi)?|exec(_lo|_hi)?)$")


def violations(asm_text: str):
    """[(line number, text, kernel)] of wide buffer stores whose soffset is a register."""
    out = []
    kernel = None
    for i, line in enumerate(asm_text.split("\n"), 1):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            kernel = m.group(1)
        m = _WIDE.match(line)
        if not m:
            continue
        ops = [o.strip() for o in m.group(2).split(",")]
        # vdata, vaddr (or "off"), srsrc, soffset [modifiers...]
        if len(ops) < 4:
            out.append((i, line.strip(), kernel))
            continue
        soff = ops[3].split()[0]
        if _SGPR.match(soff):
            out.append((i, line.strip(), kernel))
    return out


def wide_store_count(asm_text: str) -> int:
    return sum(1 for l in asm_text.split("\n") if _WIDE.match(l))


def build_asm() -> str:
    subprocess.run(["make", "-C", CSRC, "asm"], check=True, stdout=subprocess.DEVNULL)
    return ASM


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else build_asm()
    text = open(path).read()
    bad = violations(text)
    print(f"{wide_store_count(text)} wide buffer stores, {len(bad)} with a register soffset")
    for i, l, k in bad:
        print(f"  line {i} ({k}): {l}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
