"""Static check of k_steps_lds2's inline-assembly prefetch loads in libmev's device assembly.

The one-pair-ahead input loads of the two-group rollout kernel are inline assembly
(mev_step.hip, pf_b32 / pf_b64: "; mev-prefetch"), which the compiler does not track: the
hardware writes their destination registers whenever the loads land, and the kernel waits for
them itself (lds2_pf_wait: an explicit s_waitcnt, then every register tied to it by an empty
asm, "; mev-prefetch-wait"). That is only sound if the compiler keeps each prefetched value in
the register the load wrote until that wait: no copy (a copy would read the register before the
data landed) and no spill. This check, per kernel with prefetch loads:
  * the registers tied at the waits are exactly the registers the loads wrote (a split live
    range -- a copy at a loop edge -- shows as a tied register that no load wrote);
  * no instruction between a prefetch load and the next wait in the code reads one of the
    loaded registers (copies, spills, any use), other than further prefetch loads;
  * no instruction between them writes one (a register reused while the load is in flight);
  * no call (s_swappc / s_call) while one is in flight, unless an s_waitcnt vmcnt(0) precedes
    it in its block, after the block's last prefetch load: the callee's save / restore of a
    register it uses would lose the data.

python tools/check_prefetch_regs.py [file.s]   (default: builds `make asm` and checks it)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mobile-env-gan_amd", "csrc")
ASM = os.path.join(ROOT, "mobile-env-gan_amd", "lib", "mev_step-gfx950.s")

_REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_KERNEL = re.compile(r"^(_Z\S+):")


def regs_of(text: str):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _split_operands(line: str):
    code = line.split(";")[0].strip()
    parts = code.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    return parts[0], [o.strip() for o in parts[1].split(",")]


def _dead_high_addend(op, ops, hit, lines, idx, horizon=4000):
    """A v_mad_u64_u32 / v_mad_i64_i32 whose only in-flight operand is the HIGH half of its
    64-bit addend, with the result's high half dead on every path from it (each path redefines
    it, as the destination of an instruction that does not read it, before any read, or ends
    the program): the low 32 bits of the result do not depend on the addend's high half, so the
    register is read for nothing (the compiler's pick for a don't-care half) -- no value
    reaches any use. Conditional branches fork the walk; a label already walked is not walked
    again (its first visit decides)."""
    if op not in ("v_mad_u64_u32", "v_mad_i64_i32") or len(ops) < 5:
        return False
    m = re.match(r"v\[(\d+):(\d+)\]$", ops[-1])
    d = re.match(r"v\[(\d+):(\d+)\]$", ops[0])
    if not m or not d or hit != {int(m.group(2))}:
        return False
    hi = int(d.group(2))
    labels = {t.split(":")[0].strip(): k for k, (_, t) in enumerate(lines)
              if re.match(r"^\.LBB\w*:", t)}
    seen = set()
    work = [idx + 1]
    steps = 0
    while work:
        k = work.pop()
        while k < len(lines):
            steps += 1
            if steps > horizon:
                return False  # (not proven within the budget)
            raw = lines[k][1]
            code = raw.split(";")[0].strip()
            k += 1
            if code.endswith(":"):
                if code[:-1] in seen:
                    break
                seen.add(code[:-1])
                continue
            if not code or code.startswith("."):
                continue
            if code.startswith("s_endpgm"):
                break
            if code.startswith("s_cbranch") or code.startswith("s_branch"):
                tgt = code.split()[1]
                if tgt not in labels:
                    return False
                if code.startswith("s_branch"):
                    k = labels[tgt]
                else:
                    work.append(labels[tgt])
                continue
            o2, ops2 = _split_operands(raw)
            if not ops2 or hi not in regs_of(",".join(ops2)):
                continue
            if hi in regs_of(",".join(ops2[1:])) or hi not in regs_of(ops2[0]):
                return False  # read (or only partly written) on this path
            break  # redefined: dead on this path
    return True


def check_kernel(name: str, lines):
    """Violations [(line, text, reason)] in one kernel's lines [(number, text)]."""
    bad = []
    loaded, tied = set(), set()
    inflight = set()  # registers of loads issued since the last wait
    vm_waited = False  # an s_waitcnt vmcnt(0) earlier in the current block
    for idx, (no, text) in enumerate(lines):
        if "; mev-prefetch-wait" in text:
            regs = regs_of(text.split("mev-prefetch-wait", 1)[1])
            tied |= regs
            inflight -= regs
            continue
        if "; mev-prefetch" in text:
            op, ops = _split_operands(text)
            dst = regs_of(ops[0]) if ops else set()
            loaded |= dst
            inflight |= dst
            vm_waited = False  # (only a vmcnt(0) wait after the last prefetch load counts)
            continue
        code = text.split(";")[0]
        if code.strip().endswith(":") or text.startswith("; %bb."):
            vm_waited = False  # (a block starts: no wait of this block seen yet)
        if "s_waitcnt" in code and "vmcnt(0)" in code:
            vm_waited = True
        if inflight and re.match(r"\s*s_(swappc|call)_b64", code) and not vm_waited:
            bad.append((no, text.strip(), "call while prefetch register(s) are in flight"))
        if not inflight:
            continue
        if not code.strip() or code.strip().startswith(".") or code.strip().endswith(":"):
            continue
        op, ops = _split_operands(text)
        if not ops:
            continue
        # operands: the first is the destination for VALU / loads / moves; stores read all
        used = regs_of(",".join(ops))
        hit = used & inflight
        if hit and _dead_high_addend(op, ops, hit, lines, idx):
            continue
        if hit:
            bad.append((no, text.strip(), f"touches in-flight prefetch register(s) v{sorted(hit)}"))
    if loaded != tied:
        bad.append((lines[0][0], name,
                    f"registers loaded {sorted(loaded - tied)} not tied at a wait / tied "
                    f"{sorted(tied - loaded)} not loaded"))
    return bad, len(loaded)


def violations(asm_text: str):
    """(violations, number of kernels with prefetch loads)."""
    kernels = []
    cur = None
    for no, line in enumerate(asm_text.split("\n"), 1):
        m = _KERNEL.match(line)
        if m:
            cur = (m.group(1), [])
            kernels.append(cur)
            continue
        if cur is not None:
            cur[1].append((no, line))
            if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
                cur = None
    bad, n = [], 0
    for name, lines in kernels:
        if not any("; mev-prefetch" in t for _, t in lines):
            continue
        n += 1
        b, _ = check_kernel(name, lines)
        bad += [(no, txt, why, name) for no, txt, why in b]
    return bad, n


def build_asm() -> str:
    subprocess.run(["make", "-C", CSRC, "asm"], check=True, stdout=subprocess.DEVNULL)
    return ASM


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else build_asm()
    bad, n = violations(open(path).read())
    for no, txt, why, name in bad:
        print(f"{path}:{no}: {why}: {txt} ({name[:60]})")
    print(f"{n} kernels with prefetch loads, {len(bad)} violations")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
