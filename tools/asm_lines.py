"""Dev tool: static instruction mix of one kernel, attributed to source lines.

python tools/asm_lines.py [kernel-substring]   (default: k_step_packedILb0)
Compiles mev_step.hip to device assembly with line tables and counts VALU / SALU / memory
instructions per source line (static counts: a line inside a loop counts once)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get('MEV_SRC', os.path.join(ROOT, 'mobile-env-gan_amd', 'csrc', 'mev_step.hip'))
OUT = "/tmp/mev_step_lines.s"


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "k_step_packedILb0"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", "-gline-tables-only", "--cuda-device-only", "-S",
                    f"-I{ROOT}/include", "-o", OUT, SRC], check=True)
    text = open(OUT).read().split("\n")
    files = {}
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*%s\S*:" % want, l))
    src = open(SRC).read().split("\n")
    per = collections.defaultdict(collections.Counter)
    cur = None
    tot = collections.Counter()
    for l in text[start:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip()
        m = re.match(r"\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", t)
        if m:
            files[m.group(1)] = m.group(2)
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cat = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch", "s_branch")) else
               "smem" if op.startswith(("s_load", "s_buffer")) else
               "br" if op.startswith(("s_cbranch", "s_branch")) else
               "wait" if op.startswith("s_waitcnt") else op.split("_")[0])
        per[cur][cat] += 1
        tot[cat] += 1
    for f in re.findall(r"\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", "\n".join(text)):
        files.setdefault(f[0], f[1])
    print("total", dict(tot))
    rows = sorted(per.items(), key=lambda kv: -kv[1]["valu"])
    for key, c in rows[:45]:
        if key is None:
            desc = "?"
        else:
            fname = files.get(key[0], "?")
            desc = (src[key[1] - 1].strip()[:70] if fname.endswith("mev_step.hip") else
                    os.path.basename(fname))
        print(f"{c['valu']:4d} v {c['salu']:4d} s {c['br']:3d} b  L{key[1] if key else 0:<5d} {desc}")


if __name__ == "__main__":
    main()
