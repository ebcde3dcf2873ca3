"""Dev tool: build ablated copies of the step kernel (results are WRONG; timing only) into
mobile-env-gan_amd/lib/ablate_<name>.so, to price each phase of the packed step."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mobile-env-gan_amd", "csrc", "mev_step.hip")
OUT = os.path.join(ROOT, "mobile-env-gan_amd", "lib")

EDITS = {
    "no_draw": [("  if (mneed_w) {", "  if (false) {")],
    "no_assoc": [("  } else if (active) {\n    const int nb = kp.B;",
                  "  } else if (active) {\n    best = (unsigned)(pos.x & 1023) << kKeyBits;\n    const int nb = 0;")],
    "no_pairwise": [("  const double sum_u = seg_sum(util, active, U, u);",
                     "  const double sum_u = util;")],
    "no_move": [("  if (active) move_ue(pos, wp, kp);\n\n  // ---- 2.", "\n  // ---- 2.")],
    "no_rate": [("  if (srv >= 0) cents = share_cents(tb.rate_full[d2s], n, tb.c100);",
                 "  if (srv >= 0) cents = (double)(d2s * n);")],
    "no_util": [("  const double util = active ? utility_of(rate, cents, kp, tb.util) : 0.0;\n\n  // ---- 5.",
                 "  const double util = active ? cents * 1e-3 : 0.0;\n\n  // ---- 5.")],
}


def build(name, edits):
    s = open(SRC).read()
    for a, b in edits:
        if a not in s:
            raise SystemExit(f"{name}: pattern not found: {a[:60]}")
        s = s.replace(a, b)
    tmp = f"/tmp/ablate_{name}.hip"
    open(tmp, "w").write(s)
    so = os.path.join(OUT, f"ablate_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", "-fPIC", "-shared", f"-I{ROOT}/include",
                    f"-I{os.path.dirname(SRC)}", "-o", so, tmp], check=True)
    return so


if __name__ == "__main__":
    names = sys.argv[1:] or list(EDITS)
    allx = []
    for n in names:
        build(n, EDITS[n])
        allx += EDITS[n]
    build("all", allx)
    print("built", names + ["all"])
