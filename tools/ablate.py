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
    "no_assoc": [("    const int4 r = at(const_cast<int4*>(tb.assoc), 16u * (uint32_t)(yi * kp.W + xi));",
                  "    const int4 r = make_int4(xi % 13, yi, xi, yi);")],
    "no_pairwise": [("  const double sum_u = ROWS ? seg_sum_rows<PC>(util, active) : seg_sum(util, active, U, u);",
                     "  const double sum_u = util;")],
    "no_move": [("  if (active) move_ue(pos, wp, kp);\n\n  // ---- 2.", "\n  // ---- 2.")],
    "no_match": [("    n = srv >= 0 ? h[srv] : 0;", "    n = srv >= 0 ? 1 + (srv & 3) : 0;")],
    "no_rate": [("  if (srv >= 0) cents = share_cents(full, n);",
                 "  if (srv >= 0) cents = (double)((int)full * n);")],
    "no_util": [("    util = exact_util ? utility_of(rate, cents, kp, tb.util) : utility_f32(cents, kp);",
                 "    util = cents * 1e-3;")],
}
COMPUTE_ONLY = [
    ("  g.t = at(st.t, 4u * (uint32_t)ec);\n  g.s = load_ue(&at(st.ue_state, 8u * ue));",
     "  g.t = (ec * 7) % 20;\n  g.s = make_int4((ec * 13 + u * 7) % 200, (ec * 3 + u * 11) % 200, "
     "((ec * 7 + u * 13) % 70 == 0) ? -1 : (ec + u * 5) % 200, (ec * 5 + u) % 200);"),
    ("  g.pa = at(pr, 48u * (uint32_t)ec);\n  g.pb = at(pr, 48u * (uint32_t)ec + 16u);",
     "  g.pa = make_ulonglong2((uint64_t)pr + ec, 7);\n  g.pb = make_ulonglong2(2 * ec + 1, 3);"),
    ("  // ---- 6. stores ----------------------------------------------------------------------\n  if (valid) {",
     "  // ---- 6. stores ----------------------------------------------------------------------\n  if (valid && kp.E < 0) {"),
    ("  if (env_ok && leader) {\n    // np.mean;", "  if (env_ok && leader && kp.E < 0) {\n    // np.mean;"),
]


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
    build("compute_only", COMPUTE_ONLY)
    for n in names:
        build("co_" + n, COMPUTE_ONLY + EDITS[n])
    build("co_all", COMPUTE_ONLY + allx)
    print("built", names + ["all", "compute_only"])
