"""Dev tool: ablated copies of the step (results WRONG; timing only) for the rollout launch,
built into mobile-env-gan_amd/lib/libmev_ab_<name>.so; time them with
  VARIANTS="ab_base ab_no_draw ..." MODES=rollout bash tools/gpu_variants.sh"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mobile-env-gan_amd", "csrc", "mev_step.hip")
OUT = os.path.join(ROOT, "mobile-env-gan_amd", "lib")

EDITS = {
    "base": [],
    "no_draw": [("  if (mneed_w) {", "  if (false) {")],
    "no_move": [("  if (active) move_ue(pos, wp, kp);\n\n  // ---- 2.", "\n  // ---- 2.")],
    "no_assoc": [("      if (active && nib != 15u) {",
                  "      if (active && nib != 15u) { srv = (int)nib; full = 1e7 + cell; }\n"
                  "      if (false) {")],
    "no_hist": [("  if (KPS(hist_lds)) {", "  n = srv >= 0 ? 1 + (srv & 3) : 0;\n  if (false) {"),
                ("  } else {\n    // lanes of the segment with the same index",
                 "  } else if (false) {\n    // lanes of the segment with the same index")],
    "no_rate": [("    cents = LDSA ? share_cents_r(full,", "    cents_f = (float)full * n; cents = LDSA ? (double)(long)(full * n) + 0 * share_cents_r(full,")],
    "no_util": [("utility_f32r<SCN>(cents_f, rate_f, kp);", "(double)(rate_f * 0.001f);")],
    # the trajectory stores still issued, with every lane's offset out of range (dropped by
    # the buffer range check): compute with no write traffic
    "oob_small": [("p.lead ? 4u * (uint32_t)p.e : nrew", "nrew + 0 * p.e"),
                  ("p.lead ? (uint32_t)p.e : ndone", "ndone + 0 * p.e")],
    "oob_obs": [("(p.valid ? 16u * p.ui : nobs) + row * robs", "nobs + 0 * p.ui + row * robs")],
    "oob_all": [("p.lead ? 4u * (uint32_t)p.e : nrew", "nrew + 0 * p.e"),
                ("p.lead ? (uint32_t)p.e : ndone", "ndone + 0 * p.e"),
                ("(p.valid ? 16u * p.ui : nobs) + row * robs", "nobs + 0 * p.ui + row * robs"),
                ("p.valid ? 4u * p.ui : nsrv, row * rsrv", "nsrv + 0 * p.ui, row * rsrv")],
    "no_reward": [("  const int isum_u = ISUM ? seg_isum_rows<PC>(active ? (int)((float)util * 0x1p25f) : 0) : 0;",
                   "  const int isum_u = ISUM ? (int)((float)util * 0x1p25f) : 0;")],
}


def build(name, edits):
    s = open(SRC).read()
    for a, b in edits:
        if a not in s:
            raise SystemExit(f"{name}: pattern not found: {a[:70]}")
        s = s.replace(a, b, 1)
    tmp = f"/tmp/ablate_{name}.hip"
    open(tmp, "w").write(s)
    return subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                             "-ffp-contract=off", "-fPIC", "-shared", "-mllvm",
                             "-amdgpu-sched-strategy=max-ilp", f"-I{ROOT}/include", "-o",
                             os.path.join(OUT, f"libmev_ab_{name}.so"), tmp],
                            stderr=subprocess.DEVNULL)


if __name__ == "__main__":
    names = sys.argv[1:] or list(EDITS)
    procs = [build(n, EDITS[n]) for n in names]
    rc = [p.wait() for p in procs]
    print(dict(zip(names, rc)))
