"""Scratch timing of the step kernel (development only; bench.py is the contract)."""
import sys
import time

import torch

sys.path.insert(0, "mobile-env-gan_amd")
sys.path.insert(0, ".")
import json  # noqa: E402

from mobile_env.core.engine import EngineParams, StepEngine  # noqa: E402

lay = json.load(open("mobile-env-gan_amd/mobile_env/scenarios/layouts.json"))
for name, E in (("large", 65536), ("medium", 4096), ("small", 65536), ("large", 262144)):
    L = lay[name]
    p = EngineParams(num_envs=E, num_ues=L["num_ues"], num_bs=len(L["bs"]))
    eng = StepEngine(p, L["bs"], 1000, device="cuda")
    eng.step(25)
    torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    eng.step(K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    U = L["num_ues"]
    bpe = 54 * U + 61
    sps = E * K / dt
    print(f"{name} E={E}: {dt / K * 1e6:.1f} us/step  {sps / 1e6:.2f} M env-steps/s  "
          f"roofline {sps * bpe / 8e12:.3f}", flush=True)
    eng.close()
