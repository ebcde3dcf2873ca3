"""Time the step kernel of one libmev build (dev tool): MEV_LIB=path python tools/variant_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
from mobile_env.core.engine import EngineParams, StepEngine  # noqa: E402
from mobile_env.scenarios.registry import LAYOUTS  # noqa: E402


def run(name, E, steps=200, vel=None):
    L = LAYOUTS[name]
    p = EngineParams(num_envs=E, num_ues=L["num_ues"], num_bs=len(L["bs"]),
                     velocity=vel if vel is not None else 1.5,
                     stream_split=int(os.environ.get("MEV_VB_SPLIT", "0")))
    eng = StepEngine(p, L["bs"], 1000, device="cuda")
    eng.step(int(os.environ.get("MEV_VB_WARMUP", "3000")))  # to steady GPU clocks
    torch.cuda.synchronize()
    reps = 20  # back-to-back launches from the C loop per timed chunk
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps // reps)]
    for a, b in ev:
        a.record()
        eng.step(reps)
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 / reps for a, b in ev)
    eng.close()
    U = L["num_ues"]
    return {"scenario": name, "E": E, "vel": p.velocity, "us_mean": sum(t) / len(t),
            "us_med": t[len(t) // 2], "frac": E * (54 * U + 61) / (t[len(t) // 2] * 1e-6) / 8e12}


if __name__ == "__main__":
    tag = os.environ.get("TAG", os.environ.get("MEV_LIB", "default")) + \
        " split=" + os.environ.get("MEV_VB_SPLIT", "0")
    cases = (("large", 65536), ("large", 65536, 200, 10.0), ("medium", 4096), ("small", 65536))
    for args in cases[:int(os.environ.get("MEV_VB_CASES", len(cases)))]:
        r = run(*args)
        r["tag"] = tag
        print(json.dumps(r), flush=True)
