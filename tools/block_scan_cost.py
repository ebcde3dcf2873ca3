"""Dev tool: us per step of the block kernel (U = 1024 UEs, per-env layouts, 1,024 envs,
velocity 10) for several station counts -- the share of the station scan in the step.
usage: python tools/block_scan_cost.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
from mobile_env.core.engine import EngineParams, StepEngine  # noqa: E402

E, U, S = 1024, 1024, 40
for B in (2, 16, 64, 128, 256):
    rng = np.random.default_rng(B)
    bs = rng.integers(0, 200, size=(E, B, 2)).astype(np.int32)
    eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B, velocity=10.0), bs,
                     1000 + np.arange(E), device="cuda")
    eng.reset()
    tr = eng.trajectory(S)
    for _ in range(5):
        eng.rollout(S, tr)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        eng.rollout(S, tr)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"B": B, "us_per_step": a.elapsed_time(b) * 1e3 / (10 * S)}), flush=True)
    eng.close()
    del tr
