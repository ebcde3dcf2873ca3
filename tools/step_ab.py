"""Dev tool: duration of the Gym step() launch (mev_step(1)) at the bench's batch, back to back
(10 groups of 20 launches between HIP event pairs, the median group) and isolated (synchronize,
one launch between an event pair; the median of 20).
usage: MEV_LIB=... [MEV_STEP_PF=0] python tools/step_ab.py [tag]   (env E, WL)
Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

E = int(os.environ.get("E", 65536))
WL = os.environ.get("WL", "mobile-large-central-v0")
env = mobile_env.make(WL, num_envs=E, device="cuda:0", seed=1000)
env.reset()
eng = env.engine
step1 = eng.launcher(1)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:  # steady clock
    for _ in range(50):
        step1()
    torch.cuda.synchronize()
grp = []
for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        step1()
    b.record()
    torch.cuda.synchronize()
    grp.append(a.elapsed_time(b) / 20)
iso = []
for _ in range(20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    step1()
    b.record()
    torch.cuda.synchronize()
    iso.append(a.elapsed_time(b))
grp.sort()
iso.sort()
print(json.dumps({"tag": sys.argv[1] if len(sys.argv) > 1 else "", "wl": WL, "envs": E,
                  "pf": os.environ.get("MEV_STEP_PF", "1"), "kind": eng.last_launch_kind,
                  "b2b_us_median": grp[len(grp) // 2] * 1e3, "b2b_us_min": grp[0] * 1e3,
                  "iso_us_median": iso[len(iso) // 2] * 1e3}))
