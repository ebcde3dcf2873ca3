"""Dev tool: host-side cost of bench.py's timed region for one isolated rollout launch (65,536
mobile-large envs, --steps 20 as the driver runs it): median wall time over repetitions of
  sync; t0; [events]; launch; [events]; sync; t1
for event modes (torch event records around the launch / the launch's own dispatch records
them / none) and synchronize forms. usage: python tools/timed_region_probe.py [n]"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
E = 65536
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
env = mobile_env.make("mobile-large-central-v0", num_envs=E, device=dev, seed=1000)
env.reset()
eng = env.engine
traj = eng.trajectory(200)
big = eng.launcher(200, traj)
t = time.perf_counter()
while time.perf_counter() - t < 2.0:
    for _ in range(8):
        big()
    torch.cuda.synchronize()
stream = torch.cuda.current_stream(dev)
plain = eng.launcher(n, traj)
syncs = {"sync()": lambda: torch.cuda.synchronize(), "sync(dev)": lambda: torch.cuda.synchronize(dev),
         "stream": lambda: stream.synchronize()}
res = {}
for rep in range(3):
    for mode in ("none", "torch", "inlaunch"):
        for sname, sync in syncs.items():
            walls, evs = [], []
            for _ in range(20):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                b.record(stream)
                go = eng.launcher(n, traj, events=(a.cuda_event, b.cuda_event)) if mode == "inlaunch" else plain
                sync()
                t0 = time.perf_counter()
                if mode == "torch":
                    a.record(stream)
                go()
                if mode == "torch":
                    b.record(stream)
                sync()
                walls.append((time.perf_counter() - t0) * 1e6)
                if mode != "none":
                    evs.append(a.elapsed_time(b) * 1e3)
            k = f"{mode}/{sname}"
            res.setdefault(k, []).append((statistics.median(walls), statistics.median(evs) if evs else 0))
for k, v in res.items():
    print(json.dumps({"mode": k, "wall_us": [round(x[0], 1) for x in v], "event_us": [round(x[1], 1) for x in v]}))
env.close()
