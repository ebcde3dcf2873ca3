"""Dev tool: the host side of the driver's timed region (bench.py --steps 20: ONE isolated
20-step rollout launch at 65,536 mobile-large envs) under a HIP host wait policy set before the
device is initialised (hipSetDeviceFlags): auto (HIP's default), spin, yield, block.
Prints per rep the median wall time of `sync; t0; launch; sync; t1` over 40 launches, of the same
without the launch (the synchronize alone), and the launch's event time.
usage: python tools/host_wait_probe.py MODE [reps]"""
import ctypes
import json
import os
import statistics
import sys
import time

mode = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if mode != "auto":
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(ctypes.c_int(0)) == 0
    flag = {"spin": 1, "yield": 2, "block": 4}[mode]
    assert hip.hipSetDeviceFlags(ctypes.c_uint(flag)) == 0

import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
env = mobile_env.make("mobile-large-central-v0", num_envs=65536, device=dev, seed=1000)
env.reset()
eng = env.engine
traj = eng.trajectory(200)
big = eng.launcher(200, traj)
go = eng.launcher(20, traj)
stream = torch.cuda.current_stream(dev)
t = time.perf_counter()
while time.perf_counter() - t < 2.0:
    for _ in range(8):
        big()
    torch.cuda.synchronize(dev)
for r in range(reps):
    walls, empty, evs = [], [], []
    for _ in range(40):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        go()
        torch.cuda.synchronize(dev)
        walls.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        empty.append((time.perf_counter() - t0) * 1e6)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        a.record(stream)
        go()
        b.record(stream)
        torch.cuda.synchronize(dev)
        evs.append(a.elapsed_time(b) * 1e3)
    print(json.dumps({"mode": mode, "rep": r, "wall_us": round(statistics.median(walls), 1),
                      "wall_min_us": round(min(walls), 1),
                      "sync_only_us": round(statistics.median(empty), 1),
                      "event_us": round(statistics.median(evs), 1)}), flush=True)
env.close()
