"""Dev tool: fixed cost of a rollout launch vs its length, in the bench's shape (65,536
mobile-large envs, trajectory rows), measured the two ways that matter:
  * isolated: synchronize, then ONE launch between a HIP event pair and a wall-clock pair, then
    synchronize -- what bench.py's driver run (--steps 20: one 20-step launch) times;
  * back-to-back: 20 launches between one event pair (the launch tail overlaps the next ramp).
usage: python tools/launch_len.py [n ...]  (env MEV_ENGINE="key=v,key=v" for engine overrides)
Prints one JSON line per launch length."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

E = int(os.environ.get("E", 65536))
WL = os.environ.get("WL", "mobile-large-central-v0")
LENS = [int(a) for a in sys.argv[1:]] or [20, 40, 100, 200]
over = {k: int(v) for k, v in (kv.split("=") for kv in os.environ.get("MEV_ENGINE", "").split(",")
                               if kv)}
env = mobile_env.make(WL, num_envs=E, device="cuda:0", seed=1000, **over)
env.reset()
eng = env.engine
traj = eng.trajectory(max(LENS))
stream = torch.cuda.current_stream()
t_w = time.perf_counter()
go = eng.launcher(max(LENS), traj)
while time.perf_counter() - t_w < 2.0:  # steady clock
    for _ in range(8):
        go()
    torch.cuda.synchronize()
for n in LENS:
    go = eng.launcher(n, traj)
    for _ in range(5):
        go()
    torch.cuda.synchronize()
    iso_ev, iso_wall = [], []
    for _ in range(30):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(stream)
        go()
        b.record(stream)
        torch.cuda.synchronize()
        iso_wall.append((time.perf_counter() - t0) * 1e3)
        iso_ev.append(a.elapsed_time(b))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(4, 4000 // n)
    a.record(stream)
    for _ in range(reps):
        go()
    b.record(stream)
    torch.cuda.synchronize()
    b2b = a.elapsed_time(b) / reps
    print(json.dumps({"n": n, "engine": over, "iso_event_ms_median": statistics.median(iso_ev),
                      "iso_event_ms_min": min(iso_ev),
                      "iso_wall_ms_median": statistics.median(iso_wall),
                      "b2b_ms": b2b, "b2b_us_per_step": b2b * 1e3 / n,
                      "iso_us_per_step": statistics.median(iso_ev) * 1e3 / n,
                      "env_steps_per_s_iso_wall": E * n / (statistics.median(iso_wall) * 1e-3)}),
          flush=True)
env.close()
