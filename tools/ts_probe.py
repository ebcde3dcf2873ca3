"""Dev tool: phase timestamps of the two-group rollout kernel (k_steps_lds2) of one isolated
launch, from a -DMEV_TIMING build (tools/build_variant.sh WT ts with EXTRA=-DMEV_TIMING):
  MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so python tools/ts_probe.py [n ...]
Per event (0 start, 1 tables + first inputs landed, 2 first pair set up, then per pair j:
3+3j steps done, 4+3j state stored + next pair set up, 5+3j staged rows flushed; 31 end):
min / median / max over waves in us after the earliest wave start (s_memrealtime, 100 MHz)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402
from mobile_env.core import _native as N  # noqa: E402

E = int(os.environ.get("E", 65536))
LENS = [int(a) for a in sys.argv[1:]] or [20]
env = mobile_env.make("mobile-large-central-v0", num_envs=E, device="cuda:0", seed=1000)
env.reset()
eng = env.engine
L = N.lib()
L.mev_debug_timestamps.argtypes = [C.c_void_p]
buf = torch.zeros((4096 * 2, 32), dtype=torch.int64, device="cuda")
traj = eng.trajectory(max(LENS))
go = eng.launcher(max(LENS), traj)
for _ in range(200):
    go()
torch.cuda.synchronize()
for n in LENS:
    go = eng.launcher(n, traj)
    for _ in range(20):
        go()
    torch.cuda.synchronize()
    N.check(L.mev_debug_timestamps(C.c_void_p(buf.data_ptr())), "ts")
    res = []
    for rep in range(5):
        buf.zero_()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        go()
        b.record()
        torch.cuda.synchronize()
        ts = buf.cpu().numpy()
        used = ts[:, 0] > 0
        t = ts[used].astype(np.float64)
        t0 = t[:, 0].min()
        rel = (t - t0) / 100.0  # us
        ev = {}
        for k in range(32):
            col = t[:, k]
            ok = col > 0
            if ok.any():
                r = rel[ok, k]
                ev[k] = [round(float(r.min()), 2), round(float(np.median(r)), 2), round(float(r.max()), 2)]
        res.append({"event_ms": a.elapsed_time(b), "waves": int(used.sum()), "ts_us": ev})
    print(json.dumps({"n": n, "reps": res}), flush=True)
    N.check(L.mev_debug_timestamps(C.c_void_p(None)), "ts")
env.close()
