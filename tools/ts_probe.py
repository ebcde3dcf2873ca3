"""Dev tool: phase timestamps of the two-group rollout kernel (k_steps_lds2) of one isolated
launch, from a -DMEV_TIMING build (tools/build_variant.sh WT ts with EXTRA=-DMEV_TIMING):
  MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so python tools/ts_probe.py [n ...]
Per event (0 start, 1 tables + first inputs landed, 2 first pair set up, then per pair j:
3+3j steps done, 4+3j state stored + next pair set up, 5+3j staged rows flushed; 31 end; 25/26 the core clock counter at start/end ->
clk_mhz; 23/24 HW_ID / XCC_ID; env RAW=file.npy saves rep 1's raw words, SLEEP=s between launches, REPS):
min / median / max over waves in us after the earliest wave start (s_memrealtime, 100 MHz)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402
from mobile_env.core import _native as N  # noqa: E402

E = int(os.environ.get("E", 65536))
LENS = [int(a) for a in sys.argv[1:]] or [20]
over = {k: int(v) for k, v in (kv.split("=") for kv in os.environ.get("MEV_ENGINE", "").split(",")
                               if kv)}
env = mobile_env.make("mobile-large-central-v0", num_envs=E, device="cuda:0", seed=1000, **over)
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
    for rep in range(int(os.environ.get("REPS", 5))):
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
        dclk = (t[:, 26] - t[:, 25]) / np.maximum(t[:, 31] - t[:, 0], 1) * 100.0  # MHz
        if os.environ.get("RAW") and rep == 1:
            np.save(os.environ["RAW"], ts)
        xcc = t[:, 24].astype(np.int64) & 0xF
        by_xcd = [round(float(np.median(rel[xcc == x, 31])), 1) for x in range(8)]
        res.append({"by_xcd_end_us": by_xcd, "event_ms": a.elapsed_time(b), "waves": int(used.sum()),
                    "clk_mhz": [round(float(np.min(dclk))), round(float(np.median(dclk))),
                                round(float(np.max(dclk)))],
                    "ts_us": {k: v for k, v in ev.items() if k not in (23, 24, 25, 26)}})
        if os.environ.get("SLEEP"):
            time.sleep(float(os.environ["SLEEP"]))
    print(json.dumps({"n": n, "reps": res}), flush=True)
    N.check(L.mev_debug_timestamps(C.c_void_p(None)), "ts")
env.close()
