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

if os.environ.get("SPIN"):  # host wait policy: spin (hipDeviceScheduleSpin), set before any
    import ctypes as _C       # HIP call creates the device context
    assert _C.CDLL("libamdhip64.so").hipSetDeviceFlags(_C.c_uint(int(os.environ["SPIN"]))) == 0
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

E = int(os.environ.get("E", 65536))
WL = os.environ.get("WL", "mobile-large-central-v0")
LENS = [int(a) for a in sys.argv[1:]] or [20, 40, 100, 200]


class HipEvent:
    """A HIP event with explicit creation flags (hipEventCreateWithFlags), e.g. timing-only
    hipEventDisableSystemFence events (no system-scope cache writeback when recorded)."""
    _hip = None

    def __init__(self, flags):
        import ctypes as C
        if HipEvent._hip is None:
            HipEvent._hip = C.CDLL("libamdhip64.so")
        self.C = C
        self.ev = C.c_void_p()
        assert HipEvent._hip.hipEventCreateWithFlags(C.byref(self.ev), C.c_uint(flags)) == 0

    def record(self, stream):
        assert HipEvent._hip.hipEventRecord(self.ev, self.C.c_void_p(stream.cuda_stream)) == 0

    def elapsed_time(self, other):
        ms = self.C.c_float()
        assert HipEvent._hip.hipEventElapsedTime(self.C.byref(ms), self.ev, other.ev) == 0
        return ms.value
over = {k: int(v) for k, v in (kv.split("=") for kv in os.environ.get("MEV_ENGINE", "").split(",")
                               if kv)}
EVMODE = os.environ.get("EVMODE", "torch")  # torch | nofence (hipEventDisableSystemFence) | none
env = mobile_env.make(WL, num_envs=E, device="cuda:0", seed=1000, **over)
env.reset()
eng = env.engine
traj = eng.trajectory(int(os.environ.get("TRAJ_ROWS", max(LENS))))  # (buffer size: placement)
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
    if EVMODE == "inlaunch":  # the launch records its own pair (mev_rollout_timed)
        pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(30)]
        for a, b in pairs:
            a.record(stream)
            b.record(stream)
        gos = [eng.launcher(n, traj, events=(a.cuda_event, b.cuda_event)) for a, b in pairs]
        torch.cuda.synchronize()
        for (a, b), g in zip(pairs, gos):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g()
            torch.cuda.synchronize()
            iso_wall.append((time.perf_counter() - t0) * 1e3)
            iso_ev.append(a.elapsed_time(b))
    for _ in range(30 if EVMODE != "inlaunch" else 0):
        if EVMODE == "nofence":
            a, b = HipEvent(0x20000000), HipEvent(0x20000000)
        else:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if EVMODE != "none":
            a.record(stream)
        go()
        if EVMODE != "none":
            b.record(stream)
        torch.cuda.synchronize()
        iso_wall.append((time.perf_counter() - t0) * 1e3)
        iso_ev.append(a.elapsed_time(b) if EVMODE != "none" else 0.0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(4, 4000 // n)
    a.record(stream)
    for _ in range(reps):
        go()
    b.record(stream)
    torch.cuda.synchronize()
    b2b = a.elapsed_time(b) / reps
    print(json.dumps({"n": n, "engine": over, "evmode": EVMODE, "spin": os.environ.get("SPIN"), "traj_rows": traj.obs.shape[0], "iso_event_ms_median": statistics.median(iso_ev),
                      "iso_event_ms_min": min(iso_ev),
                      "iso_wall_ms_median": statistics.median(iso_wall),
                      "b2b_ms": b2b, "b2b_us_per_step": b2b * 1e3 / n,
                      "iso_us_per_step": statistics.median(iso_ev) * 1e3 / n,
                      "env_steps_per_s_iso_wall": E * n / (statistics.median(iso_wall) * 1e-3)}),
          flush=True)
if os.environ.get("SINGLE"):  # one-step launches (make().step(), mev_step(1)), back to back
    go1 = eng.launcher(1)
    for _ in range(50):
        go1()
    torch.cuda.synchronize()
    res = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(100):
            go1()
        b.record(stream)
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 10.0)  # us per launch
    print(json.dumps({"n": 1, "engine": over, "single_us_median": statistics.median(res),
                      "single_us_min": min(res)}), flush=True)
env.close()
