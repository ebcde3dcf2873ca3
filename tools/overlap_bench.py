"""Dev tool: does splitting the env batch over several HIP streams (independent env shards,
kernels of different shards free to overlap) beat one stream? Wall time per step."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
from mobile_env.core import _native as N  # noqa: E402
from mobile_env.core.engine import EngineParams, StepEngine  # noqa: E402
from mobile_env.scenarios.registry import LAYOUTS  # noqa: E402


def run(name, E, parts, K=400, vel=1.5):
    L = LAYOUTS[name]
    lib = N.lib()
    engs, streams, calls = [], [], []
    for i in range(parts):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            p = EngineParams(num_envs=E // parts, num_ues=L["num_ues"], num_bs=len(L["bs"]),
                             velocity=vel)
            eng = StepEngine(p, L["bs"], 1000 + i * (E // parts), device="cuda")
            eng.step(30)
        engs.append(eng)
        streams.append(s)
        calls.append((eng._ctx, C.byref(eng._st), C.byref(eng._out),
                      C.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    step = lib.mev_step
    chunk = int(os.environ.get("MEV_OB_CHUNK", "1"))

    def loop(n):
        for _ in range(n // chunk):
            for c in calls:
                step(c[0], c[1], c[2], chunk, c[3])

    loop(40)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(K)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    for e in engs:
        e.close()
    U = L["num_ues"]
    return {"scenario": name, "E": E, "parts": parts, "chunk": chunk, "us_per_step": dt * 1e6,
            "frac": E * (54 * U + 61) / dt / 8e12}


if __name__ == "__main__":
    for parts in (1, 2, 4, 1, 2, 4, 8):
        print(json.dumps(run("large", 65536, parts)), flush=True)
    os.environ["MEV_OB_CHUNK"] = "10"
    for parts in (1, 2, 4):
        print(json.dumps(run("large", 65536, parts)), flush=True)
