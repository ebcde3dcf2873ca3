"""Dev tool: us per step of the fused rollout's write pattern (tools/trajbench.hip) by
layout (0 step-major rows, 1 env-major rows, 2 one overwritten row) and spin work per step.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o mobile-env-gan_amd/lib/libtrajbench.so
tools/trajbench.hip"""
import ctypes as C
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "mobile-env-gan_amd", "lib", "libtrajbench.so"))
E, U, N = 65536, 30, 20
obs = torch.empty((N, E, U, 4), dtype=torch.float32, device="cuda")
srv = torch.empty((N, E, U), dtype=torch.int32, device="cuda")
rew = torch.empty((N, E), dtype=torch.float32, device="cuda")
done = torch.empty((N, E), dtype=torch.uint8, device="cuda")
tab = torch.randint(0, 100, (40000, 4), dtype=torch.int32, device="cuda")


def run(layout, mode, work, reps):
    s = torch.cuda.current_stream().cuda_stream
    rc = L.tb_run(C.c_void_p(obs.data_ptr()), C.c_void_p(srv.data_ptr()),
                  C.c_void_p(rew.data_ptr()), C.c_void_p(done.data_ptr()),
                  C.c_void_p(tab.data_ptr()), E, N, layout, mode, work, reps, C.c_void_p(s))
    assert rc == 0


for work in (0, 10, 20, 40):
    for mode in (0, 1, 2, 3):
        for layout in (0, 2):
            run(layout, mode, work, 20)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(layout, mode, work, 50)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / 50 / N
            print(json.dumps({"work": work, "mode": mode, "layout": layout,
                              "us_per_step": round(us, 2)}), flush=True)
