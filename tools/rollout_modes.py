"""Dev tool: us per step of the launch shapes at 65,536 mobile-large envs --
fused step(20) (outputs overwritten), fused rollout(20) (trajectory rows), 20 one-step launches.
usage: python tools/rollout_modes.py [E] [U-scenario]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
WL = sys.argv[2] if len(sys.argv) > 2 else "mobile-large-central-v0"
W, K, S = 2000, int(os.environ.get("K", 2000)), int(os.environ.get("S", 20))


def timed(fn):
    for _ in range(W // S):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(K // S):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / K


MODES = os.environ.get("MODES", "fused_overwrite,rollout,single,rollout10,rollout5,rollout4,"
                                "rollout2").split(",")
for mode in MODES:
    env = mobile_env.make(WL, num_envs=E, device="cuda:0", seed=1000,
                          fuse_steps=-1 if mode == "single" else 0)
    env.reset()
    eng = env.engine
    traj = eng.trajectory(S)
    if mode.startswith("rollout"):
        k = int(mode[7:] or S)

        def fn():
            for j in range(0, S, k):  # trajectory rows j..j+k of the episode
                eng.rollout(k, traj.rows(j, k))
    else:
        def fn():
            eng.step(S)
    print(json.dumps({"lib": os.path.basename(os.environ.get("MEV_LIB", "libmev.so")),
                      "mode": mode, "envs": E, "workload": WL, "us_per_step": timed(fn)}),
          flush=True)
    env.close()
    del traj
