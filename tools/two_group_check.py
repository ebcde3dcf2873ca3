import sys, os, torch, numpy as np
sys.path.insert(0, "mobile-env-gan_amd")
import mobile_env
for E in (4096, 1000, 7):
    runs = []
    for tg in (1, -1):
        env = mobile_env.make("mobile-medium-central-v0", num_envs=E, device="cuda:0", seed=5, two_groups=tg)
        env.reset()
        tr = env.engine.trajectory(45)
        env.engine.rollout(45, tr)
        torch.cuda.synchronize()
        runs.append([x.cpu() for x in (tr.obs, tr.serving, tr.reward, tr.done, env.engine.ue_state, env.engine.t)])
        env.close()
    print(E, all(torch.equal(a, b) for a, b in zip(*runs)), flush=True)
