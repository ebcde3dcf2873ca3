import sys, os, numpy as np, torch
sys.path.insert(0, "mobile-env-gan_amd"); sys.path.insert(0, ".")
from mobile_env.core.engine import EngineParams, StepEngine
from mobile_env.scenarios.registry import LAYOUTS
L = LAYOUTS["medium"]; E = 40000
for rep in range(int(os.environ.get("REPS", "3"))):
    outs = []
    for split, table, fuse in ((1, -1, 0), (2, -1, 0), (1, 0, 0), (1, -1, -1)):
        p = EngineParams(num_envs=E, num_ues=L["num_ues"], num_bs=len(L["bs"]), velocity=10.0,
                         stream_split=split, draw_table=table, fuse_steps=fuse)
        eng = StepEngine(p, L["bs"], 1000 + np.arange(E), device="cuda")
        eng.step(45); torch.cuda.synchronize()
        outs.append([x.cpu().clone() for x in (eng.ue_state, eng.pcg, eng.t, eng.obs, eng.serving, eng.reward, eng.done)])
        eng.close()
    names = ("ue_state","pcg","t","obs","serving","reward","done")
    for k, o in enumerate(outs[1:], 1):
        for n, a, b in zip(names, outs[0], o):
            if not torch.equal(a, b):
                d = (a != b).nonzero()
                print(rep, "cfg", k, n, "ndiff", d.shape[0], "first", d[:3].tolist(),
                      a[tuple(d[0])].item(), b[tuple(d[0])].item(), flush=True)
    print(rep, "done", flush=True)
