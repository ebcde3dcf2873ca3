import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_gpu_parity as T
d = T.load("large")
eng = T.make_engine(d, rate64=False, util64=False, metrics=False, fuse_steps=0)
traj = eng.trajectory(13)
eng.rollout(7, traj)
torch.cuda.synchronize()
print("got", traj.reward[:8].cpu().numpy())
print("want", d["metrics"][:, :7, 2].T)
print("done", traj.done[:8].cpu().numpy())
print("lds", eng.lds_tables_bytes)
