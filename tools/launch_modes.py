"""Dev tool: host launch modes for consecutive steps (python loop / C loop / HIP graph)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
import mobile_env  # noqa: E402

E, K = 65536, 400
env = mobile_env.make("mobile-large-central-v0", num_envs=E, device="cuda:0", seed=1000)
env.reset()
for _ in range(40):
    env.step()
torch.cuda.synchronize()


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6


def py_loop():
    for _ in range(K):
        env.step()


def c_loop():
    env.engine.step(K)


print(json.dumps({"mode": "python_loop", "us_per_step": wall(py_loop)}))
print(json.dumps({"mode": "c_loop", "us_per_step": wall(c_loop)}))
S = 20
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    env.step()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    for _ in range(S):
        env.step()
torch.cuda.synchronize()


def graph_loop():
    for _ in range(K // S):
        g.replay()


print(json.dumps({"mode": "graph20", "us_per_step": wall(graph_loop)}))
print(json.dumps({"mode": "c_loop", "us_per_step": wall(c_loop)}))
