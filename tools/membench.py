"""Dev tool: memory floor of the step's access pattern vs the real kernel (same process)."""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mobile-env-gan_amd"))
SO = os.path.join(ROOT, "mobile-env-gan_amd", "lib", "libmembench.so")


def timeit(fn, n=100, reps=20):
    """Median over n chunks of `reps` back-to-back launches issued from C (the host loop
    never starves the GPU), per launch."""
    fn(2000)  # to steady GPU clocks
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn(reps)
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 / reps for a, b in ev)
    return t[len(t) // 2]


def main():
    L = C.CDLL(SO)
    E, U = 65536, 30
    dev = torch.device("cuda")
    st = torch.zeros((E, U, 4), dtype=torch.int32, device=dev)
    pcg = torch.zeros((E, 6), dtype=torch.int64, device=dev)
    t = torch.zeros(E, dtype=torch.int32, device=dev)
    obs = torch.zeros((E, U, 4), dtype=torch.float32, device=dev)
    srv = torch.zeros((E, U), dtype=torch.int32, device=dev)
    rew = torch.zeros(E, dtype=torch.float32, device=dev)
    done = torch.zeros(E, dtype=torch.uint8, device=dev)
    s = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda x: C.c_void_p(x.data_ptr())
    algo = E * (54 * U + 61)
    us = timeit(lambda r: L.mb_pattern(p(st), p(pcg), p(t), p(obs), p(srv), p(rew), p(done), E, U, r, s()))
    print(json.dumps({"kernel": "pattern", "us": us, "algo_GBs": algo / us / 1e3}))
    n = (E * U * 16 + E * 36) // 16  # read bytes / 16
    a = torch.zeros(n * 4, dtype=torch.float32, device=dev)
    b = torch.zeros(n * 8, dtype=torch.float32, device=dev)
    us = timeit(lambda r: L.mb_stream(p(a), p(b), C.c_size_t(n), r, s()))
    print(json.dumps({"kernel": "stream1r2w", "us": us, "bytes": n * 48, "GBs": n * 48 / us / 1e3}))
    us = timeit(lambda r: L.mb_empty(p(t), 8192, r, s()))
    print(json.dumps({"kernel": "empty_8192x256", "us": us}))
    us = timeit(lambda r: L.mb_empty(p(t), 2048, r, s()))
    print(json.dumps({"kernel": "empty_2048x256", "us": us}))
    us = timeit(lambda r: L.mb_touch(p(st), p(t), E * U, r, s()))
    print(json.dumps({"kernel": "read_state_only", "us": us, "GBs": E * U * 16 / us / 1e3}))
    n2 = 64 << 20
    a = torch.zeros(n2 * 4, dtype=torch.float32, device=dev)
    b = torch.zeros(n2 * 8, dtype=torch.float32, device=dev)
    us = timeit(lambda r: L.mb_stream(p(a), p(b), C.c_size_t(n2), r, s()), 30, 2)
    print(json.dumps({"kernel": "stream1r2w_3GB", "us": us, "GBs": n2 * 48 / us / 1e3}))


if __name__ == "__main__":
    main()
