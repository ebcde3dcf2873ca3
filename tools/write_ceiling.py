"""Dev tool (GPU box): the box's HBM write rate for a plain streaming store, to set the rollout
launch's achieved rate against: torch's fill_ over an 8.0 GB buffer (the 200-step launch's own
bytes) and over 0.86 GB (the 20-step launch's), HIP events around each of 20 launches, median.
Prints one JSON line."""
import json
import statistics

import torch


def rate(nbytes: int, reps: int = 20):
    x = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    for _ in range(3):
        x.fill_(1.0)
    torch.cuda.synchronize()
    ts = []
    for i in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        x.fill_(float(i))
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    del x
    torch.cuda.empty_cache()
    t = statistics.median(ts)
    return {"bytes": nbytes, "median_ms": t * 1e3, "tb_per_s": nbytes / t / 1e12}


if __name__ == "__main__":
    print(json.dumps({"fill_8.0GB": rate(8_000_372_736), "fill_0.86GB": rate(863_502_336)}),
          flush=True)
