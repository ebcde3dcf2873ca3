"""Dev tool: throughput of the batched collectData2 driver (collect_data) incl. file writing."""
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mobile-env-gan_amd"))
from mobile_env.collect import collect_data  # noqa: E402

for n in (100, 1000):
    root = tempfile.mkdtemp(prefix="mev_collect_")
    t0 = time.perf_counter()
    collect_data(n, root, random_seed=0, device="cuda")
    dt = time.perf_counter() - t0
    nfiles = sum(len(f) for _, _, f in os.walk(root))
    print(json.dumps({"epochs": n, "seconds": dt, "epochs_per_s": n / dt, "files": nfiles,
                      "files_per_s": nfiles / dt}), flush=True)
    shutil.rmtree(root)
