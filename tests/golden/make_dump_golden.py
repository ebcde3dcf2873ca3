"""Golden files of the reference's dataset writer.

Runs ONLY in the development container (the reference checkout is at /root/reference; the
GPU box only reads the committed tests/golden/dump_mcom_custom.json). Imports the reference
with the stubs of make_golden.py, keeps its per-step dump ON (base.py:261,298-349) and runs
the collectData2.ipynb driver (cells 2-4: MComCustom(), reset(); then per epoch reset(),
save_base_station_positions(epoch), step(epoch, s) x 20, save_epoch_data(epoch)) from a
scratch directory, so the files land in <scratch>/collectData and <scratch>/collectData2.
Every file written is stored verbatim as {relative path: text}, per global random seed.
Usage:  python tests/golden/make_dump_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REF, _install_stubs  # noqa: E402

RANDOM_SEEDS = (0, 3)
EPOCHS = 2
STEPS = 20


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    from mobile_env.scenarios.custom import MComCustom  # noqa: E402

    out = {"random_seeds": list(RANDOM_SEEDS), "epochs": EPOCHS, "steps": STEPS, "runs": []}
    for k in RANDOM_SEEDS:
        scratch = tempfile.mkdtemp(prefix="mev_dump_")
        work = os.path.join(scratch, "work")
        os.makedirs(work)
        os.chdir(work)  # the reference writes to ../collectData and ../collectData2
        random.seed(k)
        env = MComCustom()
        env.reset()  # cell 3
        for epoch in range(EPOCHS):
            env.reset()
            env.save_base_station_positions(epoch)
            for s in range(STEPS):
                env.step(epoch, s)
            env.save_epoch_data(epoch)
        files = {}
        for top in ("collectData", "collectData2"):
            for dirpath, _, names in os.walk(os.path.join(scratch, top)):
                for n in names:
                    p = os.path.join(dirpath, n)
                    files[os.path.relpath(p, scratch)] = open(p).read()
        out["runs"].append({"random_seed": k, "files": files})
        print(f"random.seed({k}): {len(files)} files")
    with open(os.path.join(HERE, "dump_mcom_custom.json"), "w") as f:
        json.dump(out, f, sort_keys=True)
    print("wrote dump_mcom_custom.json")


if __name__ == "__main__":
    main()
