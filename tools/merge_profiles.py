#!/usr/bin/env python3
"""Fold the profile summaries a GPU call brought back (gpurun_out/profiles/: <tag>_kernel_stats.csv,
<tag>_pmc.json, pmc_traffic.json entries) into the committed profiles/ directory.

usage: python tools/merge_profiles.py [gpurun_out/profiles]"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "profiles")
    dst = os.path.join(ROOT, "profiles")
    for f in glob.glob(os.path.join(src, "*_kernel_stats.csv")) + \
            glob.glob(os.path.join(src, "*_pmc.json")):
        shutil.copy(f, dst)
        print("copied", os.path.basename(f))
    new = os.path.join(src, "pmc_traffic.json")
    if os.path.exists(new):
        path = os.path.join(dst, "pmc_traffic.json")
        cur = json.load(open(path)) if os.path.exists(path) else {}
        cur.update(json.load(open(new)))
        with open(path, "w") as f:
            json.dump(cur, f, indent=2)
        print("merged pmc_traffic.json")


if __name__ == "__main__":
    main()
