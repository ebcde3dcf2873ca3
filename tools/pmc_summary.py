#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

Reads the rocprofv3 CSVs of the passes (kt: kernel trace + stats; fetch / write / sq / sq2: PMC
counters), keeps the STEP kernel dispatches (k_step_packed / k_step_block, RESET=false), and
writes:
  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --stats summary (copied)
  profiles/<tag>_pmc.json           -- per-launch averages of every counter
  profiles/pmc_traffic.json         -- {workload@envs: hbm_bytes_per_launch, ...} read by bench.py
HBM bytes follow MI355X_MICROARCH.md section HBM: FETCH_SIZE (KB) x 1024 x 2 (gfx950 reports half
of a wide streaming read) + WRITE_SIZE (KB) x 1024.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


STEP_RE = re.compile(r"k_step_packed<|k_step_block<(true|false), false>")


def is_step_kernel(name: str) -> bool:
    return STEP_RE.search(name) is not None


def counters(path_glob):
    vals = {}
    for path in glob.glob(path_glob, recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if not is_step_kernel(row.get("Kernel_Name", "")):
                    continue
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def step_interval(trace_glob, steps):
    """From the kernel trace: step-kernel dispatches of the timed region (the last
    steps x parts), their average duration, and the step interval = (last end - first start)
    / steps -- with two halves per step on two streams the dispatch durations overlap, so
    the interval, not the duration, is the time of a step."""
    rows = []
    for path in glob.glob(trace_glob, recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if is_step_kernel(row.get("Kernel_Name", "")):
                    rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    if not rows or not steps:
        return None
    rows.sort()
    return rows, steps


def main():
    out, tag = sys.argv[1], sys.argv[2]
    extra = sys.argv[3] if len(sys.argv) > 3 else ""
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)
    step_avg_ns = None
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        with open(stats[0]) as f:
            for row in csv.DictReader(f):
                if is_step_kernel(row["Name"]):
                    step_avg_ns = float(row["AverageNs"])
    pmc = {}
    ndisp = {}
    for name in ("fetch", "write", "sq", "sq2"):
        v, n = counters(os.path.join(out, name, "**", "*counter_collection.csv"))
        pmc.update(v)
        ndisp.update(n)
    workload, envs, steps, warmup = "mobile-large-central-v0", 65536, 0, 0
    toks = extra.split()
    for i, t in enumerate(toks):
        if t == "--workload":
            workload = toks[i + 1]
        if t == "--envs":
            envs = int(toks[i + 1])
        if t == "--steps":
            steps = int(toks[i + 1])
        if t == "--warmup":
            warmup = int(toks[i + 1])
    summary = {"tag": tag, "workload": workload, "envs": envs, "bench_args": extra,
               "step_kernel_avg_ns": step_avg_ns, "counters_per_launch": pmc,
               "dispatches_sampled": ndisp}
    tr = step_interval(os.path.join(out, "kt", "**", "*kernel_trace.csv"), steps)
    parts = 1
    if tr:
        rows, _ = tr
        total_steps = steps + warmup
        parts = max(1, round(len(rows) / total_steps))
        timed = rows[-steps * parts:]
        span = max(e for _, e in timed) - timed[0][0]
        summary["launch_parts"] = parts
        summary["timed_dispatches"] = len(timed)
        summary["timed_dispatch_avg_ns"] = sum(e - b for b, e in timed) / len(timed)
        summary["step_interval_ns"] = span / steps
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        # per step = per dispatch x halves per step (the halves are equal-sized)
        fetch = pmc["FETCH_SIZE"] * 1024 * 2 * parts
        write = pmc["WRITE_SIZE"] * 1024 * parts
        summary["hbm_bytes_per_launch"] = fetch + write
        summary["hbm_bytes_per_step"] = fetch + write
        summary["fetch_bytes_per_launch_corrected"] = fetch
        summary["write_bytes_per_launch"] = write
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=2)
    tpath = os.path.join(prof, "pmc_traffic.json")
    traffic = {}
    if os.path.exists(tpath):
        traffic = json.load(open(tpath))
    if "hbm_bytes_per_launch" in summary:
        traffic[f"{workload}@{envs}"] = {
            "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
            "fetch_bytes_per_launch_corrected": summary["fetch_bytes_per_launch_corrected"],
            "write_bytes_per_launch": summary["write_bytes_per_launch"],
            "rocprof_kernel_avg_ns": summary.get("step_kernel_avg_ns"),
            "source": f"profiles/{tag}_pmc.json"}
        with open(tpath, "w") as f:
            json.dump(traffic, f, indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main()
