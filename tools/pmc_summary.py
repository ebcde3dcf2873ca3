#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

usage: python tools/pmc_summary.py RAW_DIR TAG "<bench args of the profile run>" [OUT_DIR]
(OUT_DIR defaults to profiles/; on the GPU box tools/profile.sh writes gpurun_out/profiles/, which
comes back with the call, and tools/merge_profiles.py folds it into profiles/)

Reads the rocprofv3 CSVs of the passes (kt: kernel trace + stats; fetch / write / sq / sq2: PMC
counters) and keeps the dispatches of the launch the bench times:
  * --launch fused (default): the fused multi-step kernel the launch selects -- k_steps_lds2,
    k_steps_packed or k_steps_block (--chunk steps each, one dispatch per chunk);
  * --launch single / split: the one-step kernels k_step_packed / k_steps_block (one step).
Writes
  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --stats summary (copied)
  profiles/<tag>_pmc.json           -- per-launch averages of every counter, timed-region
                                       launch durations from the trace, HBM bytes per launch
  profiles/pmc_traffic.json         -- {workload@envs@launch: {...}} read by bench.py
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
CHUNK = 200  # bench.py default --chunk: steps per engine call (rollout launch)

FUSED_RE = re.compile(r"k_steps_packed<|k_steps_block<|k_steps_lds2<")
SINGLE_RE = re.compile(r"k_step_packed<|k_steps_block<")


def rows_of(path_glob, name_key):
    for path in glob.glob(path_glob, recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def main():
    out, tag = sys.argv[1], sys.argv[2]
    extra = sys.argv[3] if len(sys.argv) > 3 else ""
    workload, envs, steps, warmup, launch = "mobile-large-central-v0", 65536, 0, 0, "fused"
    chunk = CHUNK
    toks = extra.split()
    for i, t in enumerate(toks[:-1]):
        if t == "--workload":
            workload = toks[i + 1]
        elif t == "--envs":
            envs = int(toks[i + 1])
        elif t == "--steps":
            steps = int(toks[i + 1])
        elif t == "--warmup":
            warmup = int(toks[i + 1])
        elif t == "--launch":
            launch = toks[i + 1]
        elif t == "--chunk":
            chunk = int(toks[i + 1])
    kre = FUSED_RE if launch == "fused" else SINGLE_RE
    chunk = min(chunk, steps) if steps else chunk  # bench.py: exactly `steps`, chunk <= steps
    prof = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)

    summary = {"tag": tag, "workload": workload, "envs": envs, "launch": launch,
               "bench_args": extra}
    stats = glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)
    full = None  # the launch's kernel: of the matching instances, the one with the most time
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        rows = [r for r in rows_of(stats[0], "Name") if kre.search(r["Name"])]
        if rows:
            row = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            full = row["Name"]
            summary["kernel"] = re.sub(r"\(\w+::KParams.*", "", row["Name"])
            summary["stats_avg_ns"] = float(row["AverageNs"])
            summary["stats_calls"] = int(row["Calls"])

    def mine(name):  # (another instance -- e.g. the warmup's one-step launch -- is not counted)
        return kre.search(name) and (full is None or name.strip() == full.strip())

    # (a trace whose names do not match the summary's exactly: every matching instance, as before)
    if full is not None and not any(mine(r.get("Kernel_Name", "")) for r in
                                    rows_of(os.path.join(out, "kt", "**", "*kernel_trace.csv"), "")):
        full = None

    # timed region from the trace: the last launches of the kernel
    trace = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in rows_of(os.path.join(out, "kt", "**", "*kernel_trace.csv"), "")
                   if mine(r.get("Kernel_Name", "")))
    steps_per_launch = chunk if launch == "fused" else 1
    parts = 2 if launch == "split" else 1
    n_timed = -(-steps // steps_per_launch) * parts  # whole chunks + the remainder launch
    if trace and n_timed:
        timed = trace[-n_timed:]
        span = max(e for _, e in timed) - timed[0][0]
        summary["steps_per_launch"] = steps_per_launch
        summary["timed_launches"] = len(timed)
        summary["timed_launch_avg_ns"] = sum(e - b for b, e in timed) / len(timed)
        summary["step_interval_ns"] = span / steps

    # counters: per-dispatch averages over the kernel's dispatches of each pass (the fused
    # warmup launches are whole chunks too, so every dispatch is the same work)
    pmc, ndisp = {}, {}
    for name in ("fetch", "write", "sq", "sq2", "sq3"):
        vals = {}
        for r in rows_of(os.path.join(out, name, "**", "*counter_collection.csv"), ""):
            if mine(r.get("Kernel_Name", "")):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc[k] = sum(v) / len(v)
            ndisp[k] = len(v)
    summary["counters_per_launch"] = pmc
    summary["dispatches_sampled"] = ndisp
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"] * 1024 * 2 * parts
        write = pmc["WRITE_SIZE"] * 1024 * parts
        summary["hbm_bytes_per_launch"] = fetch + write
        summary["hbm_bytes_per_step"] = (fetch + write) / steps_per_launch
        summary["fetch_bytes_per_launch_corrected"] = fetch
        summary["write_bytes_per_launch"] = write
    if "SQ_INSTS_VALU" in pmc:
        # per env group (the envs of one wavefront, 64 // segment pitch) and step: the
        # persistent fused kernel runs fewer waves, each over several groups
        sys.path.insert(0, os.path.join(ROOT, "mobile-env-gan_amd"))
        from mobile_env.scenarios.registry import SCENARIOS
        U = SCENARIOS[workload]["num_ues"]
        if U > 64:  # block shape: one workgroup per env -> counts per env-step
            groups = envs
        else:
            pitch = (16 if 8 < U <= 16 and 64 // U == 4 else
                     32 if 16 < U <= 32 and 64 // U == 2 else U)
            groups = -(-envs // (64 // pitch))
        summary["groups_per_launch"] = groups
        summary["valu_per_group_step"] = pmc["SQ_INSTS_VALU"] / groups / steps_per_launch
        summary["salu_per_group_step"] = pmc["SQ_INSTS_SALU"] / groups / steps_per_launch
        summary["lds_per_group_step"] = pmc.get("SQ_INSTS_LDS", 0.0) / groups / steps_per_launch
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=2)

    tpath = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    if "hbm_bytes_per_launch" in summary:
        traffic[f"{workload}@{envs}@{launch}" + (f"@{chunk}" if launch == "fused" else "")] = {
            "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
            "fetch_bytes_per_launch_corrected": summary["fetch_bytes_per_launch_corrected"],
            "write_bytes_per_launch": summary["write_bytes_per_launch"],
            "steps_per_launch": steps_per_launch,
            "rocprof_launch_avg_ns": summary.get("timed_launch_avg_ns"),
            "source": f"profiles/{tag}_pmc.json"}
        with open(tpath, "w") as f:
            json.dump(traffic, f, indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main()
