#!/usr/bin/env python3
"""Benchmark: whole-node env-steps/s of the fused HIP step on mobile-large-central-v0.

Contract (see DESIGN.md "Measurement"):
  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

* One step = one pass of the step over every env on the GPU (BASELINE.json configs[2]:
  65,536 envs of mobile-large-central-v0 per MI355X; weak scaling: each rank owns its own
  65,536 independent envs, seeds 1000 + global env index). By default steps are issued as
  ``engine.rollout(40, traj)`` (mev_rollout, two 20-step episodes with the lazy auto-reset
  between them, as the reference driver loop ``reset(); step() x 20`` repeated): ONE launch of
  the fused multi-step kernel, which keeps every env's state in registers between the steps
  and writes EVERY step's outputs (obs, serving, reward, done) to its own row of a
  [40, E, ...] trajectory buffer in HBM -- the per-step outputs the reference's driver
  consumes every step (base.py:261) -- bit-identical to 40 one-step launches (--chunk sets
  the steps per launch; 20 = one episode: ~5 % slower, the launch's fill and drain and the
  per-group prologue counted over fewer steps). ``--launch single`` issues one-step launches
  (mev_step(1), outputs overwritten) instead; ``split`` two env halves.
* Timed region: barrier + synchronize, K steps, the single final all-gather of the
  (reward, done) batch over RCCL when N > 1, synchronize + barrier. value = N*E*K / max-over-
  ranks time. Inputs are resident in HBM before timing starts.
* roofline: algorithmic bytes per launch over the launch's average duration from HIP events
  on the stream the kernel runs on (around every launch; for one-step launches around every
  chunk of 20, gaps included). One-step launch: SURVEY.md 8d's per-unit figure, (54*U + 61) B
  per env-step (canonical: state r+w 34 B/UE + outputs 20 B/UE; per env 61 B), x E. A rollout
  launch of n steps keeps the env state in registers between its steps, so its algorithmic
  bytes are every step's outputs, E * n * (20*U + 5), plus the canonical state read and
  written once, E * (34*U + 56) -- counting the canonical per-step state round trip instead
  (`canonical_equiv_*`) would put the rate above the HBM peak. The PMC `traffic` is what the
  launch actually moved.
  traffic: HBM bytes per launch from the committed rocprofv3 PMC summary
  (profiles/pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the MI355X guide), else null.
* cpu_baseline (rank 0, N = 1): the per-object CPU port of the reference step (oracle/port.py,
  bit-exact vs the reference fixtures) on a bounded sample of the same workload, one process
  per core, run before the GPU is touched.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mobile-env-gan_amd"))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), mobile-large-central-v0 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes_per_env_step(num_ues: int, per_env_bs: bool, num_bs: int) -> int:
    # SURVEY.md 8d canonical layout: per UE 34 B state r+w + 20 B outputs; per env 61 B
    return 54 * num_ues + 61 + (8 * num_bs if per_env_bs else 0)


def algorithmic_bytes_rollout(num_ues: int, per_env_bs: bool, num_bs: int, n: int) -> int:
    """Per env, one rollout launch of n steps: every step's outputs (obs 16 B + serving 4 B
    per UE, reward 4 + done 1 per env; per-env layouts: 8 B per station per step) plus the
    canonical state read and written once (34 B per UE; PCG64 state r+w 32, inc 16, t r+w 8)."""
    per_step = 20 * num_ues + 5 + (8 * num_bs if per_env_bs else 0)
    return n * per_step + 34 * num_ues + 56


# ---------------------------------------------------------------------------------------------
# CPU baseline: the per-object port of the reference step, one process per core
# ---------------------------------------------------------------------------------------------
def _cpu_worker(args):
    layout, num_ues, seed0, budget_s = args
    from oracle import port
    done = 0
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        core = port.build(layout, num_ues, seed0 + k, 1.5)
        core.reset()
        for _ in range(20):
            core.step()
            done += 1
        k += 1
    return done, time.perf_counter() - t0


def cpu_baseline(budget_s: float, procs: int):
    from mobile_env.scenarios.registry import LAYOUTS
    lay = LAYOUTS["large"]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(lay["bs"], lay["num_ues"], 1000 + 100000 * i, budget_s)
                                     for i in range(procs)])
    wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "sample": (f"oracle/port.py per-object restatement of MComCore.step, "
                       f"mobile-large-central-v0 (13 BS x 30 UE), {procs} processes x "
                       f"{budget_s:.0f} s of whole 20-step episodes, seeds 1000+, compute-only "
                       f"(no JSON dump): {steps} env-steps in {wall:.1f} s")}


def load_profile(workload: str, envs: int, launch: str = "fused", chunk: int = 40):
    """(HBM bytes per launch from the PMC passes, rocprofv3 average launch duration in ms of
    the timed region) of the committed profile of this workload and launch shape
    (tools/profile.sh + tools/pmc_summary.py), or Nones."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    ent = d.get(f"{workload}@{envs}@{launch}" + (f"@{chunk}" if launch == "fused" else "")) or {}
    avg_ns = ent.get("rocprof_launch_avg_ns")
    return ent.get("hbm_bytes_per_launch"), (avg_ns * 1e-6 if avg_ns else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--workload", default="mobile-large-central-v0")
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--launch", default="fused", choices=("fused", "single", "split"),
                    help="fused: one rollout launch per chunk of steps, every step's outputs "
                         "kept (default); single: one launch per step; split: one launch per step "
                         "on two HIP streams (two env halves)")
    ap.add_argument("--chunk", type=int, default=40,
                    help="steps per engine call: per rollout launch (fused), or per C loop of "
                         "one-step launches (single / split); 40 = two episodes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-run", action="store_true",
                    help="minimal run for rocprofv3 (no CPU baseline, no JSON extras)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not (args.no_cpu_baseline or args.profile_run):
        procs = max(1, min(16, os.cpu_count() or 1))
        cpu = cpu_baseline(args.cpu_budget, procs)

    import torch
    import torch.distributed as dist

    import mobile_env

    # one process per GPU over RCCL; on a box with fewer GPUs than ranks (rehearsal only) the
    # ranks share devices and fall back to gloo (RCCL refuses two ranks on one GPU)
    ndev = max(1, torch.cuda.device_count())
    device = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("MEV_DIST_BACKEND", "nccl" if ndev >= world else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    from mobile_env.sharding import gather_final, shard_seeds

    E = args.envs
    seeds = shard_seeds(1000, E, rank)  # rank r owns global envs [r*E, (r+1)*E)
    env = mobile_env.make(args.workload, num_envs=E, device=device, seed=int(seeds[0]),
                          stream_split=2 if args.launch == "split" else 0,
                          fuse_steps=0 if args.launch == "fused" else -1)
    U, B = env.num_ues, env.num_bs
    per_env_bs = env.engine.bs_per_env
    parts = env.engine.launch_parts
    env.reset()
    CHUNK = args.chunk  # steps per engine call (two 20-step episodes by default)
    fused = args.launch == "fused" and env.engine.fused_steps
    traj = env.engine.trajectory(CHUNK) if args.launch == "fused" else None

    def chunk():
        if traj is not None:
            env.engine.rollout(CHUNK, traj)  # every step's outputs to its own row
        else:
            env.engine.step(CHUNK)

    # warmup (also brings the GPU to its steady clock): the Gym step once, then chunks
    if args.warmup > 0:
        env.step()
        for _ in range(-(-(args.warmup - 1) // CHUNK)):
            chunk()
    torch.cuda.synchronize(device)

    # Steps are issued in chunks of CHUNK from C (fused: one rollout launch per chunk; single:
    # CHUNK back-to-back launches -- a Python call per step would make the host the bottleneck),
    # with a HIP event pair around every chunk on the caller's stream. With the two-half
    # launch shape the second half runs on the context's own stream and is joined back
    # before mev_step returns, so each event pair brackets whole steps of the full batch.
    K = -(-args.steps // CHUNK) * CHUNK
    stream = torch.cuda.current_stream(device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K // CHUNK)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        chunk()
        b.record(stream)
    if world > 1:  # the one collective: final (reward, done) batch to every rank
        if traj is not None:  # the last step's row of the trajectory
            gather_final(traj.reward[CHUNK - 1], traj.done[CHUNK - 1])
        else:
            gather_final(env.engine.reward, env.engine.done)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / K

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        value = world * E * K / elapsed
        spl = CHUNK if fused else 1  # steps per launch
        canon_bytes = E * spl * algorithmic_bytes_per_env_step(U, per_env_bs, B)
        algo_bytes = (E * algorithmic_bytes_rollout(U, per_env_bs, B, spl) if fused
                      else canon_bytes)
        launch_ms = kern_ms * spl
        achieved = algo_bytes / (launch_ms * 1e-3) / 1e9
        traffic, rocprof_ms = load_profile(args.workload, E, args.launch, CHUNK)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded PCG64 streams, build-defined BS layout)",
            "config": {"workload": args.workload, "envs_per_gpu": E, "global_envs": world * E,
                       "num_ues": U, "num_bs": B,
                       "parallelism": f"env-sharded x{world}, no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_frac": (traffic / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                          if traffic else None),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "canonical_bytes_per_env_step": algorithmic_bytes_per_env_step(
                             U, per_env_bs, B),
                         "canonical_equiv_achieved": canon_bytes / (launch_ms * 1e-3) / 1e9,
                         "canonical_equiv_frac": (canon_bytes / (launch_ms * 1e-3) / 1e9 /
                                                  HBM_PEAK_GBS),
                         "steps_per_launch": spl,
                         "launch_ms": launch_ms,
                         "rocprof_launch_ms": rocprof_ms,
                         "launch_shape": (
                             f"fused rollout: {spl} steps per launch, env state in registers "
                             f"between them, every step's outputs to its own trajectory row"
                             if fused else
                             f"{parts} halves per step on {parts} HIP streams" if parts > 1
                             else "one kernel per step")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
