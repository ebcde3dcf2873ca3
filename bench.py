#!/usr/bin/env python3
"""Benchmark: whole-node env-steps/s of the fused HIP step on mobile-large-central-v0.

Contract (see DESIGN.md "Measurement"):
  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

* One step = one pass of the step over every env on the GPU (BASELINE.json configs[2]:
  65,536 envs of mobile-large-central-v0 per MI355X; weak scaling: each rank owns its own
  65,536 independent envs, seeds 1000 + global env index). Steps are issued as rollout launches
  of ``--chunk`` steps (default 200 = ten 20-step episodes with the lazy auto-reset between
  them, as the reference driver loop ``reset(); step() x 20`` repeated): ONE launch of the fused
  multi-step kernel per chunk, which keeps every env's state in registers between its steps and
  writes EVERY step's outputs (obs, serving, reward, done) to its own row of a trajectory buffer
  in HBM -- the per-step outputs the reference's driver consumes every step (base.py:261) --
  bit-identical to one-step launches. Exactly K steps are timed: K // chunk launches of
  ``chunk`` steps and one launch of the remainder. ``--launch single`` issues one-step
  launches (mev_step(1), the Gym ``step()``) instead.
* Warmup: W steps, and then more until ``--warmup-floor-s`` seconds of back-to-back launches
  have run (untimed; the chip reaches its steady clock -- a 5-step warmup would time a cold
  launch), then one untimed rehearsal of the timed region (its launches, gather and syncs).
  ``warmup`` in the line is W as requested; ``warmup_executed`` what ran.
* Timed region: barrier + synchronize, then the clock runs over the K steps and, when N > 1, a
  synchronize and the single final all-gather of the (reward, done) batch over RCCL, to the
  synchronize after it; the trailing barrier is outside the window (timed on its own,
  `distributed.trailing_barrier_ms`). value = N*E*K / max-over-ranks window. Nothing else runs inside it (no event record). Inputs are resident in
  HBM before timing starts. With N > 1 both collectives (final batch, obs) run once in the
  untimed warmup, so the timed gather is not the process's first; the line reports the timed
  gather's own wall time (`distributed.final_gather_ms`, its share of the window) and the
  rate without it (`distributed.value_steps_only`).
* roofline (the timed launch shape): algorithmic bytes per launch over the launch's average
  duration from HIP events on the stream the kernel runs on, measured after the timed region
  on 30 launches of the timed shape (isolated launches when the region was one launch). A rollout launch of n steps keeps
  the env state in registers between its steps, so its algorithmic bytes are every step's
  outputs, E * n * (20*U + 5), plus the canonical state read and written once,
  E * (34*U + 56); SURVEY.md 8d's canonical per-step figure (54*U + 61 B per env-step) counts a
  state round trip per step that the launch does not make, and would put the rate above the
  HBM peak (`canonical_equiv_frac`). `traffic`: HBM bytes per launch from the committed
  rocprofv3 PMC summary (profiles/pmc_traffic.json; FETCH_SIZE x 2 + WRITE_SIZE per the MI355X
  guide), else null.
* roofline_step: the one-step launch of ``make().step()`` (mev_step(1)), timed after the timed
  region (200 back-to-back launches in 10 groups, HIP events around each group), on SURVEY.md
  8d's canonical bytes per env-step x E -- the canonical unit of work at its canonical byte
  count.
* cpu_baseline (rank 0, N = 1): the per-object CPU port of the reference step (oracle/port.py,
  bit-exact vs the reference fixtures) on a bounded sample of the same workload, one process
  per core of the host share, run before the GPU is touched.
* N > 1 without a launcher (``python bench.py --gpus N``, WORLD_SIZE unset): this process starts
  the N rank processes itself (torch.distributed.run on 127.0.0.1, a free port) before it touches
  the GPU, and exits with their exit code; each rank runs the contract above. The line reports
  the world size and backend the ranks saw, and (outside the step timing) the north-star final
  obs all-gather over RCCL (mobile_env.sharding.gather_obs): its time and bytes.
* --stub-engine: a CPU stand-in engine with the gloo backend (tests of the launcher, sharding and
  timing glue on a machine without a GPU; never a measurement).
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


def dtype_string(state_bytes_per_ue: int) -> str:
    """The arithmetic types the timed path computes in: the UE state rows in their kernel form
    (mev_state_bytes_per_ue: 4 = the compact uint8 x4 rows of maps <= 255 per side, every
    registered scenario; 8 = int16 x4), int32 squared distances and association keys, float64
    rates and ResourceFair cents, float32 obs and utility, and the reward as an int32 2^-25
    fixed-point sum over the env's UEs (float32 at the end)."""
    state = ("uint8x4 compact UE state (x, y, waypoint; 255 = none)" if state_bytes_per_ue == 4
             else "int16x4 UE state (x, y, waypoint)")
    return (f"mixed: {state}, int32 d2 / association keys, f64 rate and cents, f32 obs / "
            "utility, int32 2^-25 fixed-point reward sum -> f32")


def algorithmic_bytes_per_env_step(num_ues: int, per_env_bs: bool, num_bs: int) -> int:
    # SURVEY.md 8d canonical layout: per UE 34 B state r+w + 20 B outputs; per env 61 B
    return 54 * num_ues + 61 + (8 * num_bs if per_env_bs else 0)


def algorithmic_bytes_rollout(num_ues: int, per_env_bs: bool, num_bs: int, n: int) -> int:
    """Per env, one rollout launch of n steps: every step's outputs (obs 16 B + serving 4 B
    per UE, reward 4 + done 1 per env) plus the canonical state read and written once (34 B per
    UE; PCG64 state r+w 32, inc 16, t r+w 8; per-env layouts: the 8 B per station read once)."""
    per_step = 20 * num_ues + 5
    return n * per_step + 34 * num_ues + 56 + (8 * num_bs if per_env_bs else 0)


def chunk_plan(steps: int, chunk: int):
    """Launch sizes that add up to exactly `steps`: whole chunks, then the remainder."""
    chunk = max(1, min(chunk, steps)) if steps > 0 else 1
    plan = [chunk] * (steps // chunk)
    if steps % chunk:
        plan.append(steps % chunk)
    return plan


def timed_run(issue, plan, sync, barrier, collective=None):
    """The timed region: barrier + sync, then the clock runs over every launch of `plan` and the
    final collective (if any), up to the sync after them. Nothing else happens inside it: no
    event is recorded (a launch's duration is measured after the region, `launch_timing`). With a
    collective the launches are synchronised before it, so that its share of the window is known
    (`final_gather_ms`). The trailing barrier only lines the ranks up for what follows: it is
    timed on its own and NOT part of the window (with N > 1 an RCCL barrier is an all-reduce plus
    a sync, tens of us against a ~190 us 20-step window) -- each rank's window ends when its own
    work and the gather have completed, and the line takes the max over ranks of that.
    Returns (wall s of the window, wall s to the end of the launches, wall s of the collective,
    wall s of the trailing barrier)."""
    barrier()
    sync()
    t0 = time.perf_counter()
    for n in plan:
        issue(n)
    t_steps = t_coll = None
    if collective is not None:
        sync()
        t_steps = time.perf_counter() - t0
        collective()
    sync()
    t_end = time.perf_counter()
    if collective is not None:
        t_coll = t_end - t0 - t_steps
    else:
        t_steps = t_end - t0
    barrier()
    return t_end - t0, t_steps, t_coll, time.perf_counter() - t_end


def launch_timing(issue, n, reps, sync, make_event, isolated):
    """Average duration in ms of a launch of n steps, from an event pair around each of `reps`
    launches on the launch stream, run AFTER the timed region: isolated launches (synchronize
    before each; the shape of a timed region of one launch, the driver's --steps 20) or back to
    back (the shape of a timed region of many launches). Returns (mean, median) in ms."""
    evs = [(make_event(), make_event()) for _ in range(reps)]
    sync()
    for a, b in evs:
        if isolated:
            sync()
        a.record()
        issue(n)
        b.record()
    sync()
    ms = sorted(a.e.elapsed_time(b.e) for a, b in evs)
    return sum(ms) / len(ms), ms[len(ms) // 2]


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a float over the ranks of the default group (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------------------------------------
# CPU baseline: the per-object port of the reference step, one process per core
# ---------------------------------------------------------------------------------------------
def _cpu_worker(args):
    layout, num_bs, num_ues, velocity, seed0, budget_s, classes = args
    import numpy as np
    from oracle import port
    done = 0
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        # per-env-layout workloads: a uniform integer layout per episode (vector._bs_layouts)
        lay = layout if layout is not None else \
            np.random.default_rng(seed0 + k).integers(0, 200, size=(num_bs, 2)).tolist()
        core = port.build(lay, num_ues, seed0 + k, velocity, classes=classes)
        core.reset()
        for _ in range(20):  # an episode, or as much of it as the budget allows
            core.step()
            done += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        k += 1
    return done, time.perf_counter() - t0


def host_share_cores() -> int:
    """Cores of the host share this process may use: its affinity set, capped by the pool's
    per-GPU CPU share (OMP_NUM_THREADS is set to it on the GPU boxes, 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(budget_s: float, procs: int, workload: str = "mobile-large-central-v0"):
    """The per-object port of the reference step on `workload`'s sizes (registered ids; the
    default velocity 1.5 of MComCore.default_config where the scenario sets none)."""
    from mobile_env.scenarios import registry
    sp = registry.spec(workload)
    lay = registry.LAYOUTS[sp["layout"]]["bs"] if not sp["per_env_layout"] else None
    U, B = sp["num_ues"], sp["num_bs"]
    vel = sp["velocity"] if sp["velocity"] is not None else 1.5
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(lay, B, U, vel, 1000 + 100000 * i, budget_s,
                                      sp.get("classes")) for i in range(procs)])
    wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": (f"oracle/port.py per-object restatement of MComCore.step, "
                       f"{workload} ({B} BS x {U} UE), {procs} processes (one per "
                       f"core of the host share) x {budget_s:.0f} s of 20-step episodes, "
                       f"seeds 1000+, compute-only (no JSON dump): {steps} env-steps in "
                       f"{wall:.1f} s")}


def load_profile(workload: str, envs: int, launch: str = "fused", chunk: int = 200):
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


def roofline(algo_bytes, launch_ms, traffic):
    achieved = algo_bytes / (launch_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_frac": (traffic / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                             if traffic else None),
            "algorithmic_bytes_per_launch": algo_bytes, "launch_ms": launch_ms}


class StubEnv:
    """CPU stand-in for the GPU engine (--stub-engine; tests only): after k steps every env's
    reward is its config seed + k, done = (k % 20 == 0) and its obs rows hold the seed -- so a
    gathered batch is checkable."""
    bs_per_env = False
    launch_parts = 1
    fused_steps = True

    def __init__(self, num_envs, num_ues, num_bs, seeds):
        import torch
        self.engine = self
        self.num_ues, self.num_bs = num_ues, num_bs
        self.seeds = torch.as_tensor(seeds, dtype=torch.float32)
        self.k = 0
        self.obs = torch.zeros((num_envs, num_ues, 4))
        self.reward = torch.zeros(num_envs)
        self.done = torch.zeros(num_envs, dtype=torch.uint8)

    def trajectory(self, n):
        import types
        import torch
        E, U = self.obs.shape[:2]
        return types.SimpleNamespace(obs=torch.zeros((n, E, U, 4)), reward=torch.zeros((n, E)),
                                     done=torch.zeros((n, E), dtype=torch.uint8))

    def launcher(self, n, traj=None):
        def go():
            for i in range(n):
                self.k += 1
                r, d = self.seeds + self.k, int(self.k % 20 == 0)
                o, rw, dn = ((traj.obs[i], traj.reward[i], traj.done[i]) if traj is not None
                             else (self.obs, self.reward, self.done))
                o.copy_(self.seeds[:, None, None].expand_as(o))
                rw.copy_(r)
                dn.fill_(d)
        return go

    def reset(self):
        self.k = 0

    def step(self):
        self.launcher(1)()

    def close(self):
        pass


def spawn_ranks(n: int, argv) -> int:
    """``bench.py --gpus N`` without a launcher: start the N ranks under torch.distributed.run
    (127.0.0.1, a free port) and return their exit code. This process has not touched the GPU
    (nothing before this point initialises HIP), so starting fresh processes is safe."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__),
           *argv]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--warmup-floor-s", type=float, default=2.0,
                    help="untimed warmup continues until this many seconds have run")
    ap.add_argument("--workload", default="mobile-large-central-v0")
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--launch", default="fused", choices=("fused", "single", "split"),
                    help="fused: one rollout launch per chunk of steps, every step's outputs "
                         "kept (default); single: one launch per step; split: one launch per step "
                         "on two HIP streams (two env halves)")
    ap.add_argument("--chunk", type=int, default=200,
                    help="steps per engine call: per rollout launch (fused), or per C loop of "
                         "one-step launches (single / split); 200 = ten episodes (measured at "
                         "65,536 large envs: 40 steps 6.6e9, 80 7.0e9, 200 7.3e9, 400 7.4e9 "
                         "env-steps/s -- the per-launch tail and the per-group prologue amortised)")
    ap.add_argument("--step-launches", type=int, default=200,
                    help="one-step launches timed after the timed region for roofline_step")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="engine launch-shape override (EngineParams: lds_tables, two_groups, "
                         "stage_rows, xcd_remap, scenario_constants), for A/B runs")
    ap.add_argument("--host-wait", default="auto", choices=("auto", "spin", "block"),
                    help="HIP host wait policy for synchronize (hipSetDeviceFlags before the "
                         "device is initialised): auto (HIP's default), spin, blocking")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearsals", type=int, default=20,
                    help="untimed runs of the timed region at the end of the warmup")
    ap.add_argument("--timed-repeats", type=int, default=1,
                    help="dev A/B: run the timed region this many more times after the measured "
                         "one and report their windows (`timed_repeats_ms`); value stays the first")
    ap.add_argument("--profile-run", action="store_true",
                    help="minimal run for rocprofv3 (no CPU baseline, no step roofline)")
    ap.add_argument("--stub-engine", action="store_true",
                    help="CPU stand-in engine + gloo (tests of the multi-rank glue; no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:  # no launcher: start the ranks
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    stub = args.stub_engine

    cpu = None
    if rank == 0 and world == 1 and not (args.no_cpu_baseline or args.profile_run or stub):
        cpu = cpu_baseline(args.cpu_budget, host_share_cores(), args.workload)

    import torch
    import torch.distributed as dist

    # one process per GPU over RCCL; on a box with fewer GPUs than ranks (rehearsal only) the
    # ranks share devices and fall back to gloo (RCCL refuses two ranks on one GPU)
    if stub:
        device, ndev = torch.device("cpu"), 0
    else:
        ndev = max(1, torch.cuda.device_count())
        device = torch.device("cuda", local_rank % ndev)
        if args.host_wait != "auto":  # before anything creates the device's context
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            assert hip.hipSetDevice(ctypes.c_int(device.index)) == 0
            flag = {"spin": 1, "block": 4}[args.host_wait]  # hipDeviceSchedule{Spin,BlockingSync}
            assert hip.hipSetDeviceFlags(ctypes.c_uint(flag)) == 0
        torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "gloo" if stub else os.environ.get("MEV_DIST_BACKEND",
                                                     "nccl" if ndev >= world else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    from mobile_env.sharding import gather_final, gather_obs, shard_seeds

    E = args.envs
    seeds = shard_seeds(1000, E, rank)  # rank r owns global envs [r*E, (r+1)*E)
    overrides = {k: int(v) for k, v in (kv.split("=", 1) for kv in args.engine)}
    if stub:
        from mobile_env.scenarios import registry
        sp = registry.spec(args.workload)
        env = StubEnv(E, sp["num_ues"], sp["num_bs"], seeds)
    else:
        import mobile_env
        env = mobile_env.make(args.workload, num_envs=E, device=device, seed=int(seeds[0]),
                              stream_split=2 if args.launch == "split" else 0,
                              fuse_steps=0 if args.launch == "fused" else -1, **overrides)
    eng = env.engine

    def sync():
        if not stub:
            torch.cuda.synchronize(device)
    U, B = env.num_ues, env.num_bs
    per_env_bs = eng.bs_per_env
    parts = eng.launch_parts
    env.reset()
    K = args.steps
    plan = chunk_plan(K, args.chunk)
    CHUNK = plan[0]
    fused = args.launch == "fused" and eng.fused_steps
    traj = eng.trajectory(CHUNK) if args.launch == "fused" else None
    stream = None if stub else torch.cuda.current_stream(device)

    launchers = {}

    def issue(n):  # fused: every step's outputs to its own trajectory row
        if n not in launchers:  # prebuilt ctypes arguments: one foreign call per launch
            launchers[n] = eng.launcher(n, traj)
        launchers[n]()

    class _Ev:
        def __init__(self):  # recorded once here: the HIP event exists before the timed region
            self.e = torch.cuda.Event(enable_timing=True)
            self.e.record(stream)

        def record(self):
            self.e.record(stream)

    class _WallEv:  # (stub engine: host clock)
        def __init__(self):
            self.t = time.perf_counter()

        def record(self):
            self.t = time.perf_counter()

        @property
        def e(self):
            return self

        def elapsed_time(self, other):
            return (other.t - self.t) * 1e3

    gathered = {}

    gbuf = None
    if world > 1:  # the final batch's send / receive buffers (5 B per env), allocated once
        gdev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        gbuf = (torch.empty(5 * E, dtype=torch.uint8, device=gdev),
                torch.empty((world, 5 * E), dtype=torch.uint8, device=gdev))

    def collective():  # the one collective: the final (reward, done) batch to every rank
        if traj is not None:  # the last step's row of the trajectory
            r, d = traj.reward[plan[-1] - 1], traj.done[plan[-1] - 1]
        else:
            r, d = eng.reward, eng.done
        gathered["rd"] = gather_final(r, d, packed=True, buf=gbuf)  # (unpacked after timing)

    def obs_last():
        return traj.obs[plan[-1] - 1] if traj is not None else eng.obs

    # warmup: W steps, then whole chunks until the floor time has passed (steady clock)
    warm = 0
    t_w = time.perf_counter()
    if args.warmup > 0:
        env.step()  # the Gym surface once
        warm = 1
        for n in chunk_plan(args.warmup - 1, CHUNK) if args.warmup > 1 else []:
            issue(n)
            warm += n
        sync()
        while time.perf_counter() - t_w < args.warmup_floor_s:
            for _ in range(16):
                issue(CHUNK)
                warm += CHUNK
            sync()
    sync()
    warm_gathers = None
    if world > 1:  # both collectives once, untimed: the timed one is not the process's first
        t0 = time.perf_counter()
        collective()
        sync()
        t1 = time.perf_counter()
        gather_obs(obs_last())
        sync()
        warm_gathers = {"final_ms": (t1 - t0) * 1e3, "obs_ms": (time.perf_counter() - t1) * 1e3}
        gathered.clear()

    for n in set(plan):  # every launch of the timed region prebuilt
        if n not in launchers:
            launchers[n] = eng.launcher(n, traj)
    barrier = dist.barrier if world > 1 else (lambda: None)
    # the last warmup piece: untimed rehearsals of the timed region itself (the same launches,
    # gather and synchronisation; --rehearsals, at most ~0.1 s of them), so that the measured
    # region is not the first run of its host code path and of its isolated-launch rhythm -- the
    # first run of a one-launch region measured ~7-9 us (4-5 %) slower than every later one in
    # the same process (tools/gpu_bench_driver.sh)
    t_r = time.perf_counter()
    for _ in range(args.rehearsals):
        timed_run(issue, plan, sync, barrier, collective if world > 1 else None)
        warm += sum(plan)
        if time.perf_counter() - t_r > 0.1:
            break
    elapsed, t_steps, t_gather, t_barrier = timed_run(issue, plan, sync, barrier,
                                                      collective if world > 1 else None)
    elapsed = max_over_ranks(elapsed, device)
    t_barrier = max_over_ranks(t_barrier, device)
    repeats = []
    for _ in range(max(0, args.timed_repeats - 1)):
        repeats.append(max_over_ranks(timed_run(issue, plan, sync, barrier,
                                                collective if world > 1 else None)[0], device) * 1e3)
    t_steps = max_over_ranks(t_steps, device)
    t_gather = max_over_ranks(t_gather, device) if t_gather is not None else None
    if "rd" in gathered:
        from mobile_env.sharding import unpack_final
        gathered["rd"] = unpack_final(gathered["rd"])

    # after the timed region: the north-star final obs batch to every rank (RCCL all-gather over
    # xGMI; obs of the last step), timed on its own (barrier + sync around, max over ranks)
    obs_gather = None
    if world > 1:
        ol = obs_last()
        barrier()
        sync()
        t0 = time.perf_counter()
        g_obs = gather_obs(ol)
        sync()
        ms = max_over_ranks((time.perf_counter() - t0) * 1e3, device)
        nbytes = ol.numel() * ol.element_size()
        obs_gather = {"ms": ms, "bytes_per_rank": nbytes, "gathered_bytes": world * nbytes,
                      "shape": list(g_obs.shape), "backend": dist.get_backend(),
                      "bus_GBps": (world - 1) * nbytes / (ms * 1e-3) / 1e9,
                      "checksum": float(g_obs[..., 0].double().sum())}
        del g_obs
    # the launch shape's duration, measured after the timed region with an event pair around
    # each launch: isolated launches when the region was one launch (the driver's shape), else
    # back to back like the region's
    reps = max(3, min(30, int(0.05 / max(CHUNK * 8e-6, 1e-6))))
    if args.profile_run:  # (rocprofv3 runs: the timed region's launches stay the trace's last)
        reps = 0
        chunk_ms = chunk_ms_med = elapsed * 1e3 / len(plan)
    else:
        chunk_ms, chunk_ms_med = launch_timing(issue, CHUNK, reps, sync,
                                               _WallEv if stub else _Ev, isolated=len(plan) == 1)

    step_roof = None
    if rank == 0 and fused and not args.profile_run and args.step_launches > 0 and not stub:
        # the Gym step() launch (mev_step(1)), canonical bytes, timed after the timed region:
        # back-to-back launches between one event pair (an event pair around every launch
        # adds ~2 us of marker overhead to a 19 us kernel), in 10 groups for the spread
        step1 = eng.launcher(1)
        for _ in range(20):
            step1()
        ngrp = 10
        per = max(1, args.step_launches // ngrp)
        evs = [(_Ev(), _Ev()) for _ in range(ngrp)]
        for a, b in evs:
            a.record()
            for _ in range(per):
                step1()
            b.record()
        torch.cuda.synchronize(device)
        ms = sorted(a.e.elapsed_time(b.e) / per for a, b in evs)
        avg = sum(ms) / len(ms)
        # (the committed profiles are of the default launch shapes: with an --engine override
        # another kernel instance runs, and no profile of it is attached)
        tr1, rp1 = load_profile(args.workload, E, "single") if not overrides else (None, None)
        step_roof = roofline(E * algorithmic_bytes_per_env_step(U, per_env_bs, B), avg, tr1)
        step_roof.update({"median_launch_ms": ms[len(ms) // 2], "launches": per * ngrp,
                          "rocprof_launch_ms": rp1,
                          "env_steps_per_s": E / (avg * 1e-3),
                          "basis": "SURVEY.md 8d canonical bytes per env-step x E, one-step "
                                   "launch (make().step(), mev_step(1))",
                          "frac_basis": "canonical: frac counts SURVEY 8d's bytes, which the "
                                        "launch does not all move (compact uint8 / int16 "
                                        "UE state); "
                                        "traffic_frac = the PMC bytes it moves / peak"})

    if rank == 0:
        value = world * E * K / elapsed
        spl = CHUNK if fused else 1  # steps per launch
        canon_bytes = E * spl * algorithmic_bytes_per_env_step(U, per_env_bs, B)
        algo_bytes = (E * algorithmic_bytes_rollout(U, per_env_bs, B, spl) if fused
                      else canon_bytes)
        launch_ms = chunk_ms if fused else chunk_ms / CHUNK
        traffic, rocprof_ms = (load_profile(args.workload, E, args.launch, CHUNK) if not overrides
                               else (None, None))
        roof = roofline(algo_bytes, launch_ms, traffic)
        roof.update({
            "canonical_bytes_per_env_step": algorithmic_bytes_per_env_step(U, per_env_bs, B),
            "canonical_equiv_achieved": canon_bytes / (launch_ms * 1e-3) / 1e9,
            "canonical_equiv_frac": canon_bytes / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "steps_per_launch": spl,
            "launch_ms_median": chunk_ms_med if fused else chunk_ms_med / CHUNK,
            "launch_ms_basis": (f"HIP events around {reps} {'isolated' if len(plan) == 1 else 'back-to-back'} "
                                f"launches of the timed shape, run after the timed region"),
            "rocprof_launch_ms": rocprof_ms,
            "launch_shape": (
                f"fused rollout: {spl} steps per launch, env state in registers between "
                f"them, every step's outputs to its own trajectory row" if fused else
                f"{parts} halves per step on {parts} HIP streams" if parts > 1
                else "one kernel per step")})
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "warmup_executed": warm,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype_string(getattr(eng, "state_bytes_per_ue", 4)),
            "host_wait": args.host_wait,
            "data": "synthetic (seeded PCG64 streams, build-defined BS layout)",
            "config": {"workload": args.workload, "envs_per_gpu": E, "global_envs": world * E,
                       "num_ues": U, "num_bs": B, "per_env_layouts": bool(per_env_bs),
                       "launches": len(plan), "steps_per_launch": CHUNK,
                       "parallelism": f"env-sharded x{world}, no data-path collective"},
            "roofline": roof,
            "roofline_step": step_roof,
            "cpu_baseline": cpu,
            **({"timed_repeats_ms": repeats} if repeats else {}),
            "distributed": ({"world_size_seen": dist.get_world_size(),
                             "backend": dist.get_backend(),
                             "final_gather_ms": t_gather * 1e3,
                             "trailing_barrier_ms": t_barrier * 1e3,
                             "window": "max over ranks of (end of the final gather - t0); the "
                                       "trailing barrier is outside it (trailing_barrier_ms)",
                             "final_gather_share": t_gather / elapsed,
                             "value_steps_only": world * E * K / t_steps,
                             "warmup_gathers": warm_gathers,
                             "final_batch": {"shape": list(gathered["rd"].shape),
                                             "reward_sum": float(gathered["rd"][:, 0].double().sum()),
                                             "done_sum": float(gathered["rd"][:, 1].double().sum())},
                             "obs_gather": obs_gather}
                            if world > 1 else None),
        }
        if stub:
            out["data"] = "STUB ENGINE (CPU stand-in, glue test only; not a measurement)"
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
