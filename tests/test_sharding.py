"""Multi-process (world_size 2, gloo on CPU) test of the N>1 path: env shards partition the
global batch by seed, and the single final all-gather returns every rank's (reward, done)
in rank order -- equal to one unsharded run over all envs. The per-rank step is the oracle
(this test covers the host-side sharding/collective logic; the kernel is covered by the GPU
parity tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

E_PER_RANK = 6
STEPS = 23  # crosses the episode reset
BASE_SEED = 1000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mobile-env-gan_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mobile_env.scenarios.registry import LAYOUTS
    from mobile_env.sharding import gather_final, shard_seeds
    from oracle.vec import OracleBatch, OracleParams
    lay = LAYOUTS["small"]
    seeds = shard_seeds(BASE_SEED, E_PER_RANK, rank)
    ob = OracleBatch(OracleParams(velocity=10.0), lay["bs"], lay["num_ues"], seeds)
    for _ in range(STEPS):
        o = ob.step()
    reward = torch.tensor(o["metrics"][:, 2], dtype=torch.float32)
    done = torch.tensor(o["done"].astype(np.uint8))
    g = gather_final(reward, done)
    if rank == 0:
        torch.save(g, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_unsharded(tmp_path):
    world = 2
    out = str(tmp_path / "gathered.pt")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g = torch.load(out, weights_only=True)
    assert tuple(g.shape) == (world, 2, E_PER_RANK)

    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    lay = LAYOUTS["small"]
    ob = OracleBatch(OracleParams(velocity=10.0), lay["bs"], lay["num_ues"],
                     BASE_SEED + np.arange(world * E_PER_RANK))
    for _ in range(STEPS):
        o = ob.step()
    want_r = o["metrics"][:, 2].astype(np.float32).reshape(world, E_PER_RANK)
    want_d = o["done"].astype(np.float32).reshape(world, E_PER_RANK)
    np.testing.assert_array_equal(g[:, 0].numpy(), want_r)
    np.testing.assert_array_equal(g[:, 1].numpy(), want_d)


def test_shard_ranges_partition():
    from mobile_env.sharding import shard_envs, shard_seeds
    world, E = 8, 65536
    cover = np.concatenate([shard_seeds(7, E, r) for r in range(world)])
    np.testing.assert_array_equal(cover, 7 + np.arange(world * E))
    assert shard_envs(E, 3) == (3 * E, 4 * E)


def _bench_worker(rank, world, port, out_path):
    """bench.py's N > 1 glue on CPU (gloo): per-rank seeds, the timed region with the chunk
    plan, the final (reward, done) all-gather and the MAX-over-ranks time. The engine is a
    stand-in that writes its rank's (reward, done) rows and takes rank-dependent time."""
    import importlib.util
    import sys
    import time as _t
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mobile-env-gan_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from mobile_env.sharding import gather_final, shard_seeds
    E, K, chunk = 5, 23, 10
    seeds = shard_seeds(1000, E, rank)
    plan = bench.chunk_plan(K, chunk)
    reward = torch.zeros(E)
    done = torch.zeros(E, dtype=torch.uint8)
    issued = []

    def issue(n):
        issued.append(n)
        _t.sleep(0.01 * (rank + 1) * n / chunk)
        reward.copy_(torch.as_tensor(seeds, dtype=torch.float32) + sum(issued))
        done.fill_(int(sum(issued) % 20 == 0))

    got = {}

    def collective():
        got["g"] = gather_final(reward, done)

    calls = []

    def slow_trailing_barrier():  # the region's second barrier call is the trailing one
        calls.append(1)
        if len(calls) == 2:
            _t.sleep(0.3)
        dist.barrier()

    elapsed, t_steps, t_coll, t_bar = bench.timed_run(issue, plan, lambda: None,
                                                      slow_trailing_barrier, collective)
    assert 0 < t_steps <= elapsed and 0 <= t_coll <= elapsed - t_steps + 1e-9
    # the window ends at the gather's completion: the 0.3 s trailing barrier is not in it (the
    # steps take 0.023 / 0.046 s per rank), and it is reported on its own
    assert len(calls) == 2 and t_bar >= 0.3 and elapsed < 0.25
    mine = elapsed
    elapsed = bench.max_over_ranks(elapsed)
    every = [None] * world
    dist.all_gather_object(every, mine)
    if rank == 0:
        torch.save({"plan": plan, "issued": issued, "elapsed": elapsed, "every": every,
                    "g": got["g"], "value": world * E * K / elapsed}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_multi_rank_glue(tmp_path):
    world = 2
    out = str(tmp_path / "bench.pt")
    mp.spawn(_bench_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    r = torch.load(out, weights_only=False)
    assert r["plan"] == [10, 10, 3] and r["issued"] == r["plan"]  # exactly K = 23 steps
    assert r["elapsed"] == max(r["every"])
    g = r["g"]  # [world, 2, E]: rank r's rows are its own envs (seeds 1000 + r*E + i) + 23
    want = (1000 + np.arange(world * 5)).reshape(world, 5) + 23
    np.testing.assert_array_equal(g[:, 0].numpy(), want.astype(np.float32))
    np.testing.assert_array_equal(g[:, 1].numpy(), np.zeros((world, 5), np.float32))
    assert r["value"] == world * 5 * 23 / r["elapsed"]


def test_bench_spawns_its_own_ranks():
    """`python bench.py --gpus 2` as a plain command (no launcher, WORLD_SIZE unset) starts its
    two ranks itself; with the CPU stand-in engine (gloo) the line reports n_gpus 2, the world
    size the ranks saw, exactly K steps, and a final (reward, done) batch / obs gather holding
    every rank's envs: after W + K steps env g's reward is its seed 1000 + g plus the steps."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    E, K, W = 5, 23, 4
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--stub-engine", "--steps", str(K), "--warmup", str(W), "--chunk", "10",
                        "--envs", str(E), "--warmup-floor-s", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == K and out["config"]["global_envs"] == 2 * E
    dd = out["distributed"]
    assert dd["world_size_seen"] == 2 and dd["backend"] == "gloo"
    # the warmup's W steps plus its untimed rehearsals of the timed region (whole plans of K)
    assert out["warmup_executed"] >= W and (out["warmup_executed"] - W) % K == 0
    steps = out["warmup_executed"] + K
    seeds = 1000 + np.arange(2 * E)
    assert dd["final_batch"]["shape"] == [2, 2, E]
    assert dd["final_batch"]["reward_sum"] == float((seeds + steps).sum())
    assert dd["final_batch"]["done_sum"] == float(2 * E * (steps % 20 == 0))
    og = dd["obs_gather"]
    U = 30  # mobile-large-central-v0
    assert og["shape"] == [2, E, U, 4] and og["bytes_per_rank"] == E * U * 16
    assert og["checksum"] == float(seeds.sum() * U)
    assert out["value"] == pytest.approx(2 * E * K / (out["ms_per_step"] * K * 1e-3))
    # both collectives ran once in the untimed warmup (the timed gather is not the first), and
    # the timed gather's own time and the steps-only rate are reported
    wg = dd["warmup_gathers"]
    assert wg is not None and wg["final_ms"] > 0 and wg["obs_ms"] > 0
    assert 0 < dd["final_gather_ms"] <= out["ms_per_step"] * K
    assert dd["trailing_barrier_ms"] >= 0 and "trailing barrier is outside" in dd["window"]
    assert 0 < dd["final_gather_share"] < 1
    assert dd["value_steps_only"] >= out["value"]
    rf = out["roofline"]
    assert "timed region" in rf["launch_ms_basis"] and rf["launch_ms"] > 0
    assert "uint8x4" in out["dtype"] and "fixed-point reward" in out["dtype"]
