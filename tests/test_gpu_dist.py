"""The N > 1 path with the GPU engine (one process per rank, torch.distributed), on one GPU:

* two ranks (gloo: RCCL does not place two ranks on one GPU), each the GPU engine on cuda:0 with
  its env shard (sharding.shard_seeds), one 20-step rollout, the final (reward, done) batch and
  the obs batch all-gathered -- equal, byte for byte, to one unsharded engine over all envs;
* one rank over RCCL (backend "nccl", init_process_group(device_id=...)): the collectives'
  device branch (all_gather_into_tensor of the packed uint8 batch and of the obs) -- the code the
  8-GPU bench runs -- against the rank's own buffers.

The ranks run as child processes (torch.distributed.run), the comparison in this process.
Reference: base.py:230-296 (envs are independent: sharding never exchanges state).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E_PER_RANK, STEPS, BASE = 2048, 20, 1000

RANK_SCRIPT = r'''
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "mobile-env-gan_amd")]
import numpy as np, torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
backend = sys.argv[1]
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
if backend == "nccl":
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
else:
    dist.init_process_group("gloo", rank=rank, world_size=world)
import mobile_env
from mobile_env.sharding import gather_final, gather_obs, shard_seeds, unpack_final
seeds = shard_seeds({base}, {e}, rank)
env = mobile_env.make("mobile-large-central-v0", num_envs={e}, device="cuda:0", seed=int(seeds[0]))
env.reset()
tr = env.engine.rollout({steps})
g = unpack_final(gather_final(tr.reward[{steps} - 1], tr.done[{steps} - 1], packed=True))
go = gather_obs(tr.obs[{steps} - 1])
torch.cuda.synchronize()
if rank == 0:
    np.savez(sys.argv[2], final=g.cpu().numpy(), obs=go.cpu().numpy(),
             own_r=tr.reward[{steps} - 1].cpu().numpy(), own_obs=tr.obs[{steps} - 1].cpu().numpy())
dist.barrier()
dist.destroy_process_group()
env.close()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks(tmp_path, world, backend):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(root=ROOT, base=BASE, e=E_PER_RANK, steps=STEPS))
    out = tmp_path / f"out_{backend}_{world}.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script), backend,
           str(out)]
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return np.load(out)


def test_two_ranks_gpu_engine_equal_unsharded(tmp_path):
    import mobile_env
    d = _ranks(tmp_path, 2, "gloo")
    env = mobile_env.make("mobile-large-central-v0", num_envs=2 * E_PER_RANK, device="cuda:0",
                          seed=BASE)
    env.reset()
    tr = env.engine.rollout(STEPS)
    r = tr.reward[STEPS - 1].cpu().numpy().reshape(2, E_PER_RANK)
    dn = tr.done[STEPS - 1].cpu().numpy().reshape(2, E_PER_RANK)
    obs = tr.obs[STEPS - 1].cpu().numpy()
    env.close()
    np.testing.assert_array_equal(d["final"][:, 0], r)
    np.testing.assert_array_equal(d["final"][:, 1], dn.astype(np.float32))
    np.testing.assert_array_equal(d["obs"].reshape(obs.shape), obs)


def test_single_rank_rccl_collectives(tmp_path):
    d = _ranks(tmp_path, 1, "nccl")
    np.testing.assert_array_equal(d["final"][0, 0], d["own_r"])
    np.testing.assert_array_equal(d["obs"][0], d["own_obs"])
