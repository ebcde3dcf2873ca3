"""GPU parity of the kernels the BASELINE.json configs actually ship, against the oracle directly.

The launch the engine picks depends on the batch size, the launch length and the scenario's
parameters (scenario-constant instances, tie-free share, compact state, pipelined loop), so a
kernel instance can be selected by a registered scenario at its own batch size and nowhere else.
These tests run ``make(<registered id>, num_envs=<BASELINE size>)`` with its automatic choice,
assert which kernel ran (``StepEngine.last_launch_kind``, mev_last_launch_kind), and compare
every step's outputs with the oracle (oracle/vec.py, pinned to the reference's fixtures):

* BASELINE configs[1]: mobile-medium-central-v0 at 4,096 envs -> the software-pipelined
  one-group rollout, U = 15 / velocity 1.5 scenario constants, tie-free share -- every env,
  45 steps (two episode resets); and the same batch forced onto the pipelined kernel with
  32-lane segments and onto the one-group packed kernel;
* BASELINE configs[2] (the bench): mobile-large-central-v0 at 65,536 envs -> the two-group
  scenario kernel; every 16th env (4,096 of them) against the oracle run on those envs' seeds
  -- envs are independent, so the subset comparison is exact;
* the Gym step() launch of both (mev_step(1), one launch per step);
* the build-defined mobile-large-mixed-v0 (heterogeneous classes) at 65,536 envs -> the
  two-group kernel on the lds_mode 6 tables, every 16th env against the oracle;
* BASELINE configs[4]: mobile-custom-128x1024-v0 at 1,024 envs (its per-GPU batch of 8,192 over
  8 GPUs) -> the lean scenario-constant block kernel (k_steps_block, instance 4: f32 utility,
  fixed-point reward, station-culling records built in LDS), every 16th env against the oracle
  on that env's own 128-station layout; and its Gym step() launch (the two-UEs-per-lane block
  instance with the HBM culling records).

Bars (north_star): positions, serving, done bit-exact; float32 rate / utility / reward within
1e-5 relative with atol 0 (helpers.assert_step_vs_oracle).
Reference: base.py:230-296 (step), movement.py:42-62 (RandomWaypoint), channels.py:133-146.
"""
import numpy as np
import pytest

from helpers import assert_rollout_vs_oracle, assert_step_vs_oracle

pytestmark = pytest.mark.gpu


def _oracle(size, seeds, vel=1.5):
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS[size]
    return OracleBatch(OracleParams(velocity=vel), L["bs"], L["num_ues"], np.asarray(seeds))


@pytest.mark.parametrize("two_groups,kind", [(0, "lds2_pipelined"), (4, "lds2_pipelined_seg32"),
                                             (-1, "packed_fused")])
def test_medium_4096_shipped_rollout_vs_oracle(two_groups, kind):
    """BASELINE configs[1] with the kernel make() picks for it (and the packed fallback): one
    45-step rollout of every one of the 4,096 envs against the oracle, step by step."""
    import mobile_env
    E, n = 4096, 45
    env = mobile_env.make("mobile-medium-central-v0", num_envs=E, device="cuda:0", seed=5,
                          two_groups=two_groups)
    env.reset()
    eng = env.engine
    assert eng.rollout_instance == 1 and eng.share_tie_free and eng.state_bytes_per_ue == 4
    tr = eng.rollout(n)
    assert eng.last_launch_kind == kind
    o = assert_rollout_vs_oracle(tr, _oracle("medium", env.seeds.numpy()), n)
    np.testing.assert_array_equal(eng.ue_xy.cpu().numpy(), o["xy"])
    env.close()


def test_large_65536_bench_rollout_strided_vs_oracle():
    """The bench's own launch (BASELINE configs[2]: 65,536 mobile-large envs, the two-group
    scenario-constant kernel): one 45-step rollout, every 16th env against the oracle."""
    import mobile_env
    import torch
    E, n, stride = 65536, 45, 16
    env = mobile_env.make("mobile-large-central-v0", num_envs=E, device="cuda:0", seed=1000)
    env.reset()
    eng = env.engine
    assert eng.rollout_instance == 2 and eng.share_tie_free
    tr = eng.rollout(n)
    assert eng.last_launch_kind == "lds2_two_groups"
    idx = np.arange(0, E, stride)
    ob = _oracle("large", env.seeds.numpy()[idx])
    o = assert_rollout_vs_oracle(tr, ob, n, env_idx=idx)
    ti = torch.as_tensor(idx, device=eng.device)
    np.testing.assert_array_equal(eng.ue_xy.index_select(0, ti).cpu().numpy(), o["xy"])
    del tr
    env.close()
    torch.cuda.empty_cache()


def test_large_bench_short_and_long_launch_instances_agree():
    """The two-group scenario kernel comes in two instances by launch length (lds2_step RT1: the
    one-compare reward test for launches of fewer than 64 steps -- the driver's 20-step shape --
    and the original test for longer ones): a 70-step launch and a 20-step launch of the same
    65,536 envs give the same first 20 rows bit for bit, and the long launch's 70 rows match the
    oracle on every 16th env."""
    import mobile_env
    import torch
    E, stride = 65536, 16
    rows = {}
    for n in (20, 70):
        env = mobile_env.make("mobile-large-central-v0", num_envs=E, device="cuda:0", seed=4242)
        env.reset()
        eng = env.engine
        tr = eng.rollout(n)
        assert eng.last_launch_kind == "lds2_two_groups"
        rows[n] = [x[:20].cpu().numpy() for x in (tr.obs, tr.serving, tr.reward, tr.done)]
        if n == 70:
            idx = np.arange(0, E, stride)
            assert_rollout_vs_oracle(tr, _oracle("large", env.seeds.numpy()[idx]), n, env_idx=idx)
        del tr
        env.close()
        torch.cuda.empty_cache()
    for a, b, name in zip(rows[20], rows[70], ("obs", "serving", "reward", "done")):
        np.testing.assert_array_equal(a, b, err_msg=name)


@pytest.mark.parametrize("env_id,size,E,stride", [("mobile-medium-central-v0", "medium", 4096, 1),
                                                  ("mobile-large-central-v0", "large", 65536, 16)])
def test_gym_step_shipped_vs_oracle(env_id, size, E, stride):
    """The Gym surface (VectorMobileEnv.step -> mev_step(1)) at the BASELINE batch sizes: 23
    one-step launches (crossing the episode reset), checked against the oracle every step."""
    import mobile_env
    import torch
    env = mobile_env.make(env_id, num_envs=E, device="cuda:0", seed=77)
    env.reset()
    idx = np.arange(0, E, stride)
    ti = torch.as_tensor(idx, device=env.device)
    ob = _oracle(size, env.seeds.numpy()[idx])
    U = env.num_ues
    for s in range(23):
        obs, reward, term, trunc, info = env.step()
        assert env.engine.last_launch_kind == "packed_step"
        o = ob.step()
        obs = obs.view(E, U, 4).index_select(0, ti).cpu().numpy()
        assert_step_vs_oracle(o, obs, info["serving"].index_select(0, ti).cpu().numpy(),
                              reward.index_select(0, ti).cpu().numpy(),
                              trunc.index_select(0, ti).cpu().numpy(), where=f"step {s}")
        assert not bool(term.any())
    env.close()


def test_mixed_65536_rollout_strided_vs_oracle():
    """mobile-large-mixed-v0 at the bench's batch (three station and three UE classes on the
    large layout; entities.py:7-45): the heterogeneous two-group LDS kernel, one 45-step rollout,
    every 16th env against the oracle with the same classes."""
    import mobile_env
    import torch
    from mobile_env.scenarios.registry import LAYOUTS, spec
    from oracle.vec import OracleBatch, OracleParams
    E, n, stride = 65536, 45, 16
    env = mobile_env.make("mobile-large-mixed-v0", num_envs=E, device="cuda:0", seed=3000)
    env.reset()
    eng = env.engine
    tr = eng.rollout(n)
    assert eng.last_launch_kind == "lds2_het"
    c = spec("mobile-large-mixed-v0")["classes"]
    idx = np.arange(0, E, stride)
    L = LAYOUTS["large"]
    ob = OracleBatch(OracleParams(bs_classes=c["bs_classes"], ue_classes=c["ue_classes"],
                                  bs_class=c["bs_class"], ue_class=c["ue_class"]),
                     L["bs"], L["num_ues"], env.seeds.numpy()[idx])
    o = assert_rollout_vs_oracle(tr, ob, n, env_idx=idx)
    ti = torch.as_tensor(idx, device=eng.device)
    np.testing.assert_array_equal(eng.ue_xy.index_select(0, ti).cpu().numpy(), o["xy"])
    del tr
    env.close()
    torch.cuda.empty_cache()


def _custom_oracle(env, idx):
    from mobile_env.scenarios.registry import spec
    from oracle.vec import OracleBatch, OracleParams
    vel = float(spec("mobile-custom-128x1024-v0")["velocity"])
    bs = env.engine.bs_xy.cpu().numpy()[idx]  # [E', 128, 2]: each env's own layout
    cnt = env.engine.bs_count.cpu().numpy()[idx] if env.engine.bs_count is not None else None
    return OracleBatch(OracleParams(velocity=vel), bs, env.num_ues, env.seeds.numpy()[idx],
                       bs_count=cnt)


def test_custom_1024_shipped_rollout_vs_oracle():
    """BASELINE configs[4] (128 BS x 1,024 UE, velocity 10, per-env layouts drawn from each env's
    seed) at 1,024 envs with make()'s own choice -- the lean scenario-constant block rollout: one
    45-step launch (two episode resets; station culling active, >= 32 steps), every 16th env
    against the oracle step by step, then the final positions."""
    import mobile_env
    import torch
    E, n, stride = 1024, 45, 16
    env = mobile_env.make("mobile-custom-128x1024-v0", num_envs=E, device="cuda:0", seed=600)
    env.reset()
    eng = env.engine
    assert eng.rollout_instance == 4 and eng.bs_per_env
    tr = eng.rollout(n)
    assert eng.last_launch_kind == "block"
    idx = np.arange(0, E, stride)
    o = assert_rollout_vs_oracle(tr, _custom_oracle(env, idx), n, env_idx=idx)
    ti = torch.as_tensor(idx, device=eng.device)
    np.testing.assert_array_equal(eng.ue_xy.index_select(0, ti).cpu().numpy(), o["xy"])
    del tr
    env.close()
    torch.cuda.empty_cache()


def test_custom_1024_gym_step_vs_oracle():
    """The Gym surface of BASELINE configs[4] at 1,024 envs: 22 one-step launches (the reset
    inside), every 16th env against the oracle each step."""
    import mobile_env
    import torch
    E, stride = 1024, 16
    env = mobile_env.make("mobile-custom-128x1024-v0", num_envs=E, device="cuda:0", seed=700)
    env.reset()
    idx = np.arange(0, E, stride)
    ti = torch.as_tensor(idx, device=env.device)
    ob = _custom_oracle(env, idx)
    U = env.num_ues
    for s in range(22):
        obs, reward, term, trunc, info = env.step()
        assert env.engine.last_launch_kind == "block"
        o = ob.step()
        obs = obs.view(E, U, 4).index_select(0, ti).cpu().numpy()
        assert_step_vs_oracle(o, obs, info["serving"].index_select(0, ti).cpu().numpy(),
                              reward.index_select(0, ti).cpu().numpy(),
                              trunc.index_select(0, ti).cpu().numpy(), where=f"step {s}")
    env.close()
