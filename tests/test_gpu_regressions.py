"""GPU regression tests for defects found in review.

* per-UE velocities with a single channel class (mev_params.ue_velocity set, no class arrays,
  one rate table without offsets): mev_create used to dereference the absent rate-table
  offsets; built through EngineParams and through the facade's lowering (UserEquipment objects
  that differ only in velocity, entities.py:33-45), checked against the oracle;
* xcd_remap rotations 2..8 on grids that are not a multiple of 8 workgroups: every env range
  must be covered exactly once (block_slot is a bijection), so every setting gives the
  outputs of the default order, for the one-step kernel and the fused rollouts;
* mev_update_stations no longer blocks the host: a layout change followed by a rollout still
  selects the kernel that depends on the layout's distance set (|D|, read back without a
  stream sync) and gives the oracle's results.
Reference: movement.py:42-62 (per-UE velocity), base.py:230-296.
"""
import numpy as np
import pytest

from helpers import assert_rollout_vs_oracle, assert_step_vs_oracle

pytestmark = pytest.mark.gpu


def _velocity_users(U):
    return [1.0 + 0.75 * (u % 7) for u in range(U)]


@pytest.mark.parametrize("via", ["params", "lowering"])
def test_per_ue_velocity_single_class_vs_oracle(via):
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS["large"]
    U, B, E = L["num_ues"], len(L["bs"]), 300
    vel = _velocity_users(U)
    if via == "params":
        p = EngineParams(num_envs=E, num_ues=U, num_bs=B, ue_velocity=vel)
    else:
        from mobile_env.core import lowering
        from mobile_env.core.base import MComCore
        from mobile_env.core.entities import BaseStation, UserEquipment
        base = MComCore.default_config()
        stations = [BaseStation(i, (int(x), int(y)), **base["bs"])
                    for i, (x, y) in enumerate(L["bs"])]
        users = [UserEquipment(i, **dict(base["ue"], velocity=vel[i])) for i in range(U)]
        core = MComCore(stations, users, config={})
        p = lowering.lower(num_envs=E, stations=stations, users=users,
                           arrival=core.arrivalModel, channel=core.channelModel,
                           scheduler=core.schedulerModel, movement=core.movementModel,
                           utility=core.utilityModel, ep_max_time=core.EP_MAX_TIME,
                           first_step_active=True)
        assert p.ue_velocity is not None and not p.heterogeneous
    seeds = 4242 + np.arange(E)
    eng = StepEngine(p, L["bs"], seeds, device="cuda")
    ob = OracleBatch(OracleParams(ue_velocity=vel), L["bs"], U, seeds)
    for s in range(23):  # one-step launches across the episode reset
        eng.step()
        o = ob.step()
        assert_step_vs_oracle(o, eng.obs.cpu().numpy(), eng.serving.cpu().numpy(),
                              eng.reward.cpu().numpy(), eng.done.cpu().numpy(), where=f"step {s}")
    tr = eng.rollout(25)  # and a fused rollout from there
    assert_rollout_vs_oracle(tr, ob, 25)
    eng.close()


@pytest.mark.parametrize("size,E,nsteps", [("large", 8 * 13 + 3, 1), ("large", 3001, 45),
                                           ("medium", 4096 + 40, 45), ("large", 70001, 20)])
def test_xcd_remap_rotations_identical(size, E, nsteps):
    """xcd_remap -1 (dispatch order), 1 (default), 2..8 (rotated ranges) on grids that 8 does
    not divide: every step's outputs and the final state bit-identical."""
    import torch
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    L = LAYOUTS[size]
    first = None
    kinds = set()
    for remap in (-1, 1, 2, 3, 4, 5, 6, 7, 8):
        p = EngineParams(num_envs=E, num_ues=L["num_ues"], num_bs=len(L["bs"]), xcd_remap=remap)
        eng = StepEngine(p, L["bs"], 17 + np.arange(E), device="cuda")
        if nsteps == 1:
            rows = []
            for _ in range(22):
                eng.step()
                rows += [eng.obs.clone(), eng.serving.clone(), eng.reward.clone(), eng.done.clone()]
        else:
            tr = eng.rollout(nsteps)
            rows = [tr.obs, tr.serving, tr.reward, tr.done]
        kinds.add(eng.last_launch_kind)
        torch.cuda.synchronize()
        run = [x.cpu() for x in rows] + [x.cpu().clone() for x in (eng.ue_state, eng.t)]
        eng.close()
        if first is None:
            first = run
        else:
            for a, b in zip(first, run):
                assert torch.equal(a, b), f"xcd_remap={remap}"
    assert len(kinds) == 1


def test_layout_change_then_pipelined_rollout_vs_oracle():
    """A shared layout changed between rollouts (mev_update_stations, no host sync): the
    pipelined kernel's choice reads the new layout's |D| and the outputs follow the new
    layout (oracle on the new layout, from the engine's state at the change)."""
    import torch
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS["medium"]
    U, B, E = L["num_ues"], len(L["bs"]), 512
    seeds = 9 + np.arange(E)
    eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B), L["bs"], seeds,
                     device="cuda")
    eng.rollout(20)  # one whole episode on the registered layout
    assert eng.last_launch_kind == "lds2_pipelined"
    new_bs = (np.asarray(L["bs"]) + 7) % 200
    eng.set_bs_layout(torch.as_tensor(new_bs, dtype=torch.int32))
    tr = eng.rollout(45)  # the next episodes: lazy reset, then the new layout throughout
    assert eng.last_launch_kind == "lds2_pipelined"  # (|D| of the shifted layout <= 4,094)
    ob = OracleBatch(OracleParams(), new_bs.tolist(), U, seeds)
    assert_rollout_vs_oracle(tr, ob, 45)
    # every station in the map's corner: the serving distances run over every sum of two squares
    # within reach (|D| = 5,101 > 4,094, past the mode-3 ranks) -- the read-back |D| of THIS
    # layout must reach the choice: not the pipelined kernel, and the oracle's results
    far_bs = np.zeros((B, 2), dtype=np.int64)
    eng.set_bs_layout(torch.as_tensor(far_bs, dtype=torch.int32))
    tr = eng.rollout(25)  # (mid-episode: the new layout from the next step on, like the oracle's)
    assert eng.last_launch_kind == "packed_fused"
    ob.bs_xy[:] = far_bs  # (the same oracle envs continue on the new layout)
    assert_rollout_vs_oracle(tr, ob, 25)
    eng.close()


def _exact_case(case):
    """(engine params, layout, oracle params, expected launch kind) of a reward_exact case."""
    from mobile_env.core.engine import EngineParams
    from mobile_env.scenarios.registry import LAYOUTS, spec
    from oracle.vec import OracleParams
    if case == "mixed":
        c = spec("mobile-large-mixed-v0")["classes"]
        L = LAYOUTS["large"]
        kw = dict(bs_classes=c["bs_classes"], ue_classes=c["ue_classes"], bs_class=c["bs_class"],
                  ue_class=c["ue_class"])
        return (dict(num_ues=L["num_ues"], num_bs=len(L["bs"]), **kw), L["bs"], OracleParams(**kw),
                2000, "lds2_het")
    if case == "block":
        rng = np.random.default_rng(3)
        bs = rng.integers(0, 200, size=(40, 2)).astype(np.int32)
        return dict(num_ues=100, num_bs=40, velocity=4.0), bs, OracleParams(velocity=4.0), 64, "block"
    size, vel, E, kind = {"two": ("large", 1.5, 16500, "lds2_two_groups"),
                          "pipe30": ("large", 1.5, 512, "lds2_pipelined"),
                          "pipe15": ("medium", 1.5, 512, "lds2_pipelined"),
                          "packed": ("small", 1.5, 512, "packed_fused"),
                          "generic": ("large", 10.0, 512, "packed_fused")}[case]
    L = LAYOUTS[size]
    return (dict(num_ues=L["num_ues"], num_bs=len(L["bs"]), velocity=vel), L["bs"],
            OracleParams(velocity=vel), E, kind)


@pytest.mark.parametrize("case", ["two", "pipe30", "pipe15", "packed", "generic", "mixed", "block"])
def test_reward_exact_every_kernel_vs_oracle(case):
    """reward_exact = 1 sends every env-step's reward through the exact path that the lean
    kernels otherwise take only where the float32 sum could miss 1e-5 relative (reward_risky:
    mean utilities near zero) -- the two-group step's in-step path, the pipelined loop's flush,
    the packed kernels' leaders, the block kernel's row finish, the heterogeneous tables: 25
    rollout steps (a reset inside) and 3 one-step launches, the rewards within one float32 ulp
    of the oracle's float64 mean (atol 0), every other output as the oracle's."""
    from mobile_env.core.engine import EngineParams, StepEngine
    from oracle.vec import OracleBatch
    kw, bs, op, E, kind = _exact_case(case)
    seeds = 4242 + 13 * np.arange(E)
    eng = StepEngine(EngineParams(num_envs=E, reward_exact=1, **kw), bs, seeds, device="cuda")
    n = 25
    tr = eng.rollout(n)
    assert eng.last_launch_kind == kind
    ob = OracleBatch(op, bs, kw["num_ues"], seeds)
    for s in range(n):
        o = ob.step()
        np.testing.assert_array_equal(tr.serving[s].cpu().numpy(), o["serving"], err_msg=f"step {s}")
        np.testing.assert_allclose(tr.reward[s].cpu().numpy(), o["metrics"][:, 2].astype(np.float32),
                                   rtol=1.2e-7, atol=0, err_msg=f"reward step {s}")
    for s in range(3):
        eng.step()
        o = ob.step()
        np.testing.assert_allclose(eng.reward.cpu().numpy(), o["metrics"][:, 2].astype(np.float32),
                                   rtol=1.2e-7, atol=0, err_msg=f"one-step reward {s}")
    eng.close()


def _u_err(lower, upper, w1, w2, w3):
    """KParams::u_err as the host computes it (mev_step.hip, mev_create's utility section)."""
    import math
    A = abs(w1 * math.log(2.0) / math.log(w3) * (2.0 / (upper - lower)))
    r_sat = math.exp(upper * math.log(w3) / w1) - w2
    lmax = max(1.0, abs(math.log2(w2 + 0.01)), abs(math.log2(w2 + max(r_sat, 0.01))))
    off = abs(-2.0 * lower / (upper - lower) - 1.0)
    sc = max(abs(lower), abs(upper)) * 2.0 / (upper - lower)
    return (A * ((3.0 * 2.0 ** -24 + 2.2e-8) / math.log(2.0) + 2.0 ** -22 * lmax)
            + 2.0 ** -22 * (1.0 + off + sc))


@pytest.mark.parametrize("lower,upper,coeffs", [(-20.0, 20.0, (10.0, 0.0, 10.0)),
                                                (-5.0, 8.0, (4.0, 0.5, 2.0))])
def test_float32_utility_within_the_guards_bound(lower, upper, coeffs):
    """The reward guard (reward_risky) rests on a bound u_err on the float32 utility's error
    (utility_f32r: the hardware log2 taken as twice its measured worst case, tools/log2_probe.hip,
    every rounding counted at 2 ulp). On every active UE of a lean 45-step rollout (the shipped
    scenario instance at the defaults, the generic one at other utility parameters) the obs
    utility is within that bound of the oracle's float64 utility."""
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS["large"]
    E, n = 2048, 45
    seeds = 31 + np.arange(E)
    p = EngineParams(num_envs=E, num_ues=L["num_ues"], num_bs=len(L["bs"]), velocity=1.5,
                     util_lower=lower, util_upper=upper, util_coeffs=coeffs)
    eng = StepEngine(p, L["bs"], seeds, device="cuda")
    tr = eng.rollout(n)
    ob = OracleBatch(OracleParams(velocity=1.5, lower=lower, upper=upper, coeffs=coeffs), L["bs"],
                     L["num_ues"], seeds)
    worst = 0.0
    for s in range(n):
        o = ob.step()
        u = tr.obs[s, ..., 3].cpu().numpy().astype(np.float64)
        act = ~np.isnan(o["util"])
        worst = max(worst, float(np.max(np.abs(u[act] - o["util"][act]))))
    eng.close()
    bound = _u_err(lower, upper, *coeffs)
    assert worst <= bound, (worst, bound)


@pytest.mark.parametrize("size,k", [("large", 10), ("medium", 6)])
def test_reward_guard_partial_band_same_rows_every_shape(size, k):
    """The reward guard decides which env-steps take the exact path with ONE test in every
    kernel shape (the 2^-25 fixed-point sum against nact r_thr25): the two-group step's in-step
    test, the pipelined loop's flush (DETECT), the packed kernels' leaders. With the band made k
    times wider (reward_exact = -k: |mean| up to ~0.81 / ~0.49 instead of 0.086, which no
    large / medium env-step reaches) a subset of the rows -- some, not all -- takes the exact
    path; every shape then gives the same reward bits, the rows well inside the band are within
    one float32 ulp of the oracle's float64 mean (the exact path), and every row within 1e-5
    relative (atol 0) of it."""
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS[size]
    U, B, E, n = L["num_ues"], len(L["bs"]), 2000, 25
    seeds = 777 + 3 * np.arange(E)
    got = {}
    for tg, kind in ((3, "lds2_pipelined"), (1, "lds2_two_groups"), (-1, "packed_fused")):
        eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B, two_groups=tg,
                                      reward_exact=-k), L["bs"], seeds, device="cuda")
        tr = eng.rollout(n)
        assert eng.last_launch_kind == kind
        got[kind] = tr.reward.cpu().numpy()
        eng.close()
    eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B, reward_exact=-k), L["bs"],
                     seeds, device="cuda")
    rows = []
    for _ in range(n):
        eng.step()
        rows.append(eng.reward.cpu().numpy())
    assert eng.last_launch_kind == "packed_step"
    got["packed_step"] = np.stack(rows)
    eng.close()
    ref = got["lds2_pipelined"]
    for kind, v in got.items():
        np.testing.assert_array_equal(v, ref, err_msg=f"{kind} vs lds2_pipelined")
    ob = OracleBatch(OracleParams(), L["bs"], U, seeds)
    want = np.stack([ob.step()["metrics"][:, 2] for _ in range(n)])
    np.testing.assert_allclose(ref, want, rtol=1e-5, atol=0)
    # the band on the mean (mev_create: |isum| <= nact r_thr25, r_thr25 from k u_err)
    thr = (k * _u_err(-20.0, 20.0, 10.0, 0.0, 10.0) + 2.0 ** -24) / 9.5e-6 * 1.001
    inside, outside = np.abs(want) < 0.9 * thr, np.abs(want) > 1.1 * thr
    assert inside.mean() > 0.005 and outside.mean() > 0.005, (thr, inside.mean(), outside.mean())
    np.testing.assert_allclose(ref[inside], want[inside].astype(np.float32), rtol=1.2e-7, atol=0)


def test_small_deferred_reward_guard_same_rows_as_step():
    """mobile-small is the registered workload whose env-steps reach the reward guard's band
    (2.7 % of them at the default band, |mean| <= 0.086): its LDS-table rollout's rewards
    (k_steps_packed, in-step exact path) equal the one-step launches' bit for bit, over 45 steps
    (two resets) and with the band 3x wider, and are within 1e-5 relative (atol 0) of the
    oracle's float64 means."""
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS["small"]
    U, B, E, n = L["num_ues"], len(L["bs"]), 3000, 45
    seeds = 90001 + 5 * np.arange(E)
    ob = OracleBatch(OracleParams(), L["bs"], U, seeds)
    want = np.stack([ob.step()["metrics"][:, 2] for _ in range(n)])
    for rex in (0, -3):
        eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B, reward_exact=rex),
                         L["bs"], seeds, device="cuda")
        tr = eng.rollout(n)
        assert eng.last_launch_kind == "packed_fused"
        fused = tr.reward.cpu().numpy()
        eng.close()
        eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B, reward_exact=rex),
                         L["bs"], seeds, device="cuda")
        rows = []
        for _ in range(n):
            eng.step()
            rows.append(eng.reward.cpu().numpy())
        assert eng.last_launch_kind == "packed_step"
        eng.close()
        np.testing.assert_array_equal(fused, np.stack(rows), err_msg=f"reward_exact {rex}")
        np.testing.assert_allclose(fused, want, rtol=1e-5, atol=0, err_msg=f"reward_exact {rex}")


def test_small_rewards_at_the_guard_band_edge_vs_oracle():
    """The guard's band is |mean| <= ~0.086 at the default utility (u_err without round 5's
    extra factor 2): the env-steps just outside it take the float32 fast path and must
    still meet 1e-5 relative (atol 0). mobile-small has many of them (its means cluster at
    |mean| ~0.1-0.2): 20,000 envs x 45 steps of the shipped rollout and the one-step launches
    against the oracle's float64 means, with a few thousand env-steps in 0.086 < |mean| < 0.2."""
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.scenarios.registry import LAYOUTS
    from oracle.vec import OracleBatch, OracleParams
    L = LAYOUTS["small"]
    U, B, E, n = L["num_ues"], len(L["bs"]), 20000, 45
    seeds = 424242 + 7 * np.arange(E)
    ob = OracleBatch(OracleParams(), L["bs"], U, seeds)
    want = np.stack([ob.step()["metrics"][:, 2] for _ in range(n)])
    edge = (np.abs(want) > 0.0863) & (np.abs(want) < 0.2)
    assert edge.sum() > 2000, edge.sum()
    eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B), L["bs"], seeds, device="cuda")
    tr = eng.rollout(n)
    assert eng.last_launch_kind == "packed_fused"
    fused = tr.reward.cpu().numpy()
    eng.close()
    np.testing.assert_allclose(fused, want, rtol=1e-5, atol=0)
    eng = StepEngine(EngineParams(num_envs=E, num_ues=U, num_bs=B), L["bs"], seeds, device="cuda")
    rows = []
    for _ in range(n):
        eng.step()
        rows.append(eng.reward.cpu().numpy())
    assert eng.last_launch_kind == "packed_step"
    eng.close()
    np.testing.assert_array_equal(np.stack(rows), fused)
