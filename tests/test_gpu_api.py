"""GPU tests of the host surfaces: the MComCore/MComCustom facade (reference object API) and
the batched make()/reset()/step() surface, against the reference fixtures and the oracle."""
import random

import numpy as np
import pytest

from helpers import load

pytestmark = pytest.mark.gpu


def test_mcom_custom_facade_matches_reference():
    from mobile_env.scenarios.custom import MComCustom
    d = load("mcom_custom")
    for k in range(8):
        random.seed(int(d["random_seeds"][k]))
        env = MComCustom()
        users = [env.userDict[i] for i in sorted(env.userDict)]
        s = 0
        for ep in range(2):
            env.reset()
            lay = [[bs.point.x, bs.point.y] for bs in env.stationDict.values()]
            assert lay == d["bs_xy"][k, ep, :d["bs_count"][k, ep]].tolist()
            for _ in range(20):
                env.step(ep, s % 20)
                xy = [[ue.x, ue.y] for ue in users]
                assert xy == d["xy"][k, s].tolist()
                srv = [-1] * 7
                for (bs, ue) in env.bs2ue_dataRates:
                    srv[ue.ue_id] = bs.bs_id
                assert srv == d["serving"][k, s].tolist()
                rates = [float(env.allUserDataRates.get(ue, 0.0)) for ue in users]
                assert rates == d["rate"][k, s].tolist()
                ut = [env.ue_utilities.get(ue, np.nan) for ue in users]
                np.testing.assert_allclose(ut, d["util"][k, s], rtol=1e-12)
                sc = env.monitor.scalar_results
                assert sc["number connections"][-1] == d["metrics"][k, s, 0]
                np.testing.assert_allclose(sc["mean utility"][-1], d["metrics"][k, s, 2],
                                           rtol=1e-5)
                s += 1
            assert env.time_is_up
        env.close()


def test_bare_core_first_step_is_noop():
    """Bare MComCore.reset never refills activeUsers (reference base.py:75,172-209): the first
    step of each episode moves nobody and reports mean utility = lower (metrics.py:26-27)."""
    from mobile_env.core.base import MComCore
    from mobile_env.core.entities import BaseStation, UserEquipment
    cfg = MComCore.default_config()
    st = [BaseStation(i, p, **cfg["bs"]) for i, p in enumerate([(50, 50), (150, 150)])]
    us = [UserEquipment(i, **cfg["ue"]) for i in range(4)]
    env = MComCore(st, us, {"seed": 5})
    env.reset()
    before = [(u.x, u.y) for u in us]
    env.step(0, 0)
    assert [(u.x, u.y) for u in us] == before
    assert env.monitor.scalar_results["mean utility"][-1] == -20
    assert len(env.activeUsers) == 4
    env.step(0, 1)
    assert env.monitor.scalar_results["number connected"][-1] >= 0
    env.close()


@pytest.mark.parametrize("env_id", ["mobile-small-central-v0", "mobile-medium-ma-v0",
                                    "mobile-large-central-v0", "mobile-large-ma-v0",
                                    "mobile-custom-128x1024-v0"])
def test_make_reset_step_matches_oracle(env_id):
    import mobile_env
    from oracle.vec import OracleBatch, OracleParams
    from mobile_env.scenarios.registry import LAYOUTS, spec
    sp = spec(env_id)
    E = 64 if sp["num_ues"] <= 64 else 3
    env = mobile_env.make(env_id, num_envs=E, seed=300)
    obs, info = env.reset()
    if sp["per_env_layout"]:
        bs = env.engine.bs_xy.cpu().numpy()
        U = sp["num_ues"]
        ob = OracleBatch(OracleParams(velocity=float(sp["velocity"])), bs, U,
                         np.arange(E) + 300)
    else:
        lay = LAYOUTS[sp["layout"]]
        U = lay["num_ues"]
        ob = OracleBatch(OracleParams(), lay["bs"], U, np.arange(E) + 300)
    ob.reset()
    np.testing.assert_array_equal(env.engine.ue_xy.cpu().numpy(),
                                  np.stack([ob.x, ob.y], -1))
    for s in range(45 if U <= 64 else 22):
        obs, rew, term, trunc, info = env.step()
        o = ob.step()
        o4 = obs.cpu().numpy().reshape(E, U, 4)
        np.testing.assert_array_equal(info["serving"].cpu().numpy(), o["serving"])
        np.testing.assert_allclose(o4[..., 0], o["xy"][..., 0] / 200.0, rtol=1e-6)
        np.testing.assert_allclose(o4[..., 2], o["rate"].astype(np.float32), rtol=1e-5)
        if sp["mode"] == "central":
            np.testing.assert_allclose(rew.cpu().numpy(), o["metrics"][:, 2], rtol=1e-5,
                                       atol=0)
        else:
            np.testing.assert_allclose(rew.cpu().numpy(), o["util"].astype(np.float32),
                                       rtol=1e-5, atol=0)
        np.testing.assert_array_equal(trunc.cpu().numpy(), o["done"])
        assert not term.any()
    env.close()


def test_device_seeding_equals_host_seeding():
    """mev_seed_pcg64_device (SeedSequence hashing on the device) == the host version."""
    import ctypes as C
    import numpy as np
    import torch
    from mobile_env.core import _native as N
    rng = np.random.default_rng(3)
    seeds = np.concatenate([[0, 1, 4, 2**32 - 1, 2**32, 2**62 + 5, 2**63 - 1],
                            rng.integers(0, 2**63 - 1, size=5000, dtype=np.int64)]).astype(np.uint64)
    want = N.seed_pcg64(seeds)
    d_seeds = torch.from_numpy(seeds.view(np.int64)).cuda()
    rows = torch.zeros((len(seeds), 6), dtype=torch.int64, device="cuda")
    N.check(N.lib().mev_seed_pcg64_device(C.c_void_p(d_seeds.data_ptr()), len(seeds),
                                          C.c_void_p(rows.data_ptr()), None), "seed")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rows.cpu().numpy().view(np.uint64), want)
    st = np.random.PCG64(int(seeds[100])).state["state"]
    assert int(want[100, 0]) | (int(want[100, 1]) << 64) == st["state"]


def test_make_custom_layouts_are_the_fixture_layouts():
    """make("mobile-custom-128x1024-v0") draws each env's 128 stations from its seed; the
    per-env 128 x 1024 fixture (generated by the reference on those layouts) then matches the
    batched surface step by step: positions and serving bit-exact, rates within 1e-5."""
    import mobile_env
    d = load("custom128x1024_perenv")
    E = len(d["seeds"])
    env = mobile_env.make("mobile-custom-128x1024-v0", num_envs=E, seed=int(d["seeds"][0]))
    np.testing.assert_array_equal(env.engine.bs_xy.cpu().numpy(), d["bs_xy"])
    env.reset()
    np.testing.assert_array_equal(env.engine.ue_xy.cpu().numpy(), d["init_xy"][:, 0])
    for s in range(d["xy"].shape[1]):
        obs, rew, term, trunc, info = env.step()
        np.testing.assert_array_equal(env.engine.ue_xy.cpu().numpy(), d["xy"][:, s])
        np.testing.assert_array_equal(info["serving"].cpu().numpy(), d["serving"][:, s])
        o4 = obs.cpu().numpy().reshape(E, 1024, 4)
        np.testing.assert_allclose(o4[..., 2], d["rate"][:, s].astype(np.float32), rtol=1e-5)
        np.testing.assert_allclose(rew.cpu().numpy(), d["metrics"][:, s, 2], rtol=1e-5,
                                   atol=0)
    env.close()


def test_mcom_core_facade_heterogeneous_entities():
    """MComCore over stations / UEs that carry their own parameters (the reference's entity
    model, entities.py:7-45): the facade lowers them to parameter classes and reproduces the
    reference's heterogeneous fixture."""
    import json
    from mobile_env.core.base import MComCore
    from mobile_env.core.entities import BaseStation, UserEquipment
    d = load("large_mixed")
    bsc, uec = json.loads(str(d["bs_classes"])), json.loads(str(d["ue_classes"]))

    class Core(MComCore):
        _first_step_active = True  # the fixture's driver refills activeUsers at reset

    for k, seed in enumerate(d["seeds"]):
        st = [BaseStation(j, (int(x), int(y)), **bsc[c])
              for j, ((x, y), c) in enumerate(zip(d["bs_xy"], d["bs_class"]))]
        us = [UserEquipment(i, **uec[c]) for i, c in enumerate(d["ue_class"])]
        env = Core(st, us, {"seed": int(seed)})
        for ep in range(2):
            env.reset()
            env.activeUsers = sorted(us, key=lambda u: u.ue_id)
            for s in range(20):
                env.step(ep, s)
                assert [[int(u.x), int(u.y)] for u in us] == d["xy"][k, ep * 20 + s].tolist()
                rates = [float(env.allUserDataRates.get(u, 0.0)) for u in us]
                assert rates == d["rate"][k, ep * 20 + s].tolist()
        assert env.check_connectivity(st[0], us[0]) in (True, False)
        env.close()


@pytest.mark.parametrize("which", ["default", "notebook"])
def test_c_caller_libm_table_shares_round_like_reference(golden_dir, which):
    """A C caller that passes no rate table (mev_params.rate_table = NULL) gets mev_create's libm
    table; the rounded ResourceFair shares the kernels form from it (both device paths: the
    reciprocal form for every n <= 1024, the 100/n table form for n <= 64) equal the
    reference's numpy round(rate / n, 2) (base.py:427-435) on the reference's own rates."""
    import ctypes as C
    import json

    import torch
    from mobile_env.core import _native as N
    from mobile_env.core.engine import EngineParams
    c = np.load(f"{golden_dir}/channel_{which}.npz")
    bs, ue = json.loads(str(c["bs"])), json.loads(str(c["ue"]))
    cp = EngineParams(num_envs=1, num_ues=1024, num_bs=3, bs=bs,
                      ue={k: ue[k] for k in ("snr_tr", "noise", "height")}).to_c(False)
    assert not cp.rate_table  # the C library builds the table
    L = N.lib()
    ctx = C.c_void_p()
    with torch.cuda.device(0):
        N.check(L.mev_create(C.byref(cp), C.byref(ctx)), "mev_create")
        try:
            assert L.mev_d2max(ctx) == int(c["d2max"])
            ref = c["rate"]
            for path, nmax in ((0, 1024), (1, 64)):
                out = torch.empty((nmax, len(ref)), dtype=torch.float64, device="cuda")
                N.check(L.mev_share_cents(ctx, nmax, path, C.c_void_p(out.data_ptr()), None),
                        "mev_share_cents")
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                for n in range(1, nmax + 1):
                    np.testing.assert_array_equal(got[n - 1] / 100.0, np.round(ref / n, 2),
                                                  err_msg=f"path {path} share count {n}")
        finally:
            L.mev_destroy(ctx)


@pytest.mark.parametrize("U,B,launch", [(30, 13, "step"), (30, 13, "rollout"), (100, 24, "step"),
                                        (100, 24, "rollout")])
def test_checkpoint_restore_mid_episode(U, B, launch):
    """A checkpoint {ue_state, pcg (read through the synced property), t} taken mid-episode and
    restored into a fresh engine with OTHER seeds (restore_state -> mev_restore_stream_state)
    continues exactly like the saving engine -- across the episode's remaining draws (which
    come from the restored stream rows, not the new context's draw table) and the next
    episodes (the tables rebuilt from the restored state0). Velocity 10 on 200 x 200: several
    waypoint draws per episode. Packed (U = 30) and block (U = 100) shapes, one-step and
    fused rollout launches. ADVICE r03: without the restore call the new context re-read the
    episode's first table pairs."""
    import torch
    from mobile_env.core.engine import EngineParams, StepEngine
    rng = np.random.default_rng(7)
    E = 48
    bs = rng.integers(0, 200, size=(B, 2)).tolist()
    p = EngineParams(num_envs=E, num_ues=U, num_bs=B, velocity=10.0)
    a = StepEngine(p, bs, 1000 + np.arange(E), device="cuda")
    b = StepEngine(p, bs, 90000 + np.arange(E), device="cuda")
    c = StepEngine(p, bs, 90000 + np.arange(E), device="cuda")
    for eng in (a, b, c):
        eng.reset()
    a.step(7)
    ck = (a.ue_state.clone(), a.pcg.clone(), a.t.clone())
    b.restore_state(*ck)
    c.restore_state(*ck, declare=False)  # the same rows without the restore call (the bug)
    n = 33  # the rest of episode 1 (13 steps) and one more episode

    def run(eng):
        if launch == "rollout":
            tr = eng.rollout(n)
            return [tr.obs.cpu(), tr.serving.cpu(), tr.reward.cpu(), tr.done.cpu()]
        rows = []
        for _ in range(n):
            eng.step()
            rows.append([eng.obs.cpu(), eng.serving.cpu(), eng.reward.cpu(), eng.done.cpu()])
        return [torch.stack(col) for col in zip(*rows)]

    ra, rb, rc = run(a), run(b), run(c)
    for x, y in zip(ra, rb):
        assert torch.equal(x, y)
    assert torch.equal(a.ue_state, b.ue_state) and torch.equal(a.pcg, b.pcg)
    assert not torch.equal(ra[0], rc[0])  # the draw-table replay the restore call prevents
    for eng in (a, b, c):
        eng.close()
