"""GPU parity on the round-4 reference fixtures (tests/golden/make_golden.py --wide): maps of
1,500^2 and 4,096^2 (stations beyond the map's edge included), the tx = 55 channel, per-env
layouts on a 4,096 map (block kernel at U <= 64), U = 100 (block kernel), parameter classes on
a 4,096 map, and 30 distinct per-UE velocities with a per-UE snr_tr spread -- through the C ABI,
one-step launches and one 40-step rollout launch, against what the reference itself computed:
positions, serving stations and float64 rates bit-exact, float64 utilities within 1e-12, the
float32 reward within the north-star 1e-5 (relative)."""
import numpy as np
import pytest

from helpers import WIDE_FIXTURES, load, wide_engine_params

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _engine(d, **kw):
    from mobile_env.core.engine import StepEngine
    p = wide_engine_params(d, **kw)
    cnt = d["bs_count"] if "bs_count" in d else None
    return StepEngine(p, d["bs_xy"], d["seeds"], bs_count=cnt, device="cuda", rate64=True,
                      util64=True)


def _check_row(d, s, xy, srv, rate, util, reward):
    np.testing.assert_array_equal(xy, d["xy"][:, s], err_msg=f"positions step {s}")
    np.testing.assert_array_equal(srv, d["serving"][:, s], err_msg=f"serving step {s}")
    np.testing.assert_array_equal(rate, d["rate"][:, s], err_msg=f"rates step {s}")
    act = ~np.isnan(d["util"][:, s])
    np.testing.assert_allclose(util[act], d["util"][:, s][act], rtol=1e-12, atol=0)
    np.testing.assert_allclose(reward, d["metrics"][:, s, 2], rtol=RTOL, atol=0)


@pytest.mark.parametrize("name", WIDE_FIXTURES)
def test_wide_fixture_one_step_launches(name):
    d = load(name)
    eng = _engine(d)
    for s in range(d["xy"].shape[1]):
        eng.step()
        _check_row(d, s, eng.ue_xy.cpu().numpy(), eng.serving.cpu().numpy(),
                   eng.rate64.cpu().numpy(), eng.util64.cpu().numpy(), eng.reward.cpu().numpy())
    eng.close()


@pytest.mark.parametrize("name", WIDE_FIXTURES)
def test_wide_fixture_rollout_launch(name):
    d = load(name)
    eng = _engine(d)
    n = d["xy"].shape[1]
    tr = eng.rollout(n)
    W, H = int(d["width"]), int(d["height"])
    obs = tr.obs.cpu().numpy()
    for s in range(n):
        # positions from the obs rows (x / W, y / H in float32) -- exact for integers < 2^24
        xy = np.rint(np.stack([obs[s, ..., 0].astype(np.float64) * W,
                               obs[s, ..., 1].astype(np.float64) * H], -1)).astype(np.int64)
        _check_row(d, s, xy, tr.serving[s].cpu().numpy(), tr.rate64[s].cpu().numpy(),
                   tr.util64[s].cpu().numpy(), tr.reward[s].cpu().numpy())
    np.testing.assert_array_equal(eng.ue_xy.cpu().numpy(), d["xy"][:, n - 1])
    eng.close()


@pytest.mark.parametrize("launch", ["step", "rollout"])
def test_per_ue_velocities_on_block_kernel(launch):
    """The per-UE velocity fixture (30 distinct velocities, snr_tr in 4 channel classes) on the
    block kernel: the same shared layout handed over as per-env layouts (one workgroup per env,
    mev_step_shape 2) -- the other kernel family the movement table per UE goes through."""
    from mobile_env.core.engine import StepEngine
    d = load("velocities_large")
    E = len(d["seeds"])
    bs = np.broadcast_to(d["bs_xy"], (E,) + d["bs_xy"].shape).copy()
    eng = StepEngine(wide_engine_params(d), bs, d["seeds"], device="cuda", rate64=True,
                     util64=True)
    assert eng.step_shape == "block"
    n = d["xy"].shape[1]
    if launch == "step":
        for s in range(n):
            eng.step()
            _check_row(d, s, eng.ue_xy.cpu().numpy(), eng.serving.cpu().numpy(),
                       eng.rate64.cpu().numpy(), eng.util64.cpu().numpy(),
                       eng.reward.cpu().numpy())
    else:
        tr = eng.rollout(n)
        for s in range(n):
            xy = np.rint(tr.obs[s, ..., :2].double().cpu().numpy() * 200).astype(np.int64)
            _check_row(d, s, xy, tr.serving[s].cpu().numpy(), tr.rate64[s].cpu().numpy(),
                       tr.util64[s].cpu().numpy(), tr.reward[s].cpu().numpy())
    eng.close()
