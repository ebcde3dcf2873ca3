"""CPU tests of the reference's config knobs the engine lowers into kernel branches
(MComCore.default_config, reference base.py:103-153, deep-merged at base.py:47):

* movement_params.reset_rng_episode = False -- one movement stream continued across episodes
  (movement.py:16-18) instead of re-seeded at every reset;
* EP_MAX_TIME != the arrival ep_time -- the episode ends at min(EP_MAX_TIME, max departure)
  (base.py:105-109,126,407-409);
* non-default utility_params lower / upper / coeffs (utilities.py:44-55).

Fixtures: tests/golden/knob_*.npz, written by the reference itself (make_golden.py --knobs; the
driver loop runs each episode until the reference's time_is_up). Here: the NumPy oracle and
the per-object port reproduce them bit for bit (pinning the checker the GPU tests rely on), and
the facade lowers each config to the engine parameters the kernels branch on. The GPU side is
tests/test_gpu_knobs.py."""
import numpy as np
import pytest

from helpers import KNOB_FIXTURES, knob_config, knob_done, knob_oracle_params, knob_params, load
from oracle import port
from oracle.vec import OracleBatch


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_vec_oracle_matches_knob_fixture(name):
    d = load(name)
    p = knob_oracle_params(d)
    ob = OracleBatch(p, d["bs_xy"], d["xy"].shape[2], d["seeds"])
    done = knob_done(d)
    for s in range(d["xy"].shape[1]):
        o = ob.step()
        np.testing.assert_array_equal(o["xy"], d["xy"][:, s], err_msg=f"{name} step {s}")
        np.testing.assert_array_equal(o["serving"], d["serving"][:, s])
        np.testing.assert_array_equal(o["rate"], d["rate"][:, s])
        act = ~np.isnan(d["util"][:, s])
        np.testing.assert_array_equal(np.isnan(o["util"]), ~act)
        np.testing.assert_array_equal(o["util"][act], d["util"][:, s][act])
        np.testing.assert_array_equal(o["metrics"][:, :3], d["metrics"][:, s, :3])
        np.testing.assert_allclose(o["metrics"][:, 3], d["metrics"][:, s, 3], rtol=1e-12)
        np.testing.assert_array_equal(o["done"], np.full(ob.E, done[s]))


@pytest.mark.parametrize("name", ["knob_noreseed_small_v10", "knob_ept12_large",
                                  "knob_ep15_medium_v10", "knob_util_large_v10"])
def test_port_matches_knob_fixture(name):
    """The per-object port (the bench's CPU baseline) under the same knobs."""
    d = load(name)
    p = knob_oracle_params(d)
    lens = d["episode_len"][0]
    for k in range(len(d["seeds"])):
        core = port.build(d["bs_xy"], d["xy"].shape[2], int(d["seeds"][k]), float(d["velocity"]),
                          ep_time=p.arrival_ep_time, ep_max_time=p.ep_max_time, lower=p.lower,
                          upper=p.upper, coeffs=p.coeffs, reseed=p.movement_reseed)
        s = 0
        for n in lens:
            core.reset()
            for _ in range(int(n)):
                core.step()
                xy, srv, rate, util, met = core.snapshot()
                assert xy == [tuple(v) for v in d["xy"][k, s].tolist()], (name, k, s)
                assert srv == d["serving"][k, s].tolist()
                assert rate == d["rate"][k, s].tolist()
                np.testing.assert_array_equal(util, d["util"][k, s])
                s += 1


def test_noreseed_fixture_continues_the_stream():
    """Sanity of the fixture itself: without re-seeding, later episodes start elsewhere (the
    stream moved on), with it they replay the first episode's initial positions."""
    d = load("knob_noreseed_large")
    init = d["init_xy"]
    assert not np.array_equal(init[:, 0], init[:, 1])
    assert not np.array_equal(init[:, 1], init[:, 2])
    ref = load("large")  # default config: re-seeded
    np.testing.assert_array_equal(ref["init_xy"][:, 0], ref["init_xy"][:, 1])


@pytest.mark.parametrize("name", KNOB_FIXTURES)
def test_facade_lowers_knob_config(name):
    """MComCore(config) -> lowering.lower gives the engine the knob values."""
    d = load(name)
    cfg = knob_config(d)
    p = knob_params(d)
    op = knob_oracle_params(d)
    assert p.movement_reseed == op.movement_reseed
    assert p.ep_max_time == op.ep_max_time and p.arrival_exit == op.arrival_ep_time
    assert p.t_end == op.t_end == int(d["episode_len"][0][0])
    assert (p.util_lower, p.util_upper) == (float(op.lower), float(op.upper))
    assert p.util_coeffs == tuple(float(c) for c in op.coeffs)
    assert p.num_ues == d["xy"].shape[2] and p.velocity == float(d["velocity"])
    if "movement_params" in cfg:
        assert p.movement_reseed is False
