"""CPU tests of the plugin objects the facade exposes (reference core/channels.py,
schedules.py, utilities.py, movement.py): the per-entity methods reproduce the reference's
values on its own fixtures, and the channel rate table the engine uploads is the reference's
table bit for bit. No GPU is used."""
import json
import math

import numpy as np
import pytest

from helpers import load

BS = {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50}
UE = {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}


def _entities(bs=BS, ue=UE, velocity=1.5):
    from mobile_env.core.entities import BaseStation, UserEquipment
    return (BaseStation(0, (0, 0), bs["bw"], bs["freq"], bs["tx"], bs["height"]),
            UserEquipment(0, velocity, ue["snr_tr"], ue["noise"], ue["height"]))


@pytest.mark.parametrize("which", ["default", "notebook"])
def test_rate_table_is_the_reference_table(golden_dir, which):
    """mobile_env.core.channels builds the table the engine uploads (mev_params.rate_table):
    raw float64 entries equal to the reference's at every connectable d2."""
    from mobile_env.core.channels import OkumuraHata
    c = np.load(f"{golden_dir}/channel_{which}.npz")
    bs, ue = json.loads(str(c["bs"])), json.loads(str(c["ue"]))
    tab = OkumuraHata().rate_table(bs, ue)
    assert len(tab) == int(c["d2max"]) + 1
    np.testing.assert_array_equal(tab, c["rate"])


def test_c_library_table_within_a_few_ulp(golden_dir):
    """mev_build_rate_table (libm, for C callers without numpy): the same connectable range,
    every entry within a few ulp of the reference's and most equal (numpy's SIMD log10 differs
    from libm's by an ulp on a few inputs, which pow / log2 carry on: the reason the Python
    host passes numpy's table)."""
    import ctypes as C
    from mobile_env.core import _native as N
    from mobile_env.core.engine import EngineParams
    c = np.load(f"{golden_dir}/channel_default.npz")
    cp = EngineParams(num_envs=1, num_ues=5, num_bs=3).to_c(False)
    lib = N.lib()
    n = lib.mev_build_rate_table(C.byref(cp), None, 0)
    assert n == int(c["d2max"]) + 1
    tab = np.zeros(n)
    assert lib.mev_build_rate_table(C.byref(cp), tab.ctypes.data, n) == n
    ulps = np.abs(tab.view(np.int64) - c["rate"].view(np.int64))
    assert ulps.max() <= 4 and (ulps != 0).mean() < 0.01


@pytest.mark.parametrize("which", ["default", "notebook"])
def test_c_library_table_rounds_like_the_reference(golden_dir, which):
    """What a C caller of the libm table (mev_params.rate_table = NULL) depends on: the
    ResourceFair share rounded to cents, numpy round(rate / n, 2) (base.py:427-435), equals the
    reference's for every connectable d2 and every share count n <= 1024 (the largest U), on
    both channel parameter sets -- the few entries that differ by an ulp or two never move a
    cent."""
    import ctypes as C
    from mobile_env.core import _native as N
    from mobile_env.core.engine import EngineParams
    c = np.load(f"{golden_dir}/channel_{which}.npz")
    bs, ue = json.loads(str(c["bs"])), json.loads(str(c["ue"]))
    cp = EngineParams(num_envs=1, num_ues=5, num_bs=3, bs=bs,
                      ue={k: ue[k] for k in ("snr_tr", "noise", "height")}).to_c(False)
    lib = N.lib()
    n = lib.mev_build_rate_table(C.byref(cp), None, 0)
    assert n == int(c["d2max"]) + 1
    tab = np.zeros(n)
    assert lib.mev_build_rate_table(C.byref(cp), tab.ctypes.data, n) == n
    ref = c["rate"]
    assert (tab != ref).any() or which == "notebook"  # (the default table has differing entries)
    for k in range(1, 1025):
        np.testing.assert_array_equal(np.round(tab / k, 2), np.round(ref / k, 2),
                                      err_msg=f"share count {k}")


def test_channel_methods_match_reference_table(golden_dir):
    """Channel.calculateSNR / datarate + OkumuraHata.power_loss on entity pairs at integer
    squared distances d2 equal the reference's table entry (channels.py:24-27,78-83,133-146),
    and a pair past d2max is not connectable (datarate 0)."""
    from mobile_env.core.channels import OkumuraHata
    c = np.load(f"{golden_dir}/channel_default.npz")
    ch = OkumuraHata()
    bs, ue = _entities()
    rng = np.random.default_rng(0)
    for _ in range(300):
        x, y = (int(v) for v in rng.integers(0, 140, 2))
        ue.x, ue.y = x, y
        snr = ch.calculateSNR(bs, ue)
        d2 = x * x + y * y
        if d2 <= int(c["d2max"]):
            assert ch.datarate(bs, ue, snr) == c["rate"][d2]
        else:
            assert ch.datarate(bs, ue, snr) == 0.0


def test_resource_fair_share_matches_fixture_rates(golden_dir):
    """ResourceFair.share + numpy round(., 2) (schedules.py:20-22, base.py:435) on the full
    rates of each station's connected UEs reproduces the fixture's per-UE rates."""
    from mobile_env.core.schedules import RateFair, ResourceFair
    c = np.load(f"{golden_dir}/channel_default.npz")
    d = load("large")
    bs_xy = d["bs_xy"]
    sched = ResourceFair()
    for k in range(d["xy"].shape[0]):
        for s in range(0, d["xy"].shape[1], 3):
            xy, srv = d["xy"][k, s], d["serving"][k, s]
            for b in np.unique(srv[srv >= 0]):
                ues = np.nonzero(srv == b)[0]
                d2 = ((xy[ues] - bs_xy[b]) ** 2).sum(1)
                shares = sched.share(None, [np.float64(v) for v in c["rate"][d2]])
                got = [round(v, 2) for v in shares]
                assert got == d["rate"][k, s, ues].tolist()
    assert RateFair().share(None, [2.0, 2.0]) == 1.0


def test_bounded_log_utility_matches_fixture():
    """BoundedLogUtility.calculateUtility + scaleUtility (utilities.py:44-55) of each active
    UE's rate equals the fixture's scaled utility, bit for bit; unscale inverts scale."""
    from mobile_env.core.utilities import BoundedLogUtility
    u = BoundedLogUtility(lower=-20, upper=20, coeffs=(10, 0, 10))
    d = load("mcom_custom")
    rate, util = d["rate"].ravel(), d["util"].ravel()
    act = ~np.isnan(util)
    got = np.array([u.scaleUtility(u.calculateUtility(np.float64(r))) for r in rate[act]])
    np.testing.assert_array_equal(got, util[act])
    assert u.calculateUtility(0.0) == -20
    assert u.unscaleUtility(u.scaleUtility(7.5)) == 7.5


@pytest.mark.parametrize("name", ["large", "small_v10"])
def test_random_waypoint_plugin_reproduces_fixture_trajectories(name):
    """RandomWaypointMovement.reset / initial_position / move (movement.py:16-18,42-72), driven
    like MComCore.reset + step (ids in order, movement seed = config seed + 4), reproduce the
    reference's positions over two episodes."""
    from mobile_env.core.entities import UserEquipment
    from mobile_env.core.movement import RandomWaypointMovement
    d = load(name)
    U = d["xy"].shape[2]
    vel = float(d["velocity"])
    for k, seed in enumerate(d["seeds"]):
        mv = RandomWaypointMovement(width=200, height=200, seed=int(seed) + 4,
                                    reset_rng_episode=True)
        ues = [UserEquipment(i, vel, 2e-8, 1e-9, 1.6) for i in range(U)]
        for ep in range(2):
            mv.reset()
            for ue in ues:
                ue.x, ue.y = mv.initial_position(ue)
            assert [[ue.x, ue.y] for ue in ues] == d["init_xy"][k, ep].tolist()
            for s in range(20):
                for ue in ues:
                    ue.x, ue.y = mv.move(ue)
                assert [[int(ue.x), int(ue.y)] for ue in ues] == d["xy"][k, ep * 20 + s].tolist()


def test_no_departure_plugin():
    from mobile_env.core.arrival import NoDeparture
    a = NoDeparture(ep_time=20, seed=3, reset_rng_episode=False)
    a.reset()
    assert a.rng is not None
    _, ue = _entities()
    assert (a.setArrivalTime(ue), a.setDepartureTime(ue)) == (0, 20)
    assert math.isfinite(a.ep_time)
