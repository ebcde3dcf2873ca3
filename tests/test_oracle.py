"""CPU tests: pin the oracle (NumPy restatement + per-object port) to the reference's golden
fixtures and notebook snapshots, and property-test the step semantics."""
import math

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from helpers import FIXTURES, WIDE_FIXTURES, load, snapshots
from oracle import port
from oracle.vec import OracleBatch, OracleParams, channel_table, snr_scalar

TABLE = channel_table(OracleParams())


def _run_vec(name):
    d = load(name)
    p = OracleParams(velocity=float(d["velocity"]))
    if "bs_count" in d:
        ob = OracleBatch(p, d["bs_xy"][:, 0], d["xy"].shape[2], d["seeds"],
                         bs_count=d["bs_count"][:, 0], table=TABLE)
    else:
        ob = OracleBatch(p, d["bs_xy"], d["xy"].shape[2], d["seeds"], table=TABLE)
    for s in range(d["xy"].shape[1]):
        if "bs_count" in d and s == 20:
            for e in range(ob.E):
                ob.set_bs(e, d["bs_xy"][e, 1, :d["bs_count"][e, 1]])
        o = ob.step()
        np.testing.assert_array_equal(o["xy"], d["xy"][:, s])
        np.testing.assert_array_equal(o["serving"], d["serving"][:, s])
        np.testing.assert_array_equal(o["rate"], d["rate"][:, s])
        np.testing.assert_array_equal(np.isnan(o["util"]), np.isnan(d["util"][:, s]))
        act = ~np.isnan(d["util"][:, s])
        np.testing.assert_array_equal(o["util"][act], d["util"][:, s][act])
        np.testing.assert_array_equal(o["metrics"][:, :3], d["metrics"][:, s, :3])
        np.testing.assert_allclose(o["metrics"][:, 3], d["metrics"][:, s, 3], rtol=1e-12)
        np.testing.assert_array_equal(o["done"], np.full(ob.E, s % 20 == 19))


@pytest.mark.parametrize("name", FIXTURES)
def test_vec_oracle_matches_reference_fixture(name):
    _run_vec(name)


def test_channel_table_matches_reference(golden_dir):
    c = np.load(f"{golden_dir}/channel_default.npz")
    assert TABLE[0] == int(c["d2max"]) == 19362
    np.testing.assert_array_equal(TABLE[1], c["rate"])
    n = np.load(f"{golden_dir}/channel_notebook.npz")
    p = OracleParams(bs={"bw": 9e6, "freq": 2500, "tx": 30, "height": 50},
                     ue={"snr_tr": 2e-8, "noise": 1e-9, "height": 1.8})
    d2max, rate = channel_table(p)
    assert d2max == int(n["d2max"]) == 5379
    np.testing.assert_array_equal(rate, n["rate"])


@pytest.mark.parametrize("name,nseeds", [("small", 3), ("large", 1), ("small_v10", 2),
                                         ("large_v10", 1)])
def test_port_matches_reference_fixture(name, nseeds):
    d = load(name)
    for k in range(nseeds):
        core = port.build(d["bs_xy"], d["xy"].shape[2], int(d["seeds"][k]), float(d["velocity"]))
        got = []
        port.run_driver(core, 2, 20, on_step=lambda ep, s, c: got.append(c.snapshot()))
        for s, (xy, srv, rate, util, met) in enumerate(got):
            assert xy == [tuple(v) for v in d["xy"][k, s].tolist()]
            assert srv == d["serving"][k, s].tolist()
            assert rate == d["rate"][k, s].tolist()
            np.testing.assert_array_equal(util, d["util"][k, s])
            np.testing.assert_array_equal(met[:3], d["metrics"][k, s, :3])
            np.testing.assert_allclose(met[3], d["metrics"][k, s, 3], rtol=1e-12)


def test_port_matches_mcom_custom_fixture():
    d = load("mcom_custom")
    for k in range(3):
        got = []
        core = None
        for ep in range(2):
            lay = d["bs_xy"][k, ep, :d["bs_count"][k, ep]]
            fresh = port.build(lay, 7, int(d["seeds"][k]), 10.0)
            if core is None:
                core = fresh
            else:
                core.stations = fresh.stations
            core.reset()
            for s in range(20):
                core.step()
                got.append(core.snapshot())
        for s, (xy, srv, rate, util, met) in enumerate(got):
            assert srv == d["serving"][k, s].tolist()
            assert rate == d["rate"][k, s].tolist()
            np.testing.assert_array_equal(util, d["util"][k, s])


def test_notebook_snapshots_with_oracle():
    snaps = snapshots()
    p = OracleParams(velocity=10.0, bs=snaps["params"]["bs"],
                     ue={k: v for k, v in snaps["params"]["ue"].items() if k != "velocity"})
    table = channel_table(p)
    for snap in snaps["snapshots"]:
        ob = OracleBatch(p, snap["bs_xy"], 7, [snaps["params"]["seed"]], table=table)
        for _ in range(snap["step"] + 1):
            o = ob.step()
        assert o["xy"][0].tolist() == snap["ue_xy"]
        got = {u: (int(o["serving"][0, u]), float(o["rate"][0, u]))
               for u in range(7) if o["serving"][0, u] >= 0}
        want = {e["ue_id"]: (e["bs_id"], e["data_rate"]) for e in snap["rates"]}
        assert got == want


# -- properties of the step semantics ---------------------------------------

def test_connectivity_is_prefix_in_d2():
    p = OracleParams()
    d2max = TABLE[0]
    for d2 in list(range(0, 200)) + list(range(d2max - 500, d2max + 500)):
        assert (snr_scalar(d2, p.bs, p.ue) > p.ue["snr_tr"]) == (d2 <= d2max)


@settings(max_examples=60, deadline=None)
@given(st.integers(0, 199), st.integers(0, 199), st.integers(1, 6))
def test_tie_break_lowest_bs_id(x, y, nbs):
    # all stations at the same spot: the UE must attach to station 0 (python min() keeps the
    # first of equal keys, base.py:240)
    p = OracleParams(velocity=0.0)
    ob = OracleBatch(p, [[x, y]] * nbs, 1, [7], table=TABLE)
    ob.reset()
    ob.x[0, 0], ob.y[0, 0] = x, y
    ob.wx[0, 0], ob.wy[0, 0], ob.wvalid[0, 0] = x, y, True
    o = ob.step()
    assert o["serving"][0, 0] == 0


def test_numpy_round_semantics():
    # numpy round is rint(x*100)/100 (half-to-even on the scaled value), not python round
    assert np.round(2.675, 2) == 2.67 or np.round(2.675, 2) == 2.68
    for v in (0.125, 0.375, 2.675, 1.005, 700.195):
        assert np.round(np.float64(v), 2) == np.rint(v * 100.0) / 100.0


@settings(max_examples=20, deadline=None)
@given(st.integers(0, 10_000), st.sampled_from([1.5, 3.0, 10.0, 37.0]))
def test_ues_stay_inside_map(seed, vel):
    p = OracleParams(velocity=vel)
    ob = OracleBatch(p, [[50, 50], [150, 150]], 6, [seed], table=TABLE)
    for _ in range(25):
        o = ob.step()
        assert (o["xy"] >= 0).all() and (o["xy"] < 200).all()


def test_velocity_int_and_float_agree():
    # MComCustom uses an int velocity (custom.py:17); int*v and float*v give the same step
    d = 37
    assert (10 * d) / math.sqrt(d * d) == (10.0 * d) / math.sqrt(d * d)


def _mixed_oracle(d):
    import json
    bsc, uec = json.loads(str(d["bs_classes"])), json.loads(str(d["ue_classes"]))
    p = OracleParams(bs_classes=bsc, ue_classes=uec, bs_class=d["bs_class"].tolist(),
                     ue_class=d["ue_class"].tolist())
    return OracleBatch(p, d["bs_xy"], d["xy"].shape[2], d["seeds"])


def test_vec_oracle_matches_heterogeneous_fixture():
    """Per-station (bw, freq, tx, height) and per-UE (velocity, snr_tr, noise, height)
    parameters (entities.py:7-22,33-45; the reference evaluates the channel per pair,
    channels.py:133-146): the oracle with one table per class pair and per-UE velocities
    reproduces the reference's positions, serving stations, rates and utilities bit for bit."""
    d = load("large_mixed")
    ob = _mixed_oracle(d)
    for s in range(d["xy"].shape[1]):
        o = ob.step()
        np.testing.assert_array_equal(o["xy"], d["xy"][:, s], err_msg=f"step {s}")
        np.testing.assert_array_equal(o["serving"], d["serving"][:, s], err_msg=f"step {s}")
        np.testing.assert_array_equal(o["rate"], d["rate"][:, s], err_msg=f"step {s}")
        act = ~np.isnan(d["util"][:, s])
        np.testing.assert_array_equal(o["util"][act], d["util"][:, s][act])
        np.testing.assert_array_equal(o["metrics"][:, :3], d["metrics"][:, s, :3])


def test_port_matches_heterogeneous_fixture():
    """The per-object port with per-entity parameters (port.build(classes=...), what bench.py's
    cpu_baseline runs for mobile-large-mixed-v0) reproduces the reference's fixture."""
    import json
    d = load("large_mixed")
    classes = dict(bs_classes=json.loads(str(d["bs_classes"])),
                   ue_classes=json.loads(str(d["ue_classes"])),
                   bs_class=d["bs_class"].tolist(), ue_class=d["ue_class"].tolist())
    for k in range(len(d["seeds"])):
        core = port.build(d["bs_xy"], d["xy"].shape[2], int(d["seeds"][k]), 0.0, classes=classes)
        got = []
        port.run_driver(core, 2, 20, on_step=lambda ep, s, c: got.append(c.snapshot()))
        for s, (xy, srv, rate, util, met) in enumerate(got):
            assert xy == [tuple(v) for v in d["xy"][k, s].tolist()]
            assert srv == d["serving"][k, s].tolist()
            assert rate == d["rate"][k, s].tolist()
            np.testing.assert_array_equal(util, d["util"][k, s])


def test_mixed_scenario_is_the_fixture_mix():
    """mobile-large-mixed-v0 (the registered heterogeneous workload) carries the parameter
    classes and class assignment of the reference fixture large_mixed, on the large layout."""
    import json
    from mobile_env.scenarios import registry
    d = load("large_mixed")
    c = registry.spec("mobile-large-mixed-v0")["classes"]
    assert c["bs_classes"] == json.loads(str(d["bs_classes"]))
    assert c["ue_classes"] == json.loads(str(d["ue_classes"]))
    assert c["bs_class"] == d["bs_class"].tolist() and c["ue_class"] == d["ue_class"].tolist()
    assert registry.LAYOUTS["large"]["bs"] == d["bs_xy"].tolist()


def test_velocity_15_integer_step_matches_reference_expression():
    """The kernels' integer movement at velocity 1.5 (step_v15 in mev_step.hip: arrival at
    d2 <= 2; else per axis sgn(dx) [8 dx^2 > dy^2], and on an axis |step| 2 from an even
    coordinate, 1 from an odd one) equals movement.py:49-62's float64 expression
    np.round(position + velocity * v / norm(v)) for every displacement on a 200 x 200 map, at
    positions of both parities and at the map's edges."""
    d = np.arange(-199, 200)
    dx, dy = (a.ravel() for a in np.meshgrid(d, d, indexing="ij"))
    d2 = dx * dx + dy * dy
    keep = d2 > 2
    dx, dy, d2 = dx[keep], dy[keep], d2[keep]
    v = np.stack([dx, dy], 1)
    norm = np.sqrt(d2.astype(np.float64))  # == np.linalg.norm of each integer 2-vector
    for px, py in ((0, 1), (1, 0), (100, 101), (198, 199), (199, 198)):
        ref = np.round(np.array([px, py]) + 1.5 * v / norm[:, None]).astype(np.int64)
        ax2, ay2 = dx * dx, dy * dy
        sx = (8 * ax2 > ay2).astype(np.int64) + ((dy == 0) & (px % 2 == 0))
        sy = (8 * ay2 > ax2).astype(np.int64) + ((dx == 0) & (py % 2 == 0))
        got = np.stack([px + np.where(dx < 0, -sx, sx), py + np.where(dy < 0, -sy, sy)], 1)
        np.testing.assert_array_equal(got, ref, err_msg=f"position {(px, py)}")
    # the expression's own per-UE form (movement.py:58-60) on a sample agrees with the batch form
    rng = np.random.default_rng(0)
    for _ in range(200):
        pos = rng.integers(0, 200, size=2)
        wp = rng.integers(0, 200, size=2)
        vv = wp - pos
        if np.linalg.norm(vv) <= 1.5:
            continue
        one = np.round(pos + 1.5 * vv / np.linalg.norm(vv)).astype(int)
        n2 = float(np.sqrt(float(vv @ vv)))
        assert tuple(one) == tuple(np.round(pos + 1.5 * vv / n2).astype(int))


def test_reference_channel_tables_share_tie_free(golden_dir):
    """The LDS rollouts' fast ResourceFair share rint(full * fl(100 / n)) equals the reference's
    rint(fl(full / n) * 100) (base.py:435) for every entry of both reference channel tables and
    every share count n <= 1024 -- the exhaustive condition under which mev_create selects the
    tie-free two-group / block kernels (mev_share_tie_free; the GPU tests check the flag)."""
    for name in ("channel_default", "channel_notebook"):
        r = np.load(f"{golden_dir}/{name}.npz")["rate"]
        for n in range(1, 1025):
            np.testing.assert_array_equal(np.rint(r * (100.0 / n)), np.rint((r / n) * 100.0),
                                          err_msg=f"{name} n={n}")


@pytest.mark.parametrize("name", WIDE_FIXTURES)
def test_vec_oracle_matches_wide_fixture(name):
    """Maps wider than 200 (1,500^2 / 4,096^2, stations beyond the map's edge included), the
    tx = 55 channel, per-env layouts on a 4,096 map, U = 100, parameter classes on a 4,096 map
    and 30 distinct per-UE velocities with a per-UE snr_tr spread: the oracle reproduces the
    reference's fixtures (make_golden.py --wide) bit for bit -- positions (the int(W u)
    waypoint draws at W = 4,096, the float step of velocities 1.5 to 60), serving stations,
    rates (the tx 55 channel chain), utilities, metrics."""
    from helpers import wide_oracle
    d = load(name)
    ob = wide_oracle(d)
    for s in range(d["xy"].shape[1]):
        o = ob.step()
        np.testing.assert_array_equal(o["xy"], d["xy"][:, s], err_msg=f"step {s}")
        np.testing.assert_array_equal(o["serving"], d["serving"][:, s], err_msg=f"step {s}")
        np.testing.assert_array_equal(o["rate"], d["rate"][:, s], err_msg=f"step {s}")
        act = ~np.isnan(d["util"][:, s])
        np.testing.assert_array_equal(np.isnan(o["util"]), ~act)
        np.testing.assert_array_equal(o["util"][act], d["util"][:, s][act])
        np.testing.assert_array_equal(o["metrics"][:, :3], d["metrics"][:, s, :3])
        np.testing.assert_allclose(o["metrics"][:, 3], d["metrics"][:, s, 3], rtol=1e-12)


def test_channel_table_tx55_matches_reference(golden_dir):
    """The tx = 55 channel (the wide-map fixtures' stations) at every integer d2 up to its
    d2max = 149,716 (d2max + 1 not connectable): the oracle's table is the reference's."""
    c = np.load(f"{golden_dir}/channel_tx55.npz")
    p = OracleParams(width=4096, height=4096, bs={"bw": 9e6, "freq": 2500, "tx": 55,
                                                  "height": 50})
    d2max, rate = channel_table(p)
    assert d2max == int(c["d2max"]) == 149716
    np.testing.assert_array_equal(rate, c["rate"])
