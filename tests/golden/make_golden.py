"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Runs ONLY in the development container, where the read-only reference checkout exists at
/root/reference. Nothing on the GPU box runs this script; the tests there read the committed
.npz/.json files it produced. The reference package is imported (never copied) with three
stub modules for its render-only / geometry dependencies that are absent from the image:

* ``pygame``            -- rendering only (reference base.py:12,15)
* ``shapely.geometry``  -- ``Point(x, y).distance`` = sqrt(dx^2 + dy^2) on the integer
                           coordinates produced by entities.py:24-26,52-54 (GEOS computes the
                           same IEEE value for integer inputs; validated by the two notebook
                           snapshots, which the reference reproduces bit-for-bit with this stub)
* ``svgpath2mpl``       -- BS glyph for rendering only (reference util.py:4,24)

The per-step JSON dump of the reference (base.py:261,298-349) is disabled and the process runs
from a scratch directory. Usage:  python tests/golden/make_golden.py [--extra | --knobs]
"""
from __future__ import annotations

import json
import math
import os
import random
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
LAYOUTS = os.path.join(HERE, "..", "..", "mobile-env-gan_amd", "mobile_env", "scenarios",
                       "layouts.json")
METRIC_NAMES = ["number connections", "number connected", "mean utility", "mean datarate"]


def _install_stubs():
    import matplotlib
    matplotlib.use("Agg")
    from matplotlib.path import Path

    pg = types.ModuleType("pygame")
    pg.Surface = object
    sys.modules["pygame"] = pg

    class Point:
        def __init__(self, x, y):
            self.x = float(x)
            self.y = float(y)

        def distance(self, other):
            dx = self.x - other.x
            dy = self.y - other.y
            return math.sqrt(dx * dx + dy * dy)

    shp = types.ModuleType("shapely")
    geom = types.ModuleType("shapely.geometry")
    geom.Point = Point
    shp.geometry = geom
    sys.modules["shapely"] = shp
    sys.modules["shapely.geometry"] = geom

    svg = types.ModuleType("svgpath2mpl")
    svg.parse_path = lambda s: Path(np.zeros((3, 2)))
    sys.modules["svgpath2mpl"] = svg


def _import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    from mobile_env.core import base as ref_base  # noqa: E402
    from mobile_env.core.entities import BaseStation, UserEquipment  # noqa: E402
    from mobile_env.core.channels import OkumuraHata  # noqa: E402
    from mobile_env.scenarios import custom as ref_custom  # noqa: E402

    # disable per-step disk dump (base.py:261)
    ref_base.MComCore.save_layout_and_data_rates = lambda self, e, s: None
    return ref_base, BaseStation, UserEquipment, OkumuraHata, ref_custom


def _record_step(env, users):
    """Snapshot the reference env state after one step() call."""
    U = len(users)
    xy = np.array([[int(ue.x), int(ue.y)] for ue in users], dtype=np.int64)
    serving = np.full(U, -1, dtype=np.int64)
    for (bs, ue) in env.bs2ue_dataRates.keys():
        serving[ue.ue_id] = bs.bs_id
    rate = np.array([float(env.allUserDataRates.get(ue, 0.0)) for ue in users])
    util = np.array([float(env.ue_utilities[ue]) if ue in env.ue_utilities else np.nan
                     for ue in users])
    met = np.array([float(env.monitor.scalar_results[n][-1]) for n in METRIC_NAMES])
    return xy, serving, rate, util, met


def _make_fixed_core(ref_base, BaseStation, UserEquipment):
    class FixedCore(ref_base.MComCore):
        """MComCore over a fixed station list, with the episode bookkeeping that the only
        runnable scenario performs after reset (custom.py:53-62): activeUsers = UEs with
        startTime <= 0 sorted by id, and the history lists initialised."""

        def reset(self, *, seed=None):
            super().reset(seed=seed)
            self.activeUsers = sorted(
                [ue for ue in self.userDict.values() if ue.startTime <= 0],
                key=lambda ue: ue.ue_id)
            self.users_dataRateList = {ue.ue_id: [] for ue in self.userDict.values()}
            self.users_trajectoryList = {ue.ue_id: [] for ue in self.userDict.values()}

    def build(bs_xy, num_ues, seed, bs_params=None, ue_params=None, extra=None):
        cfg = FixedCore.default_config()
        if bs_params:
            cfg["bs"].update(bs_params)
        if ue_params:
            cfg["ue"].update(ue_params)
        stations = [BaseStation(i, (int(x), int(y)), **cfg["bs"]) for i, (x, y) in enumerate(bs_xy)]
        users = [UserEquipment(i, **cfg["ue"]) for i in range(num_ues)]
        config = {"seed": seed, "bs": cfg["bs"], "ue": cfg["ue"]}
        if extra:
            config.update(extra)
        return FixedCore(stations, users, config), users

    return build


def run_episodes(env, users, episodes, steps):
    """collectData2.ipynb driver loop: reset(); step(epoch, s) for s in range(steps)."""
    rec = {k: [] for k in ("init_xy", "xy", "serving", "rate", "util", "metrics")}
    for ep in range(episodes):
        env.reset()
        rec["init_xy"].append([[int(ue.x), int(ue.y)] for ue in users])
        for s in range(steps):
            env.step(ep, s)
            xy, srv, rate, util, met = _record_step(env, users)
            rec["xy"].append(xy)
            rec["serving"].append(srv)
            rec["rate"].append(rate)
            rec["util"].append(util)
            rec["metrics"].append(met)
    return {k: np.asarray(v) for k, v in rec.items()}


def rate_table(OkumuraHata, bs_params, ue_params, d2_hi):
    """Reference channel chain evaluated at every integer squared distance d2 in [0, d2_hi]:
    (snr, datarate) through OkumuraHata.power_loss / Channel.calculateSNR / Channel.datarate
    (channels.py:24-27,78-83,133-146), using duck-typed entities whose point distance is
    sqrt(d2)."""

    class _P:
        def __init__(self, d2):
            self.d2 = d2

        def distance(self, other):
            return math.sqrt(other.d2)

    class _BS:
        point = _P(0)
        bw = bs_params["bw"]
        frequency = bs_params["freq"]
        tx_power = bs_params["tx"]
        height = bs_params["height"]

    class _UE:
        height = ue_params["height"]
        noise = ue_params["noise"]
        snr_threshold = ue_params["snr_tr"]

    ch = OkumuraHata()
    ue = _UE()
    snr = np.empty(d2_hi + 1)
    rate = np.empty(d2_hi + 1)
    for d2 in range(d2_hi + 1):
        ue.point = _P(d2)
        s = ch.calculateSNR(_BS, ue)
        snr[d2] = float(s)
        rate[d2] = float(ch.datarate(_BS, ue, s))
    return snr, rate


def _build_mixed(ref_base, BaseStation, UserEquipment, bs_xy, bs_params, ue_params, seed):
    """FixedCore over stations / UEs that each carry their OWN parameters (entities.py:7-22,
    33-45): bs_params / ue_params are lists of kwargs per entity."""
    build = _make_fixed_core(ref_base, BaseStation, UserEquipment)
    env, _ = build(bs_xy, len(ue_params), seed)  # for the FixedCore class and config
    stations = [BaseStation(i, (int(x), int(y)), **bs_params[i]) for i, (x, y) in enumerate(bs_xy)]
    users = [UserEquipment(i, **ue_params[i]) for i in range(len(ue_params))]
    return type(env)(stations, users, {"seed": seed}), users


def extra_fixtures(ref_base, BaseStation, UserEquipment):
    """Round-2 fixtures: per-env 128-station layouts at 1024 UEs (the layout mode of
    mobile-custom-128x1024-v0), and heterogeneous per-station / per-UE parameters."""
    out = {}
    build = _make_fixed_core(ref_base, BaseStation, UserEquipment)
    # -- per-env 128 x 1024: 3 envs, each its own uniform-integer layout (the registry's
    #    synthetic layouts: torch.Generator seeded with the env seed, randint(0, 200)), 3 steps
    import torch
    seeds = [2024, 2025, 2026]
    lays, runs = [], []
    for sd in seeds:
        g = torch.Generator()
        g.manual_seed(sd)
        bs = torch.randint(0, 200, (128, 2), generator=g, dtype=torch.int32).numpy()
        env, users = build(bs.tolist(), 1024, sd, ue_params={"velocity": 10})
        env.reset()
        init = [[int(ue.x), int(ue.y)] for ue in users]
        recs = []
        for s in range(3):
            env.step(0, s)
            recs.append(_record_step(env, users))
        lays.append(bs)
        runs.append((init, recs))
        print("custom128x1024_perenv seed", sd)
    out["custom128x1024_perenv"] = dict(
        bs_xy=np.asarray(lays, dtype=np.int64), seeds=np.asarray(seeds), velocity=np.float64(10),
        init_xy=np.asarray([[r[0]] for r in runs]),
        **{k: np.asarray([[rec[i] for rec in r[1]] for r in runs])
           for i, k in enumerate(("xy", "serving", "rate", "util", "metrics"))})

    # -- heterogeneous parameters on the large layout: station tx / height / bw / freq by station
    #    index, UE velocity / snr_tr / noise / height by UE index; 3 seeds x 2 episodes
    layouts = json.load(open(LAYOUTS))
    lay = layouts["large"]
    B, U = len(lay["bs"]), lay["num_ues"]
    bs_classes = [{"bw": 9e6, "freq": 2500, "tx": 40, "height": 50},
                  {"bw": 9e6, "freq": 2500, "tx": 30, "height": 50},
                  {"bw": 5e6, "freq": 1800, "tx": 35, "height": 30}]
    ue_classes = [{"velocity": 1.5, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.6},
                  {"velocity": 10, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.8},
                  {"velocity": 3, "snr_tr": 1e-7, "noise": 2e-9, "height": 1.5}]
    bs_cls = [i % 3 for i in range(B)]
    ue_cls = [(i * 7) % 3 for i in range(U)]
    runs = []
    hseeds = [2024, 5, 77]
    for sd in hseeds:
        env, users = _build_mixed(ref_base, BaseStation, UserEquipment, lay["bs"],
                                  [bs_classes[c] for c in bs_cls],
                                  [ue_classes[c] for c in ue_cls], sd)
        runs.append(run_episodes(env, users, episodes=2, steps=20))
    out["large_mixed"] = dict(
        bs_xy=np.asarray(lay["bs"], dtype=np.int64), seeds=np.asarray(hseeds),
        velocity=np.float64(np.nan),
        bs_class=np.asarray(bs_cls), ue_class=np.asarray(ue_cls),
        bs_classes=json.dumps(bs_classes), ue_classes=json.dumps(ue_classes),
        **{k: np.stack([r[k] for r in runs]) for k in runs[0]})
    return out


def run_until_done(env, users, episodes):
    """The driver loop with the episode ending where the reference says it does:
    reset(); step() while not time_is_up (base.py:407-409: time >= min(EP_MAX_TIME,
    max_departure))."""
    rec = {k: [] for k in ("init_xy", "xy", "serving", "rate", "util", "metrics")}
    lens = []
    for ep in range(episodes):
        env.reset()
        rec["init_xy"].append([[int(ue.x), int(ue.y)] for ue in users])
        s = 0
        while not env.time_is_up:
            env.step(ep, s)
            xy, srv, rate, util, met = _record_step(env, users)
            for k, v in zip(("xy", "serving", "rate", "util", "metrics"), (xy, srv, rate, util, met)):
                rec[k].append(v)
            s += 1
        lens.append(s)
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["episode_len"] = np.asarray(lens)
    return out


# Reference config knobs the engine lowers into kernel branches (MComCore.default_config,
# base.py:103-153, deep-merged at base.py:47): name -> (layout, num_ues, velocity, seeds,
# episodes, config overrides). "block" variants use 96 UEs (U > 64: the one-workgroup-per-env
# kernel).
KNOBS = {
    "knob_noreseed_large": ("large", None, None, [2024, 99], 3,
                            {"movement_params": {"reset_rng_episode": False}}),
    "knob_noreseed_small_v10": ("small", None, 10, [5, 2024], 3,
                                {"movement_params": {"reset_rng_episode": False}}),
    "knob_ept12_large": ("large", None, None, [2024, 7], 3, {"EP_MAX_TIME": 12}),
    "knob_ept30_medium": ("medium", None, None, [2024, 11], 2, {"EP_MAX_TIME": 30}),
    "knob_ep15_medium_v10": ("medium", None, 10, [3, 2024], 3,
                             {"arrival_params": {"ep_time": 15}}),
    "knob_util_large_v10": ("large", None, 10, [2024, 31], 2,
                            {"utility_params": {"lower": -10, "upper": 15, "coeffs": (5, 1, 2)}}),
    "knob_block_noreseed": ("large", 96, 10, [2024, 8], 3,
                            {"movement_params": {"reset_rng_episode": False}}),
    "knob_block_ept12": ("large", 96, 10, [2024], 3, {"EP_MAX_TIME": 12}),
    "knob_block_util": ("large", 96, 10, [17], 2,
                        {"utility_params": {"lower": -10, "upper": 15, "coeffs": (5, 1, 2)}}),
}


def knob_fixtures(ref_base, BaseStation, UserEquipment):
    build = _make_fixed_core(ref_base, BaseStation, UserEquipment)
    layouts = json.load(open(LAYOUTS))
    defaults = ref_base.MComCore.default_config()
    out = {}
    for name, (lay_name, nue, vel, seeds, episodes, cfg) in KNOBS.items():
        lay = layouts[lay_name]
        U = nue or lay["num_ues"]
        runs = []
        for seed in seeds:
            env, users = build(lay["bs"], U, seed,
                               ue_params={"velocity": vel} if vel is not None else None,
                               extra=json.loads(json.dumps(cfg)))
            runs.append(run_until_done(env, users, episodes))
        out[name] = dict(
            bs_xy=np.asarray(lay["bs"], dtype=np.int64), seeds=np.asarray(seeds, dtype=np.int64),
            velocity=np.float64(vel if vel is not None else defaults["ue"]["velocity"]),
            config=json.dumps(cfg),
            **{k: np.stack([r[k] for r in runs]) for k in runs[0]})
        print(name, "episode lengths", runs[0]["episode_len"].tolist())
    return out


def main_knobs():
    ref_base, BaseStation, UserEquipment, OkumuraHata, ref_custom = _import_reference()
    scratch = tempfile.mkdtemp(prefix="mev_golden_")
    os.chdir(scratch)
    for name, arrs in knob_fixtures(ref_base, BaseStation, UserEquipment).items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print("wrote", name)


def main_extra():
    ref_base, BaseStation, UserEquipment, OkumuraHata, ref_custom = _import_reference()
    scratch = tempfile.mkdtemp(prefix="mev_golden_")
    os.chdir(scratch)
    for name, arrs in extra_fixtures(ref_base, BaseStation, UserEquipment).items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print("wrote", name)


def main():
    ref_base, BaseStation, UserEquipment, OkumuraHata, ref_custom = _import_reference()
    scratch = tempfile.mkdtemp(prefix="mev_golden_")
    os.chdir(scratch)
    build = _make_fixed_core(ref_base, BaseStation, UserEquipment)
    layouts = json.load(open(LAYOUTS))
    defaults = ref_base.MComCore.default_config()
    out = {}

    # -- fixed-layout scenarios (build-defined layouts), several config seeds, 2 episodes ----------
    plans = [
        ("small", None, [2024, 7, 123]),
        ("medium", None, [2024, 11]),
        ("large", None, [2024, 99]),
        ("small_v10", ("small", 10), [5, 2024]),
        ("large_v10", ("large", 10), [31]),
    ]
    for name, variant, seeds in plans:
        base_name, vel = variant if variant else (name, None)
        lay = layouts[base_name]
        runs = []
        for seed in seeds:
            ue_p = {"velocity": vel} if vel is not None else None
            env, users = build(lay["bs"], lay["num_ues"], seed, ue_params=ue_p)
            runs.append(run_episodes(env, users, episodes=2, steps=20))
        out[name] = dict(
            bs_xy=np.asarray(lay["bs"], dtype=np.int64),
            seeds=np.asarray(seeds, dtype=np.int64),
            velocity=np.float64(vel if vel is not None else defaults["ue"]["velocity"]),
            **{k: np.stack([r[k] for r in runs]) for k in runs[0]},
        )

    # -- MComCustom (custom.py) with the global `random` seeded: BS layout redrawn per reset -------
    runs, bs_layouts = [], []
    for k in range(8):
        random.seed(k)
        env = ref_custom.MComCustom()
        users = [env.userDict[i] for i in sorted(env.userDict)]
        rec = {n: [] for n in ("init_xy", "xy", "serving", "rate", "util", "metrics")}
        lay_k = []
        for ep in range(2):
            env.reset()
            lay_k.append([[int(bs.point.x), int(bs.point.y)] for bs in env.stationDict.values()])
            rec["init_xy"].append([[int(ue.x), int(ue.y)] for ue in users])
            for s in range(20):
                env.step(ep, s)
                xy, srv, rate, util, met = _record_step(env, users)
                for n, v in zip(("xy", "serving", "rate", "util", "metrics"),
                                (xy, srv, rate, util, met)):
                    rec[n].append(v)
        runs.append({n: np.asarray(v) for n, v in rec.items()})
        bs_layouts.append(lay_k)
    # ragged BS counts (5..10): pad with -1
    bs_pad = np.full((8, 2, 10, 2), -1, dtype=np.int64)
    bs_cnt = np.zeros((8, 2), dtype=np.int64)
    for k, lay_k in enumerate(bs_layouts):
        for ep, lay in enumerate(lay_k):
            bs_pad[k, ep, :len(lay)] = lay
            bs_cnt[k, ep] = len(lay)
    out["mcom_custom"] = dict(bs_xy=bs_pad, bs_count=bs_cnt, random_seeds=np.arange(8),
                              seeds=np.full(8, defaults["seed"]), velocity=np.float64(10),
                              **{k: np.stack([r[k] for r in runs]) for k in runs[0]})

    # -- custom 128 BS x 1024 UE, velocity 10, 3 steps (reference: ~1.5 s/step) --------------------
    bs128 = np.random.default_rng(0).integers(0, 200, size=(128, 2))
    env, users = build(bs128.tolist(), 1024, 2024, ue_params={"velocity": 10})
    env.reset()
    init = [[int(ue.x), int(ue.y)] for ue in users]
    recs = []
    for s in range(3):
        env.step(0, s)
        recs.append(_record_step(env, users))
    out["custom128x1024"] = dict(
        bs_xy=bs128.astype(np.int64), seeds=np.asarray([2024]), velocity=np.float64(10),
        init_xy=np.asarray([[init]]),
        **{k: np.asarray([[r[i] for r in recs]])
           for i, k in enumerate(("xy", "serving", "rate", "util", "metrics"))})

    # -- notebook snapshots (GNN.ipynb:86-93 and :909-1047) -----------------------------------------
    snaps = json.load(open(os.path.join(HERE, "notebook_snapshots.json")))
    nb_bs = snaps["params"]["bs"]
    nb_ue = snaps["params"]["ue"]
    for snap in snaps["snapshots"]:
        env, users = build(snap["bs_xy"], 7, snaps["params"]["seed"], bs_params=nb_bs,
                           ue_params=nb_ue)
        env.reset()
        for s in range(snap["step"] + 1):
            env.step(0, s)
        xy, srv, rate, util, met = _record_step(env, users)
        assert xy.tolist() == snap["ue_xy"], (snap["source"], xy.tolist())
        got = {int(u): (int(srv[u]), float(rate[u])) for u in range(7) if srv[u] >= 0}
        want = {int(e["ue_id"]): (int(e["bs_id"]), float(e["data_rate"])) for e in snap["rates"]}
        assert got == want, (snap["source"], got, want)
    print("notebook snapshots reproduced by the reference: OK")

    # -- channel tables: reference snr/datarate at every integer d2 ---------------------------------
    tables = {}
    for tag, bsp, uep in (("default", defaults["bs"], defaults["ue"]),
                          ("notebook", {**defaults["bs"], **nb_bs}, {**defaults["ue"], **nb_ue})):
        snr, rate = rate_table(OkumuraHata, bsp, uep, 80000)
        conn = snr > uep["snr_tr"]
        d2max = int(np.nonzero(conn)[0].max())
        assert conn[: d2max + 1].all() and not conn[d2max + 1:].any(), "connectivity not a prefix"
        tables[tag] = dict(d2max=np.int64(d2max), rate=rate[: d2max + 1],
                           snr_margin=np.float64(np.min(np.abs(snr / uep["snr_tr"] - 1.0))),
                           bs=json.dumps(bsp), ue=json.dumps(uep))
        print(tag, "d2max", d2max)

    for name, arrs in out.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    for tag, arrs in tables.items():
        np.savez_compressed(os.path.join(HERE, f"channel_{tag}.npz"), **arrs)
    print("wrote", sorted(out) + [f"channel_{t}" for t in tables])


def _build_cfg(ref_base, BaseStation, UserEquipment, bs_xy, bs_params, ue_params, seed, extra):
    """FixedCore over stations / UEs with per-entity kwargs (lists) and config overrides (map
    size: "width" / "height" and movement_params, base.py:104-108,130-134)."""
    build = _make_fixed_core(ref_base, BaseStation, UserEquipment)
    env, _ = build(bs_xy, len(ue_params), seed)  # for the FixedCore class
    stations = [BaseStation(i, (int(x), int(y)), **bs_params[i]) for i, (x, y) in enumerate(bs_xy)]
    users = [UserEquipment(i, **ue_params[i]) for i in range(len(ue_params))]
    cfg = {"seed": seed}
    cfg.update(json.loads(json.dumps(extra)))
    return type(env)(stations, users, cfg), users


def _map_cfg(w, h):
    return {"width": w, "height": h, "movement_params": {"width": w, "height": h}}


# Round-4 fixtures (--wide): maps wider than 200, a tx = 55 channel, stations outside the map,
# per-env layouts, U > 64, heterogeneous classes on a 4,096 map; and per-UE velocities
# (30 distinct values) with a per-UE snr_tr spread. name -> (W, H, layouts [E] of [B][2] or one
# shared [B][2], U, bs kwargs per station (or one dict), ue kwargs per UE (or one dict), seeds,
# episodes)
def wide_plans():
    r = np.random.default_rng(1500)
    lay1500 = r.integers(0, 1500, size=(11, 2)).tolist() + [[1600, 200], [3000, 1400]]
    r = np.random.default_rng(4096)
    lay4096 = r.integers(0, 4096, size=(13, 2)).tolist()
    per_env = [np.random.default_rng(40 + k).integers(0, 4096, size=(9 + 2 * k, 2)).tolist()
               for k in range(3)]
    bs_def = {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50}
    bs55 = dict(bs_def, tx=55)
    ue_def = {"velocity": 1.5, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}
    bs_cls = [dict(bs55), {"bw": 9e6, "freq": 2500, "tx": 45, "height": 50},
              {"bw": 5e6, "freq": 1800, "tx": 50, "height": 30}]
    ue_cls = [dict(ue_def, velocity=60), {"velocity": 40, "snr_tr": 2e-8, "noise": 1e-9,
                                          "height": 1.8},
              {"velocity": 25, "snr_tr": 1e-7, "noise": 2e-9, "height": 1.5}]
    snr_spread = [2e-8, 5e-8, 1e-7, 1e-8]
    return {
        "wide1500": (1500, 1500, lay1500, 30, bs_def, ue_def, [2024, 9], 2),
        "wide4096_tx55": (4096, 4096, lay4096, 30, bs55, dict(ue_def, velocity=60),
                          [2024, 9], 2),
        "wide4096_tx55_perenv": (4096, 4096, per_env, 30, bs55, dict(ue_def, velocity=60),
                                 [3, 4, 5], 2),
        "wide1500_block": (1500, 1500, lay1500, 100, bs_def, dict(ue_def, velocity=10), [5],
                           2),
        "wide4096_mixed": (4096, 4096, lay4096, 30, [bs_cls[i % 3] for i in range(13)],
                           [ue_cls[(i * 7) % 3] for i in range(30)], [3, 2024], 2),
        # per-UE velocities (all distinct) and snr_tr from a 4-value spread, default map
        "velocities_large": (200, 200, None, 30, bs_def,
                             [dict(ue_def, velocity=1.0 + 0.75 * i,
                                   snr_tr=snr_spread[(i * 3) % 4]) for i in range(30)],
                             [2024, 77], 2),
    }


def wide_fixtures(ref_base, BaseStation, UserEquipment, OkumuraHata):
    layouts = json.load(open(LAYOUTS))
    out = {}
    for name, (W, H, lay, U, bsp, uep, seeds, episodes) in wide_plans().items():
        if lay is None:
            lay = layouts["large"]["bs"]
        per_env = isinstance(lay[0][0], list)
        runs = []
        for k, sd in enumerate(seeds):
            L = lay[k] if per_env else lay
            bl = bsp if isinstance(bsp, list) else [bsp] * len(L)
            ul = uep if isinstance(uep, list) else [uep] * U
            env, users = _build_cfg(ref_base, BaseStation, UserEquipment, L, bl, ul, sd,
                                    _map_cfg(W, H))
            runs.append(run_episodes(env, users, episodes=episodes, steps=20))
        rec = {k: np.stack([r[k] for r in runs]) for k in runs[0]}
        if per_env:
            Bm = max(len(x) for x in lay)
            bs_xy = np.full((len(lay), Bm, 2), 0, dtype=np.int64)
            for k, x in enumerate(lay):
                bs_xy[k, :len(x)] = x
            extra = dict(bs_xy=bs_xy, bs_count=np.asarray([len(x) for x in lay]))
        else:
            extra = dict(bs_xy=np.asarray(lay, dtype=np.int64))
        out[name] = dict(
            width=np.int64(W), height=np.int64(H), seeds=np.asarray(seeds, dtype=np.int64),
            bs_params=json.dumps(bsp), ue_params=json.dumps(uep),
            velocity=np.float64(uep["velocity"] if isinstance(uep, dict) else np.nan),
            **extra, **rec)
        print(name, "serving share", float((rec["serving"] >= 0).mean()))
    # the tx = 55 channel at every integer d2 up to its d2max (+1: not connectable)
    bsp = wide_plans()["wide4096_tx55"][4]
    uep = {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}
    hi = 2 * 1023 * 1023
    lo, top = 0, hi
    while lo < top:  # the last connectable d2 (connectivity is a prefix: checked below)
        mid = (lo + top + 1) // 2
        snr, _ = rate_table_range(OkumuraHata, bsp, uep, mid, mid)
        if snr[0] > uep["snr_tr"]:
            lo = mid
        else:
            top = mid - 1
    d2max = lo
    snr, rate = rate_table_range(OkumuraHata, bsp, uep, 0, d2max + 1)
    conn = snr > uep["snr_tr"]
    assert conn[: d2max + 1].all() and not conn[d2max + 1:].any(), "connectivity not a prefix"
    out["channel_tx55"] = dict(d2max=np.int64(d2max), rate=rate[: d2max + 1],
                               snr_margin=np.float64(np.min(np.abs(snr / uep["snr_tr"] - 1.0))),
                               bs=json.dumps(bsp), ue=json.dumps(uep))
    print("channel_tx55 d2max", d2max)
    return out


def rate_table_range(OkumuraHata, bs_params, ue_params, d2_lo, d2_hi):
    """rate_table over [d2_lo, d2_hi] only."""

    class _P:
        def __init__(self, d2):
            self.d2 = d2

        def distance(self, other):
            return math.sqrt(other.d2)

    class _BS:
        point = _P(0)
        bw = bs_params["bw"]
        frequency = bs_params["freq"]
        tx_power = bs_params["tx"]
        height = bs_params["height"]

    class _UE:
        height = ue_params["height"]
        noise = ue_params["noise"]
        snr_threshold = ue_params["snr_tr"]

    ch = OkumuraHata()
    ue = _UE()
    n = d2_hi - d2_lo + 1
    snr = np.empty(n)
    rate = np.empty(n)
    for i in range(n):
        ue.point = _P(d2_lo + i)
        s = ch.calculateSNR(_BS, ue)
        snr[i] = float(s)
        rate[i] = float(ch.datarate(_BS, ue, s))
    return snr, rate


def main_wide():
    ref_base, BaseStation, UserEquipment, OkumuraHata, ref_custom = _import_reference()
    scratch = tempfile.mkdtemp(prefix="mev_golden_")
    os.chdir(scratch)
    for name, arrs in wide_fixtures(ref_base, BaseStation, UserEquipment, OkumuraHata).items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print("wrote", name)


if __name__ == "__main__":
    # --extra: only the round-2 fixtures (per-env 128 x 1024, heterogeneous parameters);
    # --knobs: only the round-3 config-knob fixtures (KNOBS); --wide: only the round-4 wide-map /
    # tx 55 / per-UE velocity fixtures (wide_plans)
    if "--extra" in sys.argv[1:]:
        main_extra()
    elif "--knobs" in sys.argv[1:]:
        main_knobs()
    elif "--wide" in sys.argv[1:]:
        main_wide()
    else:
        main()
