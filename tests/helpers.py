"""Shared helpers for the parity tests: load golden fixtures, build engines / oracles."""
from __future__ import annotations

import json
import os

import numpy as np

from conftest import GOLDEN

DEFAULT_BS = {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50}
DEFAULT_UE = {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}

# fixture name -> (num_ues, per-env ragged layout?)
FIXTURES = ("small", "medium", "large", "small_v10", "large_v10", "mcom_custom",
            "custom128x1024", "custom128x1024_perenv")
# reference config knobs (tests/golden/make_golden.py --knobs: KNOBS)
KNOB_FIXTURES = ("knob_noreseed_large", "knob_noreseed_small_v10", "knob_ept12_large",
                 "knob_ept30_medium", "knob_ep15_medium_v10", "knob_util_large_v10",
                 "knob_block_noreseed", "knob_block_ept12", "knob_block_util")


def load(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return {k: d[k] for k in d.files}


def snapshots():
    return json.load(open(os.path.join(GOLDEN, "notebook_snapshots.json")))


def layout_for(d, episode=0):
    """(bs_xy, bs_count) for the engine/oracle: [B,2] shared, or [E,B,2] + counts."""
    if "bs_count" in d:
        return d["bs_xy"][:, episode], d["bs_count"][:, episode]
    return d["bs_xy"], None


def make_oracle(d, bs=None, ue=None):
    from oracle.vec import OracleBatch, OracleParams
    p = OracleParams(velocity=float(d["velocity"]), bs=dict(bs or DEFAULT_BS),
                     ue=dict(ue or DEFAULT_UE))
    bs_xy, cnt = layout_for(d)
    return OracleBatch(p, bs_xy, d["xy"].shape[2], d["seeds"], bs_count=cnt)


def make_engine(d, device="cuda", bs=None, ue=None, stream_split=0, draw_table=-1, fuse_steps=0,
                **kw):
    from mobile_env.core.engine import EngineParams, StepEngine
    bs_xy, cnt = layout_for(d)
    E = len(d["seeds"])
    U = d["xy"].shape[2]
    B = bs_xy.shape[-2]
    p = EngineParams(num_envs=E, num_ues=U, num_bs=B, velocity=float(d["velocity"]),
                     bs=dict(bs or DEFAULT_BS), ue=dict(ue or DEFAULT_UE),
                     stream_split=stream_split, draw_table=draw_table,
                     fuse_steps=fuse_steps)
    return StepEngine(p, bs_xy, d["seeds"], bs_count=cnt, device=device, **kw)


def synced_pcg(eng):
    """The engine's pcg rows with every stream state materialised (mev_sync_stream_state: the
    kernels leave the state column to the draw table while an episode's draws stay inside it),
    so launch shapes with and without the table compare equal."""
    eng.sync_stream_state()
    return eng.pcg


def knob_config(d):
    """The reference config overrides a knob fixture was generated with."""
    return json.loads(str(d["config"]))


def knob_oracle_params(d):
    """OracleParams of a knob fixture, read from its reference config dict (the keys of
    MComCore.default_config, base.py:103-153)."""
    from oracle.vec import OracleParams
    cfg = knob_config(d)
    up = cfg.get("utility_params", {})
    return OracleParams(
        velocity=float(d["velocity"]), ep_max_time=int(cfg.get("EP_MAX_TIME", 20)),
        arrival_ep_time=int(cfg.get("arrival_params", {}).get("ep_time", 20)),
        lower=up.get("lower", -20), upper=up.get("upper", 20),
        coeffs=tuple(up.get("coeffs", (10, 0, 10))),
        movement_reseed=bool(cfg.get("movement_params", {}).get("reset_rng_episode", True)))


def knob_params(d, num_envs=None):
    """EngineParams of a knob fixture lowered the way the facade lowers a reference config:
    MComCore(stations, users, config) (deep merge into default_config, plugin objects built
    from config[k] / config[k + "_params"], base.py:47-61) -> lowering.lower. The episode draw
    table is left automatic (the facade itself turns it off)."""
    from mobile_env.core import lowering
    from mobile_env.core.base import MComCore
    from mobile_env.core.entities import BaseStation, UserEquipment
    base = MComCore.default_config()
    U = d["xy"].shape[-2]
    stations = [BaseStation(i, (int(x), int(y)), **base["bs"])
                for i, (x, y) in enumerate(d["bs_xy"])]
    users = [UserEquipment(i, **dict(base["ue"], velocity=float(d["velocity"])))
             for i in range(U)]
    core = MComCore(stations, users, config=knob_config(d))
    p = lowering.lower(num_envs=num_envs or len(d["seeds"]), stations=stations, users=users,
                       arrival=core.arrivalModel, channel=core.channelModel,
                       scheduler=core.schedulerModel, movement=core.movementModel,
                       utility=core.utilityModel, ep_max_time=core.EP_MAX_TIME,
                       first_step_active=True)
    p.draw_table = -1
    return p


def knob_engine(d, num_envs=None, device="cuda", rate64=False, util64=False, metrics=False,
                **launch):
    """StepEngine over a knob fixture: env i runs the fixture's seed i % n (replicas give
    batch sizes that select the large-batch kernels); `launch` sets EngineParams fields."""
    from mobile_env.core.engine import StepEngine
    p = knob_params(d, num_envs)
    for k, v in launch.items():
        setattr(p, k, v)
    E = p.num_envs
    seeds = np.asarray(d["seeds"])[np.arange(E) % len(d["seeds"])]
    return StepEngine(p, d["bs_xy"], seeds, device=device, rate64=rate64, util64=util64,
                      metrics=metrics)


def knob_done(d):
    """done flag of every fixture step (the last step of each episode)."""
    lens = np.asarray(d["episode_len"])[0]
    ends = np.cumsum(lens) - 1
    done = np.zeros(int(lens.sum()), dtype=bool)
    done[ends] = True
    return done


# Round-4 reference fixtures (tests/golden/make_golden.py --wide): maps wider than 200, a tx 55
# channel, per-env layouts, U > 64, classes on a 4,096 map, per-UE velocities
WIDE_FIXTURES = ("wide1500", "wide4096_tx55", "wide4096_tx55_perenv", "wide1500_block",
                 "wide4096_mixed", "velocities_large")


def fixture_entities(d):
    """Parameters of a --wide fixture: (bs dict, ue dict incl. velocity) when every entity has
    the same, else the per-entity lists as parameter classes {bs_classes, ue_classes, bs_class,
    ue_class} (unique tuples in first-appearance order)."""
    bsp, uep = json.loads(str(d["bs_params"])), json.loads(str(d["ue_params"]))

    def classes(lst, keys):
        uniq, idx = [], []
        for x in lst:
            t = tuple(x[k] for k in keys)
            if t not in uniq:
                uniq.append(t)
            idx.append(uniq.index(t))
        return [dict(zip(keys, t)) for t in uniq], idx

    out = {}
    if isinstance(bsp, list):
        out["bs_classes"], out["bs_class"] = classes(bsp, ("bw", "freq", "tx", "height"))
        if len(out["bs_classes"]) == 1:
            del out["bs_classes"], out["bs_class"]
        bsp = bsp[0]
    if isinstance(uep, list):
        # channel classes over (snr_tr, noise, height); velocities per UE (mev_params.ue_velocity)
        vel = [float(u["velocity"]) for u in uep]
        out["ue_classes"], out["ue_class"] = classes(uep, ("snr_tr", "noise", "height"))
        for c in out["ue_classes"]:
            c["velocity"] = vel[out["ue_class"].index(out["ue_classes"].index(c))]
        if len(out["ue_classes"]) == 1:
            del out["ue_classes"], out["ue_class"]
        if len(set(vel)) > 1:
            out["ue_velocity"] = vel
        uep = uep[0]
    return bsp, uep, out


def wide_oracle(d, table=None):
    from oracle.vec import OracleBatch, OracleParams
    bsp, uep, cls = fixture_entities(d)
    p = OracleParams(width=int(d["width"]), height=int(d["height"]),
                     velocity=float(uep["velocity"]), bs=dict(bsp),
                     ue={k: uep[k] for k in ("snr_tr", "noise", "height")}, **cls)
    cnt = d["bs_count"] if "bs_count" in d else None
    return OracleBatch(p, d["bs_xy"], d["xy"].shape[2], d["seeds"], bs_count=cnt, table=table)


def wide_engine_params(d, **kw):
    from mobile_env.core.engine import EngineParams
    bsp, uep, cls = fixture_entities(d)
    return EngineParams(num_envs=len(d["seeds"]), num_ues=int(d["xy"].shape[2]),
                        num_bs=int(d["bs_xy"].shape[-2]), width=int(d["width"]),
                        height=int(d["height"]), velocity=float(uep["velocity"]),
                        bs=dict(bsp), ue={k: uep[k] for k in ("snr_tr", "noise", "height")},
                        **cls, **kw)


RTOL = 1e-5  # north_star: fp32 data-rates / utilities within 1e-5 relative, atol 0 everywhere


def assert_step_vs_oracle(o, obs, serving, reward, done, env_idx=None, W=200, H=200, where=""):
    """One step's outputs of the kernels ([E', U, 4] obs, [E', U] serving, [E'] reward / done,
    numpy) against the oracle's step `o` for envs `env_idx` (None: all): positions and serving
    bit-exact, done exact, float32 rate / utility / reward within RTOL relative with atol 0 --
    near zero too: the float32 utility runs only where it holds relative precision (default
    parameters; otherwise the exact table, KParams::util_exact) and rewards whose fixed-point
    sum could miss 1e-5 relative are re-formed from the exact utilities (the reward guard)."""
    sel = slice(None) if env_idx is None else env_idx
    xy = o["xy"][sel]
    np.testing.assert_array_equal(obs[..., 0], xy[..., 0].astype(np.float32)
                                  * np.float32(1.0 / W), err_msg=f"x {where}")
    np.testing.assert_array_equal(obs[..., 1], xy[..., 1].astype(np.float32)
                                  * np.float32(1.0 / H), err_msg=f"y {where}")
    np.testing.assert_array_equal(serving, o["serving"][sel], err_msg=f"serving {where}")
    np.testing.assert_allclose(obs[..., 2], o["rate"][sel].astype(np.float32), rtol=RTOL,
                               atol=0, err_msg=f"rate {where}")
    util = o["util"][sel]
    act = ~np.isnan(util)
    np.testing.assert_allclose(obs[..., 3][act], util[act].astype(np.float32), rtol=RTOL,
                               atol=0, err_msg=f"utility {where}")
    np.testing.assert_allclose(reward, o["metrics"][sel, 2], rtol=RTOL, atol=0,
                               err_msg=f"reward {where}")
    np.testing.assert_array_equal(np.asarray(done).astype(bool), o["done"][sel],
                                  err_msg=f"done {where}")


def assert_rollout_vs_oracle(tr, ob, n, env_idx=None, W=200, H=200):
    """Every row of a rollout trajectory `tr` (n steps) against n oracle steps."""
    idx = None if env_idx is None else np.asarray(env_idx)
    o = None
    for s in range(n):
        o = ob.step()
        rows = [getattr(tr, f)[s] for f in ("obs", "serving", "reward", "done")]
        if idx is not None:
            import torch
            ti = torch.as_tensor(idx, device=rows[0].device)
            rows = [r.index_select(0, ti) for r in rows]
        obs, srv, rew, dn = (r.cpu().numpy() for r in rows)
        assert_step_vs_oracle(o, obs, srv, rew, dn, env_idx=None, W=W, H=H, where=f"step {s}")
    return o
