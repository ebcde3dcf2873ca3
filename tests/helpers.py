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
