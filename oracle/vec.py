"""NumPy restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Vectorised over E independent envs; per env it follows the reference op by op:

* reset            base.py:172-209 + custom.py:53-54 (activeUsers = all UEs with startTime <= 0)
* movement         movement.py:16-18 (re-seed per episode), 42-62 (move), 64-72 (initial_position)
* channel          channels.py:24-27 (calculateSNR), 78-83 (datarate), 133-146 (OkumuraHata)
* association      base.py:212-214, 236-241 (closest connectable BS, first in station order on ties)
* scheduling       base.py:421-435 + schedules.py:20-22 (ResourceFair share, numpy round to 0.01)
* utility          base.py:253-258 + utilities.py:44-55 (BoundedLogUtility, scaled)
* metrics          metrics.py:5-28 (number connections/connected, mean utility, mean datarate)
* bookkeeping      base.py:280-291, 407-409 (time, activeUsers, episode end); arrival.py:28-36

The channel chain depends on a (BS, UE) pair only through the integer squared distance d2
(entities.py:24-26,52-54 truncate coordinates to int), so it is evaluated once per integer d2
with NumPy *scalar* arithmetic -- the same operations and types the reference uses
(``10 ** np.float64`` is scalar libm ``pow``; ``np.log10``/``np.log2`` are the ufunc loops) -- and
looked up per pair. SNR is monotone in d2, so "connectable" is ``d2 <= d2max``
(checked: connectivity is a prefix of d2).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

EPSILON = 1e-16  # channels.py:8


@dataclass
class OracleParams:
    width: int = 200
    height: int = 200
    ep_max_time: int = 20          # base.py:105,109
    arrival_ep_time: int = 20      # base.py:126 (NoDeparture exit time)
    velocity: float = 1.5          # base.py:119
    bs: dict = field(default_factory=lambda: {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50})
    ue: dict = field(default_factory=lambda: {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6})
    lower: float = -20             # base.py:136
    upper: float = 20
    coeffs: tuple = (10, 0, 10)
    movement_reseed: bool = True   # movement_params reset_rng_episode (base.py:133, movement.py:16-18)
    # heterogeneous entities (entities.py:7-22,33-45): per-station / per-UE parameter classes
    # ({bw, freq, tx, height} / {velocity, snr_tr, noise, height}) and each entity's class
    bs_classes: list = None
    ue_classes: list = None
    bs_class: list = None
    ue_class: list = None
    # per-UE velocities (the reference's UserEquipment.velocity, entities.py:33-45; overrides
    # `velocity` / the UE classes' velocity)
    ue_velocity: list = None

    @property
    def t_end(self) -> int:
        # time_is_up (base.py:407-409): time >= min(EP_MAX_TIME, max_departure)
        return min(self.ep_max_time, self.arrival_ep_time)


def snr_scalar(d2: int, bs: dict, ue: dict):
    """calculateSNR for a pair at integer squared distance d2 (channels.py:24-27,133-146)."""
    distance = math.sqrt(float(d2))
    f = bs["freq"]
    ch = 0.8 + (1.1 * np.log10(f) - 0.7) * ue["height"] - 1.56 * np.log10(f)
    tmp_1 = 69.55 - ch + 26.16 * np.log10(f) - 13.82 * np.log10(bs["height"])
    tmp_2 = 44.9 - 6.55 * np.log10(bs["height"])
    loss = tmp_1 + tmp_2 * np.log10(distance + EPSILON)
    power = 10 ** ((bs["tx"] - loss) / 10)
    return power / ue["noise"]


def channel_table(p: OracleParams, d2_hi: int | None = None):
    """(d2max, rate_full[0..d2max]) -- datarate (channels.py:78-83) at every integer d2."""
    if d2_hi is None:
        d2_hi = (p.width - 1) ** 2 + (p.height - 1) ** 2
    rates = []
    d2max = -1
    for d2 in range(d2_hi + 1):
        snr = snr_scalar(d2, p.bs, p.ue)
        if not snr > p.ue["snr_tr"]:
            break
        rates.append(float(p.bs["bw"] * np.log2(1 + snr)))
        d2max = d2
    # connectivity must be a prefix in d2 for the d2 <= d2max test to be exact
    for d2 in range(d2max + 1, min(d2_hi, d2max + 2000) + 1):
        assert not snr_scalar(d2, p.bs, p.ue) > p.ue["snr_tr"], "connectivity not a prefix of d2"
    return d2max, np.asarray(rates, dtype=np.float64)


class OracleBatch:
    """E independent envs sharing params; BS layout shared [B,2] or per env [E,B,2] (+count)."""

    def __init__(self, p: OracleParams, bs_xy, num_ues: int, seeds, bs_count=None,
                 table=None):
        self.p = p
        bs_xy = np.asarray(bs_xy, dtype=np.int64)
        self.seeds = np.asarray(seeds, dtype=np.int64).reshape(-1)
        self.E = len(self.seeds)
        if bs_xy.ndim == 2:
            bs_xy = np.broadcast_to(bs_xy, (self.E,) + bs_xy.shape)
        self.bs_xy = np.array(bs_xy)
        self.B = self.bs_xy.shape[1]
        self.bs_count = (np.full(self.E, self.B) if bs_count is None
                         else np.asarray(bs_count, dtype=np.int64).reshape(-1))
        self.U = int(num_ues)
        self.d2max, self.rate_full = table if table is not None else channel_table(p)
        # per (station, UE) pair: its class pair's d2max and table (one pair when homogeneous);
        # the velocity per UE
        self.vel = np.full(self.U, float(p.velocity))
        self.pair_d2max = np.full((self.B, self.U), self.d2max, dtype=np.int64)
        self.pair_id = np.zeros((self.B, self.U), dtype=np.int64)
        self.tables = [self.rate_full]
        if p.bs_classes is not None or p.ue_classes is not None:
            bsc = p.bs_classes or [p.bs]
            uec = p.ue_classes or [dict(p.ue, velocity=p.velocity)]
            bcl = np.asarray(p.bs_class if p.bs_class is not None else [0] * self.B)
            ucl = np.asarray(p.ue_class if p.ue_class is not None else [0] * self.U)
            d2m, self.tables = [], []
            for b in bsc:
                for u in uec:
                    q = OracleParams(width=p.width, height=p.height, bs=dict(b),
                                     ue={k: u[k] for k in ("snr_tr", "noise", "height")})
                    dm, tab = channel_table(q)
                    d2m.append(dm)
                    self.tables.append(tab)
            self.pair_id = bcl[:, None] * len(uec) + ucl[None, :]
            self.pair_d2max = np.asarray(d2m, dtype=np.int64)[self.pair_id]
            self.vel = np.asarray([float(uec[c]["velocity"]) for c in ucl])
        if p.ue_velocity is not None:
            self.vel = np.asarray(p.ue_velocity, dtype=np.float64).reshape(self.U)
        self.t = np.full(self.E, p.t_end, dtype=np.int64)   # "episode over": next step resets
        self.x = np.zeros((self.E, self.U), dtype=np.int64)
        self.y = np.zeros((self.E, self.U), dtype=np.int64)
        self.wx = np.zeros((self.E, self.U), dtype=np.int64)
        self.wy = np.zeros((self.E, self.U), dtype=np.int64)
        self.wvalid = np.zeros((self.E, self.U), dtype=bool)
        self.gens = [None] * self.E

    # -- reset: base.py:172-209, movement.py:16-18,36-39,64-72 ---------------------------------
    def reset(self, envs=None):
        envs = range(self.E) if envs is None else envs
        W, H = self.p.width, self.p.height
        for e in envs:
            # movement seed = config seed + 4 (base.py:156-168); re-seeded every episode when
            # reset_rng_episode (the default), else created once and continued (movement.py:16-18)
            g = self.gens[e]
            if self.p.movement_reseed or g is None:
                g = np.random.default_rng(int(self.seeds[e]) + 4)
            self.gens[e] = g
            for u in range(self.U):
                self.x[e, u] = int(g.uniform(0, W))
                self.y[e, u] = int(g.uniform(0, H))
            self.wvalid[e] = False
            self.t[e] = 0

    def set_bs(self, e, xy):
        xy = np.asarray(xy, dtype=np.int64)
        self.bs_xy[e, :len(xy)] = xy
        self.bs_count[e] = len(xy)

    # -- step: base.py:230-296 ---------------------------------------------------------------------
    def step(self):
        p = self.p
        lazy = np.nonzero(self.t >= p.t_end)[0]
        if len(lazy):
            self.reset(lazy)
        t = self.t
        W, H = p.width, p.height
        vel = self.vel[None, :]
        # NoDeparture: start 0, exit arrival_ep_time; active during step t iff start <= t < exit
        active = np.broadcast_to(((t >= 0) & (t < p.arrival_ep_time))[:, None],
                                 (self.E, self.U)).copy()

        # movement (movement.py:42-62): waypoint draws in ue_id order, per env sequential
        for u in range(self.U):
            need = active[:, u] & ~self.wvalid[:, u]
            for e in np.nonzero(need)[0]:
                g = self.gens[e]
                self.wx[e, u] = int(g.uniform(0, W))
                self.wy[e, u] = int(g.uniform(0, H))
            self.wvalid[need, u] = True
        dx = self.wx - self.x
        dy = self.wy - self.y
        nrm = np.sqrt((dx * dx + dy * dy).astype(np.float64))
        snap = active & (nrm <= vel)
        move = active & ~snap
        with np.errstate(invalid="ignore", divide="ignore"):
            nx = np.rint(self.x + (vel * dx) / nrm)
            ny = np.rint(self.y + (vel * dy) / nrm)
        self.x = np.where(snap, self.wx, np.where(move, nx, self.x)).astype(np.int64)
        self.y = np.where(snap, self.wy, np.where(move, ny, self.y)).astype(np.int64)
        self.wvalid &= ~snap

        # association (base.py:236-241)
        bx = self.bs_xy[:, None, :, 0]
        by = self.bs_xy[:, None, :, 1]
        d2 = (self.x[:, :, None] - bx) ** 2 + (self.y[:, :, None] - by) ** 2      # [E,U,B]
        valid_bs = np.arange(self.B)[None, None, :] < self.bs_count[:, None, None]
        conn = (d2 <= self.pair_d2max.T[None]) & valid_bs & active[:, :, None]
        big = np.iinfo(np.int64).max
        srv = np.argmin(np.where(conn, d2, big), axis=2)
        has = conn.any(axis=2)
        serving = np.where(has, srv, -1)
        d2s = np.take_along_axis(d2, np.maximum(serving, 0)[:, :, None], axis=2)[:, :, 0]

        # ResourceFair share + round (base.py:421-435, schedules.py:21-22)
        nb = np.zeros((self.E, self.B), dtype=np.int64)
        for b in range(self.B):
            nb[:, b] = (serving == b).sum(axis=1)
        n = np.take_along_axis(nb, np.maximum(serving, 0), axis=1)
        if len(self.tables) == 1:
            full = self.rate_full[np.where(has, d2s, 0)]
        else:  # the serving pair's class-pair table
            pid = self.pair_id.T[np.arange(self.U)[None, :], np.maximum(serving, 0)]
            full = np.array([self.tables[k][d] if h else 0.0
                             for k, d, h in zip(pid.ravel(), d2s.ravel(), has.ravel())]
                            ).reshape(d2s.shape)
        share = np.where(has, full / np.maximum(n, 1), 0.0)
        rate = np.where(has, np.round(share, 2), 0.0)

        # utility (utilities.py:44-58)
        lower, upper = p.lower, p.upper
        w1, w2, w3 = p.coeffs
        with np.errstate(divide="ignore", invalid="ignore"):
            u_raw = np.clip(w1 * np.log(w2 + rate) / np.log(w3), lower, upper)
        u_raw = np.where(rate <= 0.0, lower, u_raw)
        util = 2 * (u_raw - lower) / (upper - lower) - 1
        util = np.where(active, util, np.nan)

        # metrics (metrics.py:5-28)
        ncon = (serving >= 0).sum(axis=1).astype(np.float64)
        mean_u = np.empty(self.E)
        mean_r = np.empty(self.E)
        for e in range(self.E):
            a = active[e]
            mean_u[e] = np.mean(util[e, a]) if a.any() else lower
            c = serving[e] >= 0
            mean_r[e] = np.mean(rate[e, c]) if c.any() else 0.0
        metrics = np.stack([ncon, ncon, mean_u, mean_r], axis=1)

        self.t = t + 1
        done = self.t >= p.t_end
        return dict(xy=np.stack([self.x, self.y], axis=-1), serving=serving, rate=rate,
                    util=util, metrics=metrics, done=done, d2=d2s)
