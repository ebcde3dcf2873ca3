"""Per-object pure-Python restatement of the reference step -- TEST INFRASTRUCTURE ONLY.

Same structure and per-call cost profile as the reference's CPU path (entity objects,
plugin objects, dict/set bookkeeping, the channel chain evaluated per (BS, UE) pair with
NumPy scalars), used by the parity tests on small cases and timed by ``bench.py`` as the
``cpu_baseline`` ("port"). The per-step JSON dump (base.py:261,298-349) is not performed
(compute-only baseline).

Reference call stack restated (file:line in /root/reference/mobile_env):
  Core.reset   <- core/base.py:172-209, scenarios/custom.py:53-62
  Core.step    <- core/base.py:230-296
  Movement     <- core/movement.py:16-18, 36-72
  channel      <- core/channels.py:24-27, 78-83, 133-146; entities.py:24-26,52-54
  share        <- core/schedules.py:20-22; base.py:421-435
  utility      <- core/utilities.py:44-58
  metrics      <- core/metrics.py:5-28
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict

import numpy as np

EPS = 1e-16


class Station:
    def __init__(self, sid, x, y, bw, freq, tx, height):
        self.sid, self.x, self.y = sid, x, y
        self.bw, self.freq, self.tx, self.height = bw, freq, tx, height

    def ipos(self):
        return int(self.x), int(self.y)


class Device:
    def __init__(self, uid, velocity, snr_tr, noise, height):
        self.uid = uid
        self.velocity, self.snr_tr, self.noise, self.height = velocity, snr_tr, noise, height
        self.x = self.y = None
        self.start = self.exit = None

    def ipos(self):
        return int(self.x), int(self.y)


class Hata:
    """Okumura-Hata path loss + SNR + Shannon rate for one pair."""

    @staticmethod
    def snr(bs: Station, ue: Device):
        (bx, by), (ux, uy) = bs.ipos(), ue.ipos()
        dist = math.sqrt(float((bx - ux) ** 2 + (by - uy) ** 2))
        lf = np.log10(bs.freq)
        corr = 0.8 + (1.1 * lf - 0.7) * ue.height - 1.56 * lf
        a = 69.55 - corr + 26.16 * np.log10(bs.freq) - 13.82 * np.log10(bs.height)
        b = 44.9 - 6.55 * np.log10(bs.height)
        loss = a + b * np.log10(dist + EPS)
        return 10 ** ((bs.tx - loss) / 10) / ue.noise

    @staticmethod
    def rate(bs: Station, ue: Device, snr):
        return bs.bw * np.log2(1 + snr) if snr > ue.snr_tr else 0.0


class Waypoints:
    def __init__(self, width, height, seed, reseed=True):
        self.w, self.h, self.seed, self.reseed = width, height, seed, reseed
        self.rng = None
        self.target = {}

    def reset(self):
        if self.reseed or self.rng is None:
            self.rng = np.random.default_rng(self.seed)
        self.target = {}

    def spawn(self, ue):
        return int(self.rng.uniform(0, self.w)), int(self.rng.uniform(0, self.h))

    def move(self, ue):
        if ue not in self.target:
            self.target[ue] = (int(self.rng.uniform(0, self.w)), int(self.rng.uniform(0, self.h)))
        here = np.array([ue.x, ue.y])
        goal = np.array(self.target[ue])
        if np.linalg.norm(here - goal) <= ue.velocity:
            return self.target.pop(ue)
        d = goal - here
        nxt = np.round(here + ue.velocity * d / np.linalg.norm(d)).astype(int)
        return tuple(nxt)


class Core:
    """Compute-only restatement of MComCore (+ MComCustom reset bookkeeping)."""

    def __init__(self, stations, devices, *, width=200, height=200, seed=2024, ep_time=20,
                 ep_max_time=20, lower=-20, upper=20, coeffs=(10, 0, 10), reseed=True):
        self.stations = list(stations)
        self.devices = sorted(devices, key=lambda d: d.uid)
        self.mover = Waypoints(width, height, seed + 4, reseed)   # seeding(): movement = seed+4
        self.ep_time, self.ep_max_time = ep_time, ep_max_time
        self.lower, self.upper, self.coeffs = lower, upper, coeffs
        self.time = 0
        self.active = []
        self.links = defaultdict(set)
        self.rates = {}
        self.ue_rate = Counter()
        self.util = {}
        self.history = []

    def reset(self):
        self.time = 0
        self.mover.reset()
        for d in self.devices:
            d.start, d.exit = 0, self.ep_time
        for d in self.devices:
            d.x, d.y = self.mover.spawn(d)
        self.links = defaultdict(set)
        self.rates = {}
        self.active = [d for d in self.devices if d.start <= 0]
        self.history = []

    def _utility(self, r):
        w1, w2, w3 = self.coeffs
        if r <= 0.0:
            u = self.lower
        else:
            u = np.clip(w1 * np.log(w2 + r) / np.log(w3), self.lower, self.upper)
        return 2 * (u - self.lower) / (self.upper - self.lower) - 1

    def step(self):
        for d in self.active:
            d.x, d.y = self.mover.move(d)
        self.links = defaultdict(set)
        for d in self.active:
            ok = [bs for bs in self.stations if Hata.snr(bs, d) > d.snr_tr]
            if ok:
                best = min(ok, key=lambda bs: np.linalg.norm(
                    [d.x - bs.ipos()[0], d.y - bs.ipos()[1]]))
                self.links[best].add(d)
        self.rates = {}
        for bs in self.stations:
            members = list(self.links.get(bs, ()))
            full = [Hata.rate(bs, d, Hata.snr(bs, d)) for d in members]
            shares = [r / len(full) for r in full]
            for d, r in zip(members, shares):
                self.rates[(bs, d)] = round(r, 2)
        self.ue_rate = Counter()
        for (bs, d), r in self.rates.items():
            self.ue_rate.update({d: r})
        self.util = {d: self._utility(self.ue_rate.get(d, 0.0)) for d in self.active}
        n_links = sum(len(v) for v in self.links.values())
        mean_u = np.mean(list(self.util.values())) if self.util else self.lower
        mean_r = np.mean(list(self.ue_rate.values())) if self.ue_rate else 0.0
        self.history.append((n_links, n_links, mean_u, mean_r))
        self.time += 1
        self.active = [d for d in self.devices if d.exit > self.time >= d.start]

    def snapshot(self):
        srv = {d.uid: bs.sid for (bs, d) in self.rates}
        return ([(int(d.x), int(d.y)) for d in self.devices],
                [srv.get(d.uid, -1) for d in self.devices],
                [float(self.ue_rate.get(d, 0.0)) for d in self.devices],
                [float(self.util[d]) if d in self.util else float("nan") for d in self.devices],
                self.history[-1])


def build(bs_xy, num_ues, seed, velocity, bs=None, ue=None, classes=None, **kw):
    """classes: heterogeneous entities (entities.py:7-22,33-45, every object its own
    parameters) as {bs_classes, ue_classes, bs_class, ue_class} -- station j gets
    bs_classes[bs_class[j]], UE u gets ue_classes[ue_class[u]] (velocity included)."""
    bs = bs or {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50}
    ue = ue or {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}
    bsp = [classes["bs_classes"][classes["bs_class"][i]] if classes else bs
           for i in range(len(bs_xy))]
    uep = [classes["ue_classes"][classes["ue_class"][i]] if classes else dict(ue, velocity=velocity)
           for i in range(num_ues)]
    stations = [Station(i, int(x), int(y), q["bw"], q["freq"], q["tx"], q["height"])
                for i, ((x, y), q) in enumerate(zip(bs_xy, bsp))]
    devices = [Device(i, q["velocity"], q["snr_tr"], q["noise"], q["height"])
               for i, q in enumerate(uep)]
    return Core(stations, devices, seed=seed, **kw)


def run_driver(core, episodes, steps, on_step=None):
    """collectData2.ipynb loop: reset(); step() x steps, per episode."""
    for ep in range(episodes):
        core.reset()
        for s in range(steps):
            core.step()
            if on_step is not None:
                on_step(ep, s, core)
