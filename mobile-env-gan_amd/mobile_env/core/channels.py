"""Channel plugins (reference core/channels.py:11-27,78-83,132-146).

The step kernels never evaluate the channel per pair: a pair's SNR depends on the pair only
through the integer squared distance d2 (positions are int-truncated, entities.py:24-26,
52-54), so the whole chain Okumura-Hata -> SNR -> Shannon rate is tabulated once per parameter
set over every integer d2 (:meth:`Channel.rate_table`) and uploaded when the engine is built
(mev_params.rate_table); the kernels look the serving pair up in it.

The table is built HERE, on the host, with numpy -- the library the reference computes it
with -- in the reference's operation order, so its entries are the reference's own values:
numpy's float64 ``log10`` / ``log2`` loops (SIMD on AVX-512 hosts) differ from the C
library's by one ulp on some inputs, so a table built with libm or on the device is not
bit-exact (round 1 had such a device table).

The per-pair methods (``power_loss``, ``calculateSNR``, ``datarate``) are the reference's, for
callers that use the plugin objects directly (e.g. coverage plots); the step never calls them.
"""
from __future__ import annotations

import math

import numpy as np

EPSILON = 1e-16  # channels.py:8
# largest squared distance of a UE on the map to a station (coordinates < 1024, mev.h); on maps
# beyond 1024 also the longest connectable distance (mev.h kMaxMap: the association keys hold
# the squared distance in 22 bits)
D2_TOP = 2 * 1023 * 1023


class Channel:
    def __init__(self, **kwargs):
        pass

    def reset(self) -> None:
        pass

    def power_loss(self, bs, ue) -> float:
        raise NotImplementedError(f"{type(self).__name__} defines no power_loss")

    def calculateSNR(self, bs, ue):
        """channels.py:24-27: linear SNR of the pair."""
        loss = self.power_loss(bs, ue)
        return 10 ** ((bs.tx_power - loss) / 10) / ue.noise

    @classmethod
    def datarate(cls, bs, ue, snr):
        """channels.py:78-83: Shannon rate if the pair is connectable, else 0."""
        return bs.bw * np.log2(1 + snr) if snr > ue.snr_threshold else 0.0

    def snr_of_distance(self, distance, bs: dict, ue: dict):
        """Vectorised SNR at float64 pair distances (numpy array), or raise: a channel model
        without this has no table lowering."""
        raise NotImplementedError(
            f"{type(self).__name__}: only OkumuraHata has a device lowering")

    def rate_table(self, bs: dict, ue: dict, width: int = 200, height: int = 200):
        """Full (unshared) rate at every connectable integer squared distance: float64
        [d2max + 1] with the connectable d2 exactly [0, d2max] (a prefix; checked over the
        map's squared distances, and over every station distance when the whole map range
        connects). ``bs`` = {bw, freq, tx, height}, ``ue`` = {snr_tr, noise, height}.
        Memoised per parameter set (the scalar power per entry makes a table of every map
        distance cost seconds; heterogeneous contexts ask for one per class pair)."""
        key = (type(self), tuple(float(bs[k]) for k in ("bw", "freq", "tx", "height")),
               tuple(float(ue[k]) for k in ("snr_tr", "noise", "height")), int(width),
               int(height))
        tab = _RATE_TABLES.get(key)
        if tab is None:
            tab = self._rate_table(bs, ue, width, height)
            tab.setflags(write=False)
            _RATE_TABLES[key] = tab
        return tab.copy()

    def _rate_table(self, bs: dict, ue: dict, width: int, height: int):
        map_hi = (width - 1) ** 2 + (height - 1) ** 2
        snr = self._snr_table(min(map_hi, D2_TOP), bs, ue)
        conn = snr > ue["snr_tr"]
        if conn.all() and map_hi > D2_TOP:  # (maps beyond 1024: as mev_build_rate_table)
            raise ValueError("the channel connects beyond the longest supported distance "
                             f"(d2 > {D2_TOP}) on a {width} x {height} map")
        if conn.all():  # every map distance connects: stations may sit off the map
            snr = self._snr_table(D2_TOP, bs, ue)
            conn = snr > ue["snr_tr"]
        n = int(conn.sum())
        if not conn[:n].all():
            raise ValueError("channel connectivity is not a prefix of the squared distance")
        # datarate (channels.py:81): bw * log2(1 + snr), elementwise as in numpy scalars
        return np.asarray(bs["bw"] * np.log2(1 + snr[:n]), dtype=np.float64)

    def _snr_table(self, d2_hi, bs, ue):
        # shapely's distance of integer points = sqrt(d2), correctly rounded
        distance = np.sqrt(np.arange(d2_hi + 1, dtype=np.float64))
        return self.snr_of_distance(distance, bs, ue)


_RATE_TABLES: dict = {}  # Channel.rate_table's memo: (model, bs, ue, W, H) -> table


class OkumuraHata(Channel):
    def power_loss(self, bs, ue):
        """channels.py:133-146 (distance between the int-truncated positions)."""
        return self._loss(bs.point.distance(ue.point), bs.frequency, bs.height, ue.height)

    @staticmethod
    def _loss(distance, f, hb, hu):
        # the reference's operation order; numpy float64 log10 on the scalar parameters
        ch = 0.8 + (1.1 * np.log10(f) - 0.7) * hu - 1.56 * np.log10(f)
        tmp_1 = 69.55 - ch + 26.16 * np.log10(f) - 13.82 * np.log10(hb)
        tmp_2 = 44.9 - 6.55 * np.log10(hb)
        return tmp_1 + tmp_2 * np.log10(distance + EPSILON)

    def snr_of_distance(self, distance, bs: dict, ue: dict):
        loss = self._loss(distance, bs["freq"], bs["height"], ue["height"])
        # calculateSNR (channels.py:24-27): 10 ** x of a numpy float64 scalar is the C
        # library's pow (numpy scalar math); numpy's *array* power may take a SIMD path with
        # other roundings, so the power is taken per element with the scalar pow
        x = (bs["tx"] - loss) / 10
        power = np.fromiter((math.pow(10.0, v) for v in x.tolist()), dtype=np.float64,
                            count=len(x))
        return power / ue["noise"]

    def lower_params(self) -> dict:
        return {"channel": "okumura_hata"}
