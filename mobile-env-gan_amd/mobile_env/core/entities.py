"""Entities (reference core/entities.py:6-57): parameter holders + integer positions.

``.point`` truncates coordinates to int like the reference (entities.py:24-26,52-54); the
reference returns a shapely Point, here a light (x, y) tuple with a ``distance`` helper.
The engine reads entity parameters once, when it lowers a scenario to device constants.
"""
from __future__ import annotations

import math
from typing import NamedTuple, Tuple


class Point(NamedTuple):
    """shapely.geometry.Point of the integer-truncated coordinates (entities.py:24-26,52-54):
    like shapely, the coordinates read back as floats."""
    x: float
    y: float

    def distance(self, other: "Point") -> float:
        dx, dy = self.x - other.x, self.y - other.y
        return math.sqrt(dx * dx + dy * dy)


class BaseStation:
    def __init__(self, bs_id: int, pos: Tuple[float, float], bw: float, freq: float, tx: float,
                 height: float):
        self.bs_id = bs_id
        self.x, self.y = pos
        self.bw = bw                # Hz
        self.frequency = freq       # MHz
        self.tx_power = tx          # dBm
        self.height = height        # m

    @property
    def point(self) -> Point:
        return Point(float(int(self.x)), float(int(self.y)))

    def __str__(self):
        return f"BS: {self.bs_id}"


class UserEquipment:
    def __init__(self, ue_id: int, velocity: float, snr_tr: float, noise: float, height: float):
        self.ue_id = ue_id
        self.velocity = velocity
        self.snr_threshold = snr_tr
        self.noise = noise
        self.height = height
        self.x = None
        self.y = None
        self.startTime = None
        self.exitTime = None

    @property
    def point(self) -> Point:
        return Point(float(int(self.x)), float(int(self.y)))

    def __str__(self):
        return f"UE: {self.ue_id}"
