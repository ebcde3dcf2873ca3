"""Arrival plugins (reference core/arrival.py:8-36).

Plugins here are lowered to device constants by the engine (see ``lower``); the built-in
``NoDeparture`` gives every UE start 0 and exit ``ep_time``.
"""
from __future__ import annotations

import numpy as np


class Arrival:
    def __init__(self, ep_time: int, seed: int, reset_rng_episode: bool, **kwargs):
        self.ep_time = ep_time
        self.seed = seed
        self.reset_rng_episode = reset_rng_episode
        self.rng = None

    def reset(self) -> None:
        """arrival.py:15-17 (the built-in NoDeparture draws nothing from it)."""
        if self.reset_rng_episode or self.rng is None:
            self.rng = np.random.default_rng(self.seed)

    def setArrivalTime(self, ue) -> int:
        raise NotImplementedError

    def setDepartureTime(self, ue) -> int:
        raise NotImplementedError

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only NoDeparture has a device lowering")


class NoDeparture(Arrival):
    def setArrivalTime(self, ue) -> int:
        return 0

    def setDepartureTime(self, ue) -> int:
        return self.ep_time

    def lower_params(self) -> dict:
        return {"arrival_start": 0, "arrival_exit": int(self.ep_time)}
