"""Movement plugins (reference core/movement.py:7-72).

``RandomWaypointMovement`` runs on the GPU inside the step: one numpy-compatible PCG64 stream
per env (seeded with the movement seed = config seed + 4), lazy waypoint draws in ue_id order,
integer steps of length ``velocity`` with numpy round-half-even, snap at arrival.

The per-UE methods below are the reference's, on the plugin's own numpy Generator, for
callers that drive the plugin object directly; the engine never calls them (it keeps the
stream state on the device) and the two do not share state.
"""
from __future__ import annotations

import numpy as np


class Movement:
    def __init__(self, width: float, height: float, seed: int, reset_rng_episode: bool,
                 **kwargs):
        self.width, self.height = width, height
        self.reset_rng_episode = reset_rng_episode
        self.seed = seed
        self.rng = None

    def reset(self) -> None:
        """movement.py:16-18: (re-)seed the plugin's Generator."""
        if self.reset_rng_episode or self.rng is None:
            self.rng = np.random.default_rng(self.seed)

    def move(self, ue):
        raise NotImplementedError(f"{type(self).__name__} defines no move")

    def initial_position(self, ue):
        raise NotImplementedError(f"{type(self).__name__} defines no initial_position")

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only RandomWaypointMovement has a device lowering")


class RandomWaypointMovement(Movement):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.userMoveDirection = {}
        self.userPositionInitial = {}

    def reset(self) -> None:
        super().reset()
        self.userMoveDirection = {}
        self.userPositionInitial = {}

    def _draw(self):
        # int(uniform(0, W)), int(uniform(0, H)): two draws, x first (movement.py:45-46)
        return int(self.rng.uniform(0, self.width)), int(self.rng.uniform(0, self.height))

    def move(self, ue):
        """movement.py:42-62: draw a waypoint if the UE has none; snap to it (and drop it)
        when it is within ``velocity``, else one step toward it rounded half-to-even."""
        if ue not in self.userMoveDirection:
            self.userMoveDirection[ue] = self._draw()
        here = np.array([ue.x, ue.y])
        target = np.array(self.userMoveDirection[ue])
        if np.linalg.norm(here - target) <= ue.velocity:
            return self.userMoveDirection.pop(ue)
        v = target - here
        return tuple(np.round(here + ue.velocity * v / np.linalg.norm(v)).astype(int))

    def initial_position(self, ue):
        """movement.py:64-72: drawn once per UE and episode, then repeated."""
        if ue not in self.userPositionInitial:
            self.userPositionInitial[ue] = self._draw()
        return self.userPositionInitial[ue]

    def lower_params(self) -> dict:
        return {"width": int(self.width), "height": int(self.height),
                "movement_seed": int(self.seed),
                "movement_reseed": bool(self.reset_rng_episode)}
