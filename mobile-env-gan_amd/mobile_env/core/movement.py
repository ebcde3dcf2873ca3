"""Movement plugins (reference core/movement.py:7-72).

``RandomWaypointMovement`` runs on the GPU: one numpy-compatible PCG64 stream per env
(seeded with the movement seed = config seed + 4), lazy waypoint draws in ue_id order,
integer steps of length ``velocity`` with numpy round-half-even, snap at arrival.
"""
from __future__ import annotations


class Movement:
    def __init__(self, width: float, height: float, seed: int, reset_rng_episode: bool,
                 **kwargs):
        self.width, self.height = width, height
        self.reset_rng_episode = reset_rng_episode
        self.seed = seed

    def reset(self) -> None:
        pass

    def move(self, ue):
        raise NotImplementedError("movement is evaluated on the GPU by libmev")

    def initial_position(self, ue):
        raise NotImplementedError("movement is evaluated on the GPU by libmev")

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only RandomWaypointMovement has a device lowering")


class RandomWaypointMovement(Movement):
    def lower_params(self) -> dict:
        return {"width": int(self.width), "height": int(self.height),
                "movement_seed": int(self.seed),
                "movement_reseed": bool(self.reset_rng_episode)}
