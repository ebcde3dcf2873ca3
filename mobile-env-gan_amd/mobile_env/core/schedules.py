"""Scheduler plugins (reference core/schedules.py:7-29).

``ResourceFair`` (equal share rate / n_b, rounded by the caller to cents, base.py:435) runs
inside the step kernel: each UE's share is formed there from its station's connected-UE count.
``share`` is the reference's per-station method for callers that use the plugin directly; the
step never calls it. The reference's ``RateFair`` returns a scalar where
``allocateDataRate2User`` zips a list (base.py:435), so it cannot run in a step either; it has
no lowering here.
"""
from __future__ import annotations


class Scheduler:
    def __init__(self, **kwargs):
        pass

    def reset(self) -> None:
        pass

    def share(self, bs, rates):
        raise NotImplementedError(f"{type(self).__name__} defines no share")

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only ResourceFair has a device lowering")


class ResourceFair(Scheduler):
    def share(self, bs, rates):
        """schedules.py:20-22: every connected UE gets rate / (number of UEs)."""
        n = len(rates)
        return [r / n for r in rates]

    def lower_params(self) -> dict:
        return {"scheduler": "resource_fair"}


class RateFair(Scheduler):
    def share(self, bs, rates):
        """schedules.py:26-29 as written: one scalar, the inverse of the summed inverse rates."""
        return 1 / sum(1 / r for r in rates)
