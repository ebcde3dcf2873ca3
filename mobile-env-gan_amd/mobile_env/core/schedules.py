"""Scheduler plugins (reference core/schedules.py:7-29).

``ResourceFair`` (equal share rate / n_b) runs inside the step kernel. The reference's
``RateFair`` returns a scalar where ``allocateDataRate2User`` zips a list (base.py:435), so
it cannot run there either; it has no lowering here.
"""
from __future__ import annotations


class Scheduler:
    def __init__(self, **kwargs):
        pass

    def reset(self) -> None:
        pass

    def share(self, bs, rates):
        raise NotImplementedError("scheduling is evaluated on the GPU by libmev")

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only ResourceFair has a device lowering")


class ResourceFair(Scheduler):
    def lower_params(self) -> dict:
        return {"scheduler": "resource_fair"}


class RateFair(Scheduler):
    pass
