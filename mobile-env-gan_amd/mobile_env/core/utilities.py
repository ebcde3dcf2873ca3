"""Utility plugins (reference core/utilities.py:7-58).

``BoundedLogUtility`` (clip(w1 ln(w2 + r) / ln(w3), lower, upper), scaled to [-1, 1]) runs
inside the step kernel. The per-value methods are the reference's (numpy scalars) for callers
that use the plugin directly and for host bookkeeping (e.g. the idle value of a station).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


class Utility:
    def __init__(self, **kwargs):
        pass

    def reset(self) -> None:
        pass

    def calculateUtility(self, datarate) -> float:
        raise NotImplementedError(f"{type(self).__name__} defines no calculateUtility")

    def scaleUtility(self, utility) -> float:
        raise NotImplementedError

    def unscaleUtility(self, utility) -> float:
        raise NotImplementedError

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only BoundedLogUtility has a device lowering")


class BoundedLogUtility(Utility):
    def __init__(self, lower: float, upper: float, coeffs: Tuple[float, float, float],
                 **kwargs):
        super().__init__(**kwargs)
        self.lower = lower
        self.upper = upper
        self.coeffs = coeffs

    def calculateUtility(self, datarate) -> float:
        """utilities.py:44-53: lower for a non-positive rate, else the clipped log utility."""
        w1, w2, w3 = self.coeffs
        if datarate <= 0.0:
            return self.lower
        return np.clip(w1 * np.log(w2 + datarate) / np.log(w3), self.lower, self.upper)

    def scaleUtility(self, utility) -> float:
        return 2 * (utility - self.lower) / (self.upper - self.lower) - 1

    def unscaleUtility(self, utility) -> float:
        return (utility + 1) / 2 * (self.upper - self.lower) + self.lower

    def lower_params(self) -> dict:
        w1, w2, w3 = self.coeffs
        return {"util_lower": float(self.lower), "util_upper": float(self.upper),
                "util_coeffs": (float(w1), float(w2), float(w3))}
