"""Scalar metrics (reference core/metrics.py:5-28).

The four built-in metrics are reduced on the GPU inside the step kernel (per env:
connections, connected UEs, mean scaled utility over active UEs -- ``lower`` when none is
active -- and mean rate over connected UEs). On the MComCore facade these functions return
the kernel's values for the last step; they keep the reference's names and signature
``metric(sim)`` so they can be registered in ``config["metrics"]`` the same way.
"""
from __future__ import annotations


def _last(sim, i):
    return sim._metric_values[i]


def number_connections(sim):
    return int(_last(sim, 0))


def number_connected(sim):
    return int(_last(sim, 1))


def mean_datarate(sim):
    return float(_last(sim, 3))


def mean_utility(sim):
    return float(_last(sim, 2))
