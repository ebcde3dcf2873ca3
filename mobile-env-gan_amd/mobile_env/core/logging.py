"""Monitor (reference core/logging.py:6-87): per-step metric histories of one env."""
from __future__ import annotations

from typing import Dict


class Monitor:
    def __init__(self, scalar_metrics: Dict, ue_metrics: Dict, bs_metrics: Dict, **kwargs):
        self.scalar_metrics = scalar_metrics
        self.ue_metrics = ue_metrics
        self.bs_metrics = bs_metrics
        self.scalar_results = None
        self.ue_results = None
        self.bs_results = None

    def reset(self):
        self.scalar_results = {name: [] for name in self.scalar_metrics}
        self.ue_results = {name: [] for name in self.ue_metrics}
        self.bs_results = {name: [] for name in self.bs_metrics}

    def update(self, simulation):
        for name, fn in self.scalar_metrics.items():
            self.scalar_results[name].append(fn(simulation))
        for name, fn in self.ue_metrics.items():
            self.ue_results[name].append(fn(simulation))
        for name, fn in self.bs_metrics.items():
            self.bs_results[name].append(fn(simulation))

    def load_results(self):
        """(scalar, ue, bs) pandas DataFrames indexed like the reference (logging.py:44-75)."""
        import pandas as pd

        scalar = pd.DataFrame(self.scalar_results)
        scalar.index.names = ["Time Step"]

        def per_entity(results, key):
            cols = {(m, i): [step.get(i) for step in steps]
                    for m, steps in results.items() for i in set().union(*steps)}
            df = pd.DataFrame(cols).transpose()
            df.index.names = ["Metric", key]
            df = df.stack()
            df.index.names = ["Metric", key, "Time Step"]
            return df.reorder_levels(["Time Step", key, "Metric"]).unstack()

        return scalar, per_entity(self.ue_results, "UE ID"), per_entity(self.bs_results, "BS ID")

    def info(self):
        if any(len(v) == 0 for v in self.scalar_results.values()):
            return {}
        out = {n: v[-1] for n, v in self.scalar_results.items()}
        out.update({n: v[-1] for n, v in self.ue_results.items()})
        out.update({n: v[-1] for n, v in self.bs_results.items()})
        return out
