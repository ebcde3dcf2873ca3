"""Layout scoring on the GPU: chooseBaseStation.ipynb's ``qoeValue``.

The notebook (cells 1, 5, 9) reads an epoch's ``user_qoe_{epoch}.csv`` (the rounded QoE
values ``round(u, 2)`` of every active UE at every step, base.py:264-269), flattens them and
scores the station layout:

    score = w1 * mean(q) - w2 * var(q) - w3 * mean(q < low_qoe_threshold)

with weights (1.0, 0.1, 10.0) and threshold 0.0. The step kernel accumulates, per env and
episode, {count, sum, sum of squares, count below the threshold} of exactly those values
(``StepEngine(qoe_stats=True)``, threshold ``EngineParams.qoe_low``), so a batch of E layouts
is scored after one episode without writing or parsing any file; ``score_layouts`` runs such
a search over many MComCustom-style layouts.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

__all__ = ["layout_scores", "qoe_value_reference", "score_layouts"]

WEIGHTS = (1.0, 0.1, 10.0)


def layout_scores(stats, weights: Tuple[float, float, float] = WEIGHTS) -> Dict:
    """Scores from qoe_stats [E, 4] (tensor or array): Average QoE, QoE Variance (population,
    like np.var), Low QoE Proportion and Score, each [E]."""
    n, s, s2, low = (stats[:, i] for i in range(4))
    mean = s / n
    var = s2 / n - mean * mean
    lowp = low / n
    w1, w2, w3 = weights
    return {"Average QoE": mean, "QoE Variance": var, "Low QoE Proportion": lowp,
            "Score": w1 * mean - w2 * var - w3 * lowp}


def qoe_value_reference(qoe_dict, low_qoe_threshold=0.0, weights=WEIGHTS) -> Dict:
    """chooseBaseStation.ipynb cell 5 (test oracle for layout_scores)."""
    all_qoe = np.hstack(list(qoe_dict.values()))
    average_qoe = np.mean(all_qoe)
    qoe_variance = np.var(all_qoe)
    low_qoe_proportion = np.sum(all_qoe < low_qoe_threshold) / len(all_qoe)
    w1, w2, w3 = weights
    return {"Average QoE": average_qoe, "QoE Variance": qoe_variance,
            "Low QoE Proportion": low_qoe_proportion,
            "Score": w1 * average_qoe - w2 * qoe_variance - w3 * low_qoe_proportion}


def score_layouts(xy, count, seed: int = 2024, config=None, device=None,
                  weights=WEIGHTS, low_qoe_threshold: float = 0.0) -> Dict:
    """Score E station layouts (xy [E, B, 2] int, count [E]) in one batched MComCustom episode
    each (7 UEs at velocity 10, the movement stream of config seed ``seed``); returns the
    score dict of ``layout_scores`` as numpy arrays plus the best layout's index."""
    import torch

    from .core.engine import EngineParams, StepEngine
    from .core.util import deep_dict_merge
    from .scenarios.custom import MComCustom

    cfg = deep_dict_merge(MComCustom.default_config(), config or {})
    xy = np.asarray(xy, dtype=np.int32)
    E, B = xy.shape[0], xy.shape[1]
    p = EngineParams(
        num_envs=E, num_ues=7, num_bs=B, width=cfg["width"], height=cfg["height"],
        ep_max_time=cfg["EP_MAX_TIME"], arrival_start=0,
        arrival_exit=cfg["arrival_params"]["ep_time"], first_step_active=True,
        movement_reseed=True, velocity=cfg["ue"]["velocity"], bs=dict(cfg["bs"]),
        ue={k: cfg["ue"][k] for k in ("snr_tr", "noise", "height")},
        util_lower=cfg["utility_params"]["lower"], util_upper=cfg["utility_params"]["upper"],
        util_coeffs=tuple(cfg["utility_params"]["coeffs"]), qoe_low=low_qoe_threshold)
    eng = StepEngine(p, xy, np.full(E, seed), bs_count=np.asarray(count, dtype=np.int32),
                     device=device, qoe_stats=True)
    eng.step(p.t_end)
    out = {k: v.cpu().numpy() for k, v in layout_scores(eng.qoe_stats, weights).items()}
    torch.cuda.synchronize(eng.device)
    eng.close()
    out["best"] = int(np.argmax(out["Score"]))
    return out
