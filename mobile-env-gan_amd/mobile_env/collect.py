"""Batched data collection: the reference's collectData2.ipynb driver with every epoch as one
env of a GPU batch.

The notebook (collectData2.ipynb cells 2-4) builds one ``MComCustom``, calls ``reset()``
once, then for each epoch: ``reset()`` (a fresh layout of ``randint(5, 10)`` stations at
``int(uniform(0, 200))`` from Python's global ``random``, custom.py:68-77, and the movement
stream re-seeded from the same config seed, movement.py:16-18), ``save_base_station_positions``,
20 x ``step``, ``save_epoch_data``. Epochs differ only in their layout, so they are
independent: epoch j is env j here, with the layout of the (j+1)-th draw of the same
``random`` stream (the extra reset of cell 3 takes the first). The episodes run as one
batch on the device and :class:`~mobile_env.dataset.DatasetWriter` writes the same
collectData / collectData2 files, named by epoch.

Layouts come from Python's own ``random.Random`` (the generator the reference uses), in the
reference's call order -- no re-implementation to drift.
"""
from __future__ import annotations

import random
from typing import Optional, Tuple

import numpy as np

__all__ = ["draw_layouts", "collect_data"]

MAX_BS = 10  # randint(5, 10)


def draw_layouts(rng: random.Random, n: int, width: int = 200, height: int = 200
                 ) -> Tuple[np.ndarray, np.ndarray]:
    """n consecutive MComCustom layouts from ``rng`` (custom.py:68-77): int32 [n, 10, 2]
    (rows beyond the count are 0) and the counts [n]."""
    xy = np.zeros((n, MAX_BS, 2), dtype=np.int32)
    cnt = np.zeros(n, dtype=np.int32)
    for k in range(n):
        b = rng.randint(5, 10)
        cnt[k] = b
        for j in range(b):
            xy[k, j, 0] = int(rng.uniform(0, width))
            xy[k, j, 1] = int(rng.uniform(0, height))
    return xy, cnt


def collect_data(num_epochs: int, root: str, random_seed: Optional[int] = None,
                 steps: int = 20, device=None, batch: int = 65536, config=None) -> dict:
    """Write the collectData / collectData2 tree of ``num_epochs`` notebook epochs to
    ``root`` (the reference writes to ``..``). ``random_seed``: seed of the layout stream
    (the notebook leaves the global ``random`` unseeded; ``random.seed(k)`` before it runs
    corresponds to ``random_seed=k``). Epochs run ``batch`` at a time. Returns counts."""
    import torch

    from .core.engine import EngineParams, StepEngine
    from .core.util import deep_dict_merge
    from .dataset import DatasetWriter
    from .scenarios.custom import MComCustom

    cfg = deep_dict_merge(MComCustom.default_config(), config or {})
    t_end = min(cfg["EP_MAX_TIME"], cfg["arrival_params"]["ep_time"])
    if not 1 <= steps <= t_end:
        raise ValueError(f"steps must lie in [1, {t_end}] (the engine resets at episode end)")
    rng = random.Random(random_seed)
    draw_layouts(rng, 1, cfg["width"], cfg["height"])  # the reset of notebook cell 3
    seed = int(cfg["seed"])
    done = 0
    while done < num_epochs:
        E = min(batch, num_epochs - done)
        xy, cnt = draw_layouts(rng, E, cfg["width"], cfg["height"])
        p = EngineParams(
            num_envs=E, num_ues=7, num_bs=MAX_BS, width=cfg["width"], height=cfg["height"],
            ep_max_time=cfg["EP_MAX_TIME"], arrival_start=0,
            arrival_exit=cfg["arrival_params"]["ep_time"], first_step_active=True,
            movement_reseed=True, velocity=cfg["ue"]["velocity"], bs=dict(cfg["bs"]),
            ue={k: cfg["ue"][k] for k in ("snr_tr", "noise", "height")},
            util_lower=cfg["utility_params"]["lower"], util_upper=cfg["utility_params"]["upper"],
            util_coeffs=tuple(cfg["utility_params"]["coeffs"]))
        eng = StepEngine(p, xy, np.full(E, seed), bs_count=cnt, device=device, rate64=True,
                         util64=True)
        first = done
        writer = DatasetWriter(eng, root, epoch_of=lambda e, k, first=first: first + e,
                               episode_steps=steps)
        for _ in range(steps):
            eng.step(1)
            writer.record()
        writer.close()
        torch.cuda.synchronize(eng.device)
        eng.close()
        done += E
    return {"epochs": num_epochs, "steps": steps}
