"""Scenario registry for the batched Gym-style surface.

The reference registers no scenario ids (its package ``__init__``s are empty,
mobile_env/__init__.py:1-2, scenarios/__init__.py:1) and its only runnable scenario is
MComCustom (scenarios/custom.py:12-86). The ids below are this build's definitions
(SURVEY.md section 8): sizes follow upstream mobile-env, layouts are in layouts.json.

``central`` and ``ma`` differ only in the shape of obs/reward (per-env rows vs per-UE rows).
"""
from __future__ import annotations

import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(_HERE, "layouts.json")) as _f:
    LAYOUTS = {k: v for k, v in json.load(_f).items() if not k.startswith("_")}

SCENARIOS = {}
for _size in ("small", "medium", "large"):
    for _mode in ("central", "ma"):
        SCENARIOS[f"mobile-{_size}-{_mode}-v0"] = dict(
            layout=_size, mode=_mode, num_ues=LAYOUTS[_size]["num_ues"],
            num_bs=len(LAYOUTS[_size]["bs"]), velocity=None, per_env_layout=False)
# custom 128 BS x 1024 UE Okumura-Hata stress scenario: one random BS layout per env
# (uniform integer positions in the 200x200 map, seeded by the env's seed), velocity 10
# as in MComCustom (custom.py:16-18).
# mobile-large sizes (13 BS x 30 UE) with one random station layout per env (uniform integer
# positions, seeded by the env's seed): the per-env-layout path of the packed kernels (the
# UE x station distance scan; MComCustom and layout search run it).
SCENARIOS["mobile-large-perenv-v0"] = dict(
    layout=None, mode="central", num_ues=LAYOUTS["large"]["num_ues"],
    num_bs=len(LAYOUTS["large"]["bs"]), velocity=None, per_env_layout=True)
SCENARIOS["mobile-custom-128x1024-v0"] = dict(
    layout=None, mode="central", num_ues=1024, num_bs=128, velocity=10,
    per_env_layout=True)


def spec(env_id: str) -> dict:
    if env_id not in SCENARIOS:
        raise KeyError(f"unknown scenario {env_id!r}; known: {sorted(SCENARIOS)}")
    return dict(SCENARIOS[env_id])
