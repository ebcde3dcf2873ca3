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

# mobile-large sizes and layout with heterogeneous entities (entities.py:7-22,33-45: every
# station / UE carries its own parameters): three station classes {bw, freq, tx, height} and
# three UE classes {velocity, snr_tr, noise, height}, station j in class j % 3, UE u in class
# 7u % 3 -- the parameter mix of the reference fixture large_mixed (tests/golden/make_golden.py)
SCENARIOS["mobile-large-mixed-v0"] = dict(
    layout="large", mode="central", num_ues=LAYOUTS["large"]["num_ues"],
    num_bs=len(LAYOUTS["large"]["bs"]), velocity=None, per_env_layout=False,
    classes=dict(
        bs_classes=[{"bw": 9e6, "freq": 2500, "tx": 40, "height": 50},
                    {"bw": 9e6, "freq": 2500, "tx": 30, "height": 50},
                    {"bw": 5e6, "freq": 1800, "tx": 35, "height": 30}],
        ue_classes=[{"velocity": 1.5, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.6},
                    {"velocity": 10, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.8},
                    {"velocity": 3, "snr_tr": 1e-7, "noise": 2e-9, "height": 1.5}],
        bs_class=[j % 3 for j in range(len(LAYOUTS["large"]["bs"]))],
        ue_class=[(7 * u) % 3 for u in range(LAYOUTS["large"]["num_ues"])]))


def spec(env_id: str) -> dict:
    if env_id not in SCENARIOS:
        raise KeyError(f"unknown scenario {env_id!r}; known: {sorted(SCENARIOS)}")
    return dict(SCENARIOS[env_id])
