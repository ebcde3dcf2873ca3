"""Batched Gymnasium-style surface: ``make(id, num_envs, device)`` -> VectorMobileEnv.

The reference has no Gym surface left (MComCore has no base class, no spaces, no
reward/terminated/truncated; step returns None, base.py:28,230,296). This is the
build-defined surface the north star asks for, over E independent envs on one GPU:

* ``reset(seed=None) -> (obs, info)``
* ``step(action=None) -> (obs, reward, terminated, truncated, info)``; the reference has no
  action input (association is automatic, base.py:236-241), so ``action`` is accepted and
  ignored.
* obs = per-UE rows (x/W, y/H, data rate, scaled utility); ``central``: obs [E, U*4],
  reward [E] = mean utility (metrics.py:25-28); ``ma``: obs [E, U, 4], reward [E, U] = each
  UE's scaled utility.
* Episodes end by time limit (EP_MAX_TIME = 20): ``truncated`` is set on the last step and
  the env auto-resets at the start of its next step (``terminated`` is always False).

Returned tensors are views of the engine's device buffers and are overwritten by the next
step (zero-copy); clone them to keep them.
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from .core.engine import EngineParams, StepEngine
from .core.util import deep_dict_merge
from .scenarios import registry


class Box(NamedTuple):
    low: float
    high: float
    shape: tuple
    dtype: torch.dtype


def default_config() -> dict:
    from .core.base import MComCore
    return MComCore.default_config()


def _bs_layouts(spec, num_envs, seeds, device):
    if not spec["per_env_layout"]:
        return registry.LAYOUTS[spec["layout"]]["bs"], None
    # one uniform-integer layout per env, seeded by the env's seed (synthetic scenario)
    B = spec["num_bs"]
    out = torch.empty((num_envs, B, 2), dtype=torch.int32)
    g = torch.Generator()
    for e in range(num_envs):
        g.manual_seed(int(seeds[e]))
        out[e] = torch.randint(0, 200, (B, 2), generator=g, dtype=torch.int32)
    return out, None


class VectorMobileEnv:
    def __init__(self, env_id: str, num_envs: int = 1, device=None, seed: int = 2024,
                 config: Optional[dict] = None, metrics: bool = False, rate64: bool = False,
                 util64: bool = False, stream_split: int = 0, fuse_steps: int = 0,
                 **launch):
        """launch: EngineParams launch-shape overrides (lds_tables, two_groups, stage_rows,
        xcd_remap, scenario_constants; default 0 = automatic)."""
        spec = registry.spec(env_id)
        cfg = deep_dict_merge(default_config(), config or {})
        if spec["velocity"] is not None:
            cfg["ue"]["velocity"] = spec["velocity"]
        self.env_id = env_id
        self.mode = spec["mode"]
        self.num_envs = int(num_envs)
        self.num_ues = spec["num_ues"]
        self.num_bs = spec["num_bs"]
        self.seeds = torch.arange(self.num_envs, dtype=torch.int64) + int(seed)
        bs_xy, bs_count = _bs_layouts(spec, self.num_envs, self.seeds.tolist(), device)
        p = EngineParams(
            num_envs=self.num_envs, num_ues=self.num_ues, num_bs=self.num_bs,
            width=cfg["width"], height=cfg["height"], ep_max_time=cfg["EP_MAX_TIME"],
            arrival_start=0, arrival_exit=cfg["arrival_params"]["ep_time"],
            first_step_active=True,
            movement_reseed=cfg["movement_params"].get("reset_rng_episode", True),
            velocity=cfg["ue"]["velocity"],
            bs=dict(cfg["bs"]),
            ue={k: cfg["ue"][k] for k in ("snr_tr", "noise", "height")},
            util_lower=cfg["utility_params"]["lower"], util_upper=cfg["utility_params"]["upper"],
            util_coeffs=tuple(cfg["utility_params"]["coeffs"]),
            stream_split=stream_split, fuse_steps=fuse_steps,
            **{k: v for k, v in (spec.get("classes") or {}).items()}, **launch)
        self.engine = StepEngine(p, bs_xy, self.seeds.numpy(), bs_count=bs_count, device=device,
                                 metrics=metrics, rate64=rate64, util64=util64)
        U = self.num_ues
        if self.mode == "central":
            self.single_observation_space = Box(-float("inf"), float("inf"), (U * 4,),
                                                torch.float32)
        else:
            self.single_observation_space = Box(-float("inf"), float("inf"), (U, 4),
                                                torch.float32)
        self.single_action_space = None  # the reference has no action input
        # preallocated, so step() launches nothing but the step kernel
        self._terminated = torch.zeros((self.num_envs,), dtype=torch.bool, device=self.device)

    @property
    def device(self):
        return self.engine.device

    def _views(self):
        e = self.engine
        if self.mode == "central":
            return e.obs.view(self.num_envs, -1), e.reward
        return e.obs, e.obs[..., 3]

    def reset(self, seed=None, options=None):
        if seed is not None:
            self.seeds = torch.as_tensor(seed, dtype=torch.int64).reshape(-1)
            if self.seeds.numel() == 1:
                self.seeds = self.seeds + torch.arange(self.num_envs, dtype=torch.int64)
            self.engine.seed(self.seeds.numpy())
        self.engine.reset()
        obs, _ = self._views()
        return obs, {"serving": self.engine.serving}

    def step(self, action=None):
        self.engine.step(1)
        obs, reward = self._views()
        e = self.engine
        truncated = e.done.view(torch.bool)  # zero-copy view of the kernel's u8 flags
        terminated = self._terminated
        info = {"serving": e.serving}
        if e.metrics is not None:
            info["metrics"] = e.metrics
        return obs, reward, terminated, truncated, info

    def close(self):
        self.engine.close()


def make(env_id: str, num_envs: int = 1, device=None, **kwargs) -> VectorMobileEnv:
    return VectorMobileEnv(env_id, num_envs=num_envs, device=device, **kwargs)
