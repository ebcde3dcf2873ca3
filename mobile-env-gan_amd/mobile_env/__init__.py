"""mobile_env (MI355X build): vectorised mobile-env step engine.

* ``mobile_env.make(id, num_envs, device)`` -- batched Gym-style surface (vector.py)
* ``mobile_env.core``  -- the reference's plugin/entity/MComCore API (drop-in)
* ``mobile_env.scenarios.custom.MComCustom`` -- the reference's scenario
"""
__version__ = "0.1.0"


def make(env_id, num_envs=1, device=None, **kwargs):
    from .vector import make as _make
    return _make(env_id, num_envs=num_envs, device=device, **kwargs)


def registered_ids():
    from .scenarios.registry import SCENARIOS
    return sorted(SCENARIOS)
