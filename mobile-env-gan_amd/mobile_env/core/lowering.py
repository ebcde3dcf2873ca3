"""Lower a reference-style config dict + entity lists to device engine parameters.

The reference builds plugin objects from ``config[k]`` (class) and ``config[k + "_params"]``
(kwargs) with per-plugin seeds injected by ``seeding`` (base.py:47-61,156-170). The engine
needs flat constants instead. Only the built-in plugin classes have kernels; anything
else raises ``NotImplementedError`` (there is no CPU path to fall back to).
"""
from __future__ import annotations

from inspect import getattr_static

from .arrival import NoDeparture
from .channels import OkumuraHata
from .engine import EngineParams
from .movement import RandomWaypointMovement
from .schedules import ResourceFair
from .utilities import BoundedLogUtility

_BUILTIN = {
    "arrival": NoDeparture,
    "channel": OkumuraHata,
    "scheduler": ResourceFair,
    "movement": RandomWaypointMovement,
    "utility": BoundedLogUtility,
}


# the methods whose semantics the kernels implement, per plugin: a subclass of a built-in class
# that overrides none of them lowers like the built-in (the reference instantiates whatever
# class the config names, base.py:57-61); one that overrides any has no kernel
_KERNEL_METHODS = {
    "arrival": ("setArrivalTime", "setDepartureTime"),
    "channel": ("power_loss", "calculateSNR", "datarate", "snr_of_distance", "rate_table",
                "_loss", "_snr_table"),
    "scheduler": ("share",),
    "movement": ("move", "initial_position", "reset", "_draw"),
    "utility": ("calculateUtility", "scaleUtility", "unscaleUtility"),
}


def check_plugins(arrival, channel, scheduler, movement, utility):
    for key, obj in (("arrival", arrival), ("channel", channel), ("scheduler", scheduler),
                     ("movement", movement), ("utility", utility)):
        want = _BUILTIN[key]
        if not isinstance(obj, want):
            raise NotImplementedError(
                f"{key} plugin {type(obj).__name__} has no device kernel; the MI355X engine "
                f"implements {want.__name__} (reference default, base.py:112-116)")
        changed = [m for m in _KERNEL_METHODS[key]
                   if getattr_static(type(obj), m, None) is not getattr_static(want, m, None)]
        if changed:
            raise NotImplementedError(
                f"{key} plugin {type(obj).__name__} overrides {', '.join(changed)} of "
                f"{want.__name__}: the device kernel implements {want.__name__}'s semantics "
                f"only")


def _uniform(values, what):
    vals = list(values)
    if not vals:
        raise ValueError(f"no {what}")
    first = vals[0]
    for v in vals[1:]:
        if v != first:
            raise NotImplementedError(
                f"per-entity {what} parameters differ ({first} vs {v}); the engine lowers one "
                f"parameter set per batch")
    return first


def lower(*, num_envs, stations, users, arrival, channel, scheduler, movement, utility,
          ep_max_time, first_step_active) -> EngineParams:
    check_plugins(arrival, channel, scheduler, movement, utility)
    bsp = _uniform(((s.bw, s.frequency, s.tx_power, s.height) for s in stations), "station")
    uep = _uniform(((u.velocity, u.snr_threshold, u.noise, u.height) for u in users), "UE")
    mv = movement.lower_params()
    ar = arrival.lower_params()
    ut = utility.lower_params()
    return EngineParams(
        num_envs=num_envs, num_ues=len(users), num_bs=len(stations),
        width=mv["width"], height=mv["height"], ep_max_time=int(ep_max_time),
        arrival_start=ar["arrival_start"], arrival_exit=ar["arrival_exit"],
        first_step_active=first_step_active, movement_reseed=mv["movement_reseed"],
        velocity=float(uep[0]),
        bs={"bw": bsp[0], "freq": bsp[1], "tx": bsp[2], "height": bsp[3]},
        ue={"snr_tr": uep[1], "noise": uep[2], "height": uep[3]},
        util_lower=ut["util_lower"], util_upper=ut["util_upper"], util_coeffs=ut["util_coeffs"],
        draw_table=0)  # the facade carries pcg / t across engine rebuilds: no episode table
