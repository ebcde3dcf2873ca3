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


def _classes(values):
    """(distinct values in order of first appearance, class index of every entity)."""
    classes, index = [], []
    for v in values:
        if v not in classes:
            classes.append(v)
        index.append(classes.index(v))
    if not classes:
        raise ValueError("no entities")
    return classes, index


def lower(*, num_envs, stations, users, arrival, channel, scheduler, movement, utility,
          ep_max_time, first_step_active) -> EngineParams:
    """Flat engine parameters. Entities with different parameters (the reference keeps them
    per BaseStation / UserEquipment, entities.py:7-22,33-45) lower to parameter classes: one
    channel table per (station class, UE class) pair, the classes over the channel-relevant
    values only; the velocity (movement only, movement.py:42-62) goes per UE, any number of
    distinct values."""
    check_plugins(arrival, channel, scheduler, movement, utility)
    bsc, bsi = _classes([(s.bw, s.frequency, s.tx_power, s.height) for s in stations])
    uec, uei = _classes([(u.snr_threshold, u.noise, u.height) for u in users])
    vels = [float(u.velocity) for u in users]
    if len(bsc) > 16 or len(uec) > 16:
        raise NotImplementedError("more than 16 station or UE channel parameter classes "
                                  "(distinct (bw, freq, tx, height) / (snr_tr, noise, height))")
    mv = movement.lower_params()
    ar = arrival.lower_params()
    ut = utility.lower_params()
    bs_dicts = [{"bw": b[0], "freq": b[1], "tx": b[2], "height": b[3]} for b in bsc]
    ue_dicts = [{"velocity": vels[uei.index(c)], "snr_tr": u[0], "noise": u[1], "height": u[2]}
                for c, u in enumerate(uec)]
    het = len(bsc) > 1 or len(uec) > 1
    per_ue_vel = len(set(vels)) > 1
    return EngineParams(
        num_envs=num_envs, num_ues=len(users), num_bs=len(stations),
        width=mv["width"], height=mv["height"], ep_max_time=int(ep_max_time),
        arrival_start=ar["arrival_start"], arrival_exit=ar["arrival_exit"],
        first_step_active=first_step_active, movement_reseed=mv["movement_reseed"],
        velocity=vels[0], bs=bs_dicts[0],
        ue={k: ue_dicts[0][k] for k in ("snr_tr", "noise", "height")},
        util_lower=ut["util_lower"], util_upper=ut["util_upper"], util_coeffs=ut["util_coeffs"],
        draw_table=0,  # the facade carries pcg / t across engine rebuilds: no episode table
        bs_classes=bs_dicts if het else None, ue_classes=ue_dicts if het else None,
        bs_class=bsi if het else None, ue_class=uei if het else None,
        ue_velocity=vels if per_ue_vel else None)
