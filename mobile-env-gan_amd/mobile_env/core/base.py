"""MComCore facade: the reference's single-env object API on top of the batched GPU engine.

Mirrors ``MComCore`` (reference core/base.py:28-753) -- same constructor, config schema
(``default_config``/``seeding``/deep merge), plugin attributes, ``reset``/``step`` and the
per-step bookkeeping attributes (``activeUsers``, ``bs2ue_connections``,
``bs2ue_dataRates``, ``allUserDataRates``, ``ue_utilities``, ``monitor``, history lists) --
so code written against the reference keeps working. The step itself is one launch of the
fused HIP kernel on a 1-env :class:`~mobile_env.core.engine.StepEngine`; its results are
copied back into the entity objects and dicts after every step. For throughput use the
batched surface (:func:`mobile_env.make`).

Differences, all documented in DESIGN.md: rendering is not provided (out of scope); plugin
objects are lowered to kernels (only the built-in classes); the per-step JSON dump is
written only when ``config["dump_root"]`` is set (the reference always writes to ``..``).
"""
from __future__ import annotations

import json
import os
from collections import Counter, defaultdict
from typing import Dict, List, Set, Tuple

import numpy as np

from . import lowering, metrics
from .arrival import NoDeparture
from .channels import OkumuraHata
from .entities import BaseStation, UserEquipment
from .engine import StepEngine
from .logging import Monitor
from .movement import RandomWaypointMovement
from .schedules import ResourceFair
from .util import deep_dict_merge
from .utilities import BoundedLogUtility


class MComCore:
    NOOP_ACTION = 0
    metadata = {"render_modes": ["rgb_array", "human"]}
    # Bare MComCore.reset never refills activeUsers (base.py:75,172-209), so the first step of
    # an episode moves nobody; MComCustom refills it (custom.py:53-54).
    _first_step_active = False

    def __init__(self, stations: List[BaseStation], users: List[UserEquipment], config=None,
                 render_mode=None):
        self.max_departure = None
        if config is None:
            config = {}
        self.render_mode = render_mode
        assert render_mode in self.metadata["render_modes"] + [None]
        config = deep_dict_merge(self.default_config(), config)
        config = self.seeding(config)
        self.config = config

        self.width, self.height = config["width"], config["height"]
        self.seed = config["seed"]
        self.reset_rng_episode = config["reset_rng_episode"]
        self.rng = None

        self.arrivalModel = config["arrival"](**config["arrival_params"])
        self.channelModel = config["channel"](**config["channel_params"])
        self.schedulerModel = config["scheduler"](**config["scheduler_params"])
        self.movementModel = config["movement"](**config["movement_params"])
        self.utilityModel = config["utility"](**config["utility_params"])
        lowering.check_plugins(self.arrivalModel, self.channelModel, self.schedulerModel,
                               self.movementModel, self.utilityModel)

        self.EP_MAX_TIME = config["EP_MAX_TIME"]
        self.time = None
        self.closed = False

        self.stationDict = {bs.bs_id: bs for bs in stations}
        self.userDict = {ue.ue_id: ue for ue in users}
        self.NUM_STATIONS = len(self.stationDict)
        self.NUM_USERS = len(self.userDict)

        self.activeUsers: List[UserEquipment] = []
        self.bs2ue_connections: Dict[BaseStation, Set[UserEquipment]] = {}
        self.bs2ue_dataRates: Dict[Tuple[BaseStation, UserEquipment], float] = {}
        self.ue_utilities: Dict[UserEquipment, float] = {}
        self.allUserDataRates = None

        config["metrics"]["scalar_metrics"].update({
            "number connections": metrics.number_connections,
            "number connected": metrics.number_connected,
            "mean utility": metrics.mean_utility,
            "mean datarate": metrics.mean_datarate,
        })
        self.monitor = Monitor(**config["metrics"])

        self.users_trajectoryList = None
        self.users_dataRateList = None
        self.userQoEList = None

        self.dump_root = config.get("dump_root")
        self.device = config.get("device")
        self._engine = None
        self._engine_key = None
        self._metric_values = (0, 0, float(self.utilityModel.lower), 0.0)

    # -- config (base.py:102-170) -------------------------------------------------------------
    @classmethod
    def default_config(cls):
        width, height = 200, 200
        ep_time = 20
        config = {
            "width": width, "height": height, "EP_MAX_TIME": ep_time, "seed": 2024,
            "reset_rng_episode": False,
            "arrival": NoDeparture, "channel": OkumuraHata, "scheduler": ResourceFair,
            "movement": RandomWaypointMovement, "utility": BoundedLogUtility,
            "bs": {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50},
            "ue": {"velocity": 1.5, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.6},
        }
        config["arrival_params"] = {"ep_time": ep_time, "reset_rng_episode": False}
        config["channel_params"] = {}
        config["scheduler_params"] = {}
        config["movement_params"] = {"width": width, "height": height, "reset_rng_episode": True}
        config["utility_params"] = {"lower": -20, "upper": 20, "coeffs": (10, 0, 10)}
        config["metrics"] = {"scalar_metrics": {}, "ue_metrics": {}, "bs_metrics": {}}
        return config

    @classmethod
    def seeding(cls, config):
        seed = config["seed"]
        for num, key in enumerate(("arrival_params", "channel_params", "scheduler_params",
                                   "movement_params", "utility_params")):
            config.setdefault(key, {})
            config[key]["seed"] = seed + num + 1
        return config

    # -- engine management ----------------------------------------------------------------------
    def _stations(self):
        return list(self.stationDict.values())

    def _users(self):
        return [self.userDict[k] for k in sorted(self.userDict)]

    def _ensure_engine(self):
        stations, users = self._stations(), self._users()
        key = (tuple((bs.bs_id, bs.point, bs.bw, bs.frequency, bs.tx_power, bs.height)
                     for bs in stations),
               tuple((u.ue_id, u.velocity, u.snr_threshold, u.noise, u.height) for u in users))
        if self._engine is not None and key == self._engine_key:
            return self._engine
        carry = None
        if self._engine is not None:  # new layout (MComCustom): keep the movement stream
            carry = (self._engine.pcg.clone(), self._engine.t.clone())  # (pcg: synced)
            self._engine.close()
        p = lowering.lower(num_envs=1, stations=stations, users=users,
                           arrival=self.arrivalModel, channel=self.channelModel,
                           scheduler=self.schedulerModel, movement=self.movementModel,
                           utility=self.utilityModel, ep_max_time=self.EP_MAX_TIME,
                           first_step_active=self._first_step_active)
        bs_xy = [list(bs.point) for bs in stations]
        # the movement plugin carries its own seed (config seed + 4 via seeding()); the
        # engine adds 4 to a *config* seed, so hand it movement.seed - 4
        self._engine = StepEngine(p, bs_xy, [self.movementModel.seed - 4], device=self.device,
                                  rate64=True, util64=True, metrics=True)
        if carry is not None:
            self._engine._pcg.copy_(carry[0])
            self._engine.t.copy_(carry[1])
        self._engine_key = key
        return self._engine

    # -- reset (base.py:172-209) ------------------------------------------------------------------
    def reset(self, *, seed=None):
        self.time = 0.0
        if seed is not None:
            self.seed = seed  # like the reference, plugins keep their construction seeds
        if self.reset_rng_episode or self.rng is None:
            self.rng = np.random.default_rng(self.seed)
        for m in (self.arrivalModel, self.channelModel, self.schedulerModel,
                  self.movementModel, self.utilityModel):
            m.reset()
        for ue in self.userDict.values():
            ue.startTime = self.arrivalModel.setArrivalTime(ue)
            ue.exitTime = self.arrivalModel.setDepartureTime(ue)
        eng = self._ensure_engine()
        eng.reset()
        xy = eng.ue_xy[0].cpu().tolist()
        for ue, (x, y) in zip(self._users(), xy):
            ue.x, ue.y = int(x), int(y)
        self.bs2ue_connections = defaultdict(set)
        self.bs2ue_dataRates = defaultdict(float)
        self.ue_utilities = {}
        self.max_departure = max(ue.exitTime for ue in self.userDict.values())
        self.monitor.reset()
        self.userQoEList = {ue.ue_id: [] for ue in self.userDict.values()}
        if self.users_dataRateList is None:
            self.users_dataRateList = {ue.ue_id: [] for ue in self.userDict.values()}
        if self.users_trajectoryList is None:
            self.users_trajectoryList = {ue.ue_id: [] for ue in self.userDict.values()}

    # -- step (base.py:230-296) -------------------------------------------------------------------
    def step(self, epoch_number=None, curr_step=None):
        eng = self._ensure_engine()
        eng.step(1)
        users = self._users()
        state = eng.ue_state[0].cpu().tolist()
        srv = eng.serving[0].cpu().tolist()
        rate = eng.rate64[0].cpu().tolist()
        util = eng.util64[0].cpu().tolist()
        self._metric_values = tuple(eng.metrics[0].double().cpu().tolist())
        active = set(self.activeUsers)
        # the reference's value types (they show in save_epoch_data's CSVs): a regular move
        # yields numpy ints (movement.py:58-60), a snap the popped waypoint's python ints
        # (movement.py:53-54); a connected UE's rate and the utility of a positive rate are
        # numpy floats, the rest python floats (base.py:421-435, utilities.py:45-53)
        for ue, (x, y, wx, _) in zip(users, state):
            snapped = ue in active and wx < 0
            ue.x, ue.y = (int(x), int(y)) if snapped else (np.int64(x), np.int64(y))
        stations = self._stations()
        self.bs2ue_connections = defaultdict(set)
        self.bs2ue_dataRates = {}
        by_station = defaultdict(list)
        for ue, b in zip(users, srv):
            if b >= 0 and ue in active:
                by_station[b].append(ue)
        for b in sorted(by_station):  # station order, like the reference's dict iteration
            bs = stations[b]
            for ue in by_station[b]:
                self.bs2ue_connections[bs].add(ue)
                self.bs2ue_dataRates[(bs, ue)] = np.float64(rate[ue.ue_id])
        self.allUserDataRates = self.user_total_datarates(self.bs2ue_dataRates)
        self.ue_utilities = {
            ue: (np.float64(util[ue.ue_id]) if srv[ue.ue_id] >= 0 and rate[ue.ue_id] > 0.0
                 else float(util[ue.ue_id]))
            for ue in self.activeUsers}

        if self.dump_root is not None:
            self.save_layout_and_data_rates(epoch_number, curr_step)

        for ue in self.activeUsers:
            datarate = self.allUserDataRates.get(ue, 0.0)
            self.users_dataRateList[ue.ue_id].append(round(datarate, 2))
            self.users_trajectoryList[ue.ue_id].append((ue.x, ue.y))
            self.userQoEList[ue.ue_id].append(round(self.ue_utilities.get(ue, 0.0), 2))

        self.monitor.update(self)
        self.time += 1
        leaving = {ue for ue in self.activeUsers if ue.exitTime <= self.time}
        for bs, ues in self.bs2ue_connections.items():
            self.bs2ue_connections[bs] = ues - leaving
        self.activeUsers = sorted(
            [ue for ue in self.userDict.values() if ue.exitTime > self.time >= ue.startTime],
            key=lambda ue: ue.ue_id)
        return None

    # -- helpers with the reference's names ---------------------------------------------------------
    @property
    def time_is_up(self):
        return self.time >= min(self.EP_MAX_TIME, self.max_departure)

    def check_connectivity(self, bs: BaseStation, ue: UserEquipment) -> bool:
        """base.py:212-214: snr > snr_tr, by the channel plugin (the step's kernels use the
        equivalent integer test d2 <= d2max of the pair's parameter classes)."""
        return self.channelModel.calculateSNR(bs, ue) > ue.snr_threshold

    def available_connections(self, ue: UserEquipment) -> Set:
        return {bs for bs in self.stationDict.values() if self.check_connectivity(bs, ue)}

    def update_connections(self) -> None:
        kept = {bs: {ue for ue in ues if self.check_connectivity(bs, ue)}
                for bs, ues in self.bs2ue_connections.items()}
        self.bs2ue_connections.clear()
        self.bs2ue_connections.update(kept)

    def user_total_datarates(self, bs2ue_dataRates):
        totals = Counter()
        for (bs, ue), r in bs2ue_dataRates.items():
            totals.update({ue: r})
        return totals

    def allocateDataRate2User(self, bs) -> Dict:
        """Rates the last step's kernel allocated at ``bs`` (base.py:421-435)."""
        return {(b, ue): r for (b, ue), r in self.bs2ue_dataRates.items() if b is bs}

    def allStationUtilities(self) -> Dict:
        idle = self.utilityModel.scaleUtility(self.utilityModel.lower)
        return {bs: (sum(self.ue_utilities[ue] for ue in self.bs2ue_connections[bs])
                     / len(self.bs2ue_connections[bs])) if self.bs2ue_connections.get(bs) else idle
                for bs in self.stationDict.values()}

    # -- dataset dump (base.py:298-404; next-row 1 of SURVEY.md 8f) --------------------------------
    def _dump(self, sub, fname, obj, indent=4):
        path = os.path.join(self.dump_root, "collectData", sub, fname)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(obj, f, indent=indent)

    def save_layout_and_data_rates(self, epoch_number, curr_step):
        tag = f"{epoch_number}_{curr_step}"
        self._dump("BaseStationPosition", f"stations_info_{tag}.json",
                   [{"bs_id": bs.bs_id, "x": round(float(bs.point.x), 2),
                     "y": round(float(bs.point.y), 2)} for bs in self.stationDict.values()])
        self._dump("UserEquipmentPosition", f"user_positions_{tag}.json",
                   [{"ue_id": ue.ue_id, "x": round(float(ue.x), 2), "y": round(float(ue.y), 2)}
                    for ue in self.userDict.values()])
        self._dump("DataRate", f"data_rates_{tag}.json",
                   [{"ue_id": ue.ue_id, "bs_id": bs.bs_id, "data_rate": round(float(r), 2)}
                    for (bs, ue), r in self.bs2ue_dataRates.items()])
        self._dump("UserQoE", f"user_qoe_{tag}.json",
                   [{"ue_id": ue.ue_id, "qoe": round(self.ue_utilities.get(ue, 0.0), 2)}
                    for ue in self.userDict.values()])

    def save_epoch_data(self, epoch_number):
        import pandas as pd
        root = self.dump_root if self.dump_root is not None else ".."
        for sub, name, col, data in (
                ("DataRate", f"datarates_{epoch_number}.csv", "Data Rates",
                 self.users_dataRateList),
                ("UserEquipmentPosition", f"user_positions_{epoch_number}.csv", "Trajectory",
                 self.users_trajectoryList),
                ("UserQoE", f"user_qoe_{epoch_number}.csv", "QoE", self.userQoEList)):
            if not data:
                return
            path = os.path.join(root, "collectData2", sub, name)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            pd.DataFrame([{"User ID": k, col: v} for k, v in data.items()]).to_csv(
                path, index=False)

    # -- out of scope ---------------------------------------------------------------------------
    def render(self):
        raise NotImplementedError("rendering is out of scope for the MI355X engine")

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self.closed = True
