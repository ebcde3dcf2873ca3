"""MComCustom (reference scenarios/custom.py:12-86) over the GPU engine.

7 UEs at velocity 10; on every reset a fresh layout of randint(5, 10) stations at
int(uniform(0, 200)) positions is drawn from Python's global ``random`` module (the same
module and call order as the reference, so ``random.seed(k)`` reproduces its layouts), and
``activeUsers`` is refilled with every UE whose start time is <= 0.
"""
from __future__ import annotations

import json
import os
import random

import numpy as np

from mobile_env.core.base import MComCore
from mobile_env.core.entities import BaseStation, UserEquipment


class MComCustom(MComCore):
    _first_step_active = True

    @classmethod
    def default_config(cls):
        config = super().default_config()
        config["ue"].update({"velocity": 10})
        return config

    def __init__(self, config=None, render_mode=None):
        self.mb_iso_lines = None
        self.conn_iso_lines = None
        if config is None:
            config = {}
        # like the reference, entities are built from the class defaults (custom.py:27,33-36)
        users = [UserEquipment(ue_id=i, **self.default_config()["ue"]) for i in range(7)]
        super().__init__([], users, config, render_mode)

    def reset(self, *, seed=None):
        # station layout first: the engine is (re)built for the new layout inside reset
        stations = self.generate_base_stations(self.default_config())
        self.stationDict = {bs.bs_id: bs for bs in stations}
        self.NUM_STATIONS = len(self.stationDict)
        super().reset()
        if seed is not None:
            self.seed = seed
        self.rng = np.random.default_rng(self.seed)
        self.activeUsers = sorted([ue for ue in self.userDict.values() if ue.startTime <= 0],
                                  key=lambda ue: ue.ue_id)
        self.NUM_USERS = len(self.userDict)
        self.conn_iso_lines = None
        self.mb_iso_lines = None
        self.users_dataRateList = {ue.ue_id: [] for ue in self.userDict.values()}
        self.users_trajectoryList = {ue.ue_id: [] for ue in self.userDict.values()}

    @staticmethod
    def generate_base_stations(env_config):
        num_stations = random.randint(5, 10)
        stations = []
        for bs_id in range(num_stations):
            x = int(random.uniform(0, 200))
            y = int(random.uniform(0, 200))
            stations.append(BaseStation(bs_id=bs_id, pos=(x, y), **env_config["bs"]))
        return stations

    def save_base_station_positions(self, epoch_number):
        root = self.dump_root if self.dump_root is not None else ".."
        path = os.path.join(root, "collectData2", "BaseStationPosition",
                            f"stations_{epoch_number}.json")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump({bs.bs_id: (bs.point.x, bs.point.y) for bs in self.stationDict.values()}, f)
