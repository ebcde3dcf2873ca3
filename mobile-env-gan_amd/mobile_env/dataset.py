"""Dataset writer: the reference's per-step / per-episode data collection for a batched engine
(SURVEY.md §8f row 1).

The reference writes, for its single env, one JSON file per kind and step
(``save_layout_and_data_rates``, base.py:298-349) and, per episode, three CSV histories
(``save_epoch_data``, base.py:351-404) plus the episode's station layout
(``MComCustom.save_base_station_positions``, custom.py:79-86); the GNN and analysis notebooks
read the per-step JSON files (GNN.ipynb cell 1, analysisData.ipynb cell 0). This module
produces the same files, byte for byte, for any subset of the envs of a
:class:`~mobile_env.core.engine.StepEngine`:

* ``format_*`` -- pure formatting of one step / one episode (shared with the MComCore facade);
* :class:`DatasetWriter` -- after every engine step, gathers the selected envs' rows on the
  device, copies them to pinned host buffers on a side stream (no sync of the compute
  stream), and a writer thread formats and writes the files while the GPU keeps stepping.

Reproduced exactly, including what is incidental in the reference: JSON via
``json.dump(..., indent=4)``; values through python ``round(., 2)`` / numpy's round; the CSV
lists are ``str(list)`` of the reference's own element types -- a position the UE reached by a
regular move is a numpy int (``np.int64(..)``), one it snapped to (the popped waypoint) a
python int; a connected UE's rate is ``np.float64(..)``, an unconnected one's python ``0.0``;
the utility of a positive rate is ``np.float64(..)``, of a zero rate python ``-1.0``.
One documented difference: within a station the reference lists its UEs in python ``set``
order (object hashes, i.e. run-dependent); here they are in ``ue_id`` order.
"""
from __future__ import annotations

import json
import os
import queue
import threading
from typing import Callable, Dict, Optional

import numpy as np

__all__ = ["format_step_files", "format_station_positions", "EpisodeHistory", "DatasetWriter"]


def _dumps(obj, indent=4) -> str:
    return json.dumps(obj, indent=indent)


def format_step_files(epoch: int, step: int, bs_xy, ue_xy, serving, rate64, util64,
                      active) -> Dict[str, str]:
    """The four collectData JSON files of one env-step (base.py:298-349).

    bs_xy [B,2] int, ue_xy [U,2] int, serving [U] int (-1: none), rate64 / util64 [U] float64
    (the step's exact rounded rates and scaled utilities), active [U] bool."""
    tag = f"{epoch}_{step}"
    bs = [{"bs_id": j, "x": round(float(x), 2), "y": round(float(y), 2)}
          for j, (x, y) in enumerate(np.asarray(bs_xy).tolist())]
    ues = [{"ue_id": i, "x": round(float(x), 2), "y": round(float(y), 2)}
           for i, (x, y) in enumerate(np.asarray(ue_xy).tolist())]
    srv = np.asarray(serving)
    act = np.asarray(active, dtype=bool)
    rate = np.asarray(rate64, dtype=np.float64)
    conn = (srv >= 0) & act
    order = np.lexsort((np.arange(len(srv)), srv))  # by station, then ue_id
    rates = [{"ue_id": int(i), "bs_id": int(srv[i]), "data_rate": round(float(rate[i]), 2)}
             for i in order if conn[i]]
    # ue_utilities holds the active UEs; the others read 0.0 (base.py:340)
    util = np.asarray(util64, dtype=np.float64)
    qoe = [{"ue_id": i, "qoe": float(np.round(util[i], 2)) if act[i] else 0.0}
           for i in range(len(srv))]
    return {
        os.path.join("collectData", "BaseStationPosition", f"stations_info_{tag}.json"): _dumps(bs),
        os.path.join("collectData", "UserEquipmentPosition", f"user_positions_{tag}.json"): _dumps(ues),
        os.path.join("collectData", "DataRate", f"data_rates_{tag}.json"): _dumps(rates),
        os.path.join("collectData", "UserQoE", f"user_qoe_{tag}.json"): _dumps(qoe),
    }


def format_station_positions(epoch: int, bs_xy) -> Dict[str, str]:
    """collectData2/BaseStationPosition/stations_{epoch}.json (custom.py:79-86)."""
    pos = {j: (float(x), float(y)) for j, (x, y) in enumerate(np.asarray(bs_xy).tolist())}
    return {os.path.join("collectData2", "BaseStationPosition", f"stations_{epoch}.json"):
            json.dumps(pos)}


def _np_float(v: float) -> str:
    return f"np.float64({float(v)!r})"


class EpisodeHistory:
    """One env's per-episode histories (base.py:264-269), rendered like ``save_epoch_data``."""

    def __init__(self, num_ues: int):
        self.U = num_ues
        self.rates = [[] for _ in range(num_ues)]
        self.traj = [[] for _ in range(num_ues)]
        self.qoe = [[] for _ in range(num_ues)]

    def add(self, ue_xy, snapped, serving, rate64, util64, active):
        xy = np.asarray(ue_xy).tolist()
        srv = np.asarray(serving)
        rate = np.asarray(rate64, dtype=np.float64)
        util = np.asarray(util64, dtype=np.float64)
        for i in range(self.U):
            if not active[i]:
                continue
            connected = srv[i] >= 0
            r = round(float(rate[i]), 2)
            self.rates[i].append(_np_float(r) if connected else repr(0.0))
            x, y = xy[i]
            self.traj[i].append(f"({x}, {y})" if snapped[i]
                                else f"(np.int64({x}), np.int64({y}))")
            q = float(np.round(util[i], 2))
            self.qoe[i].append(_np_float(q) if connected and rate[i] > 0.0 else repr(q))

    @staticmethod
    def _csv(col: str, rows) -> str:
        lines = [f"User ID,{col}"]
        for i, items in enumerate(rows):
            cell = "[" + ", ".join(items) + "]"
            lines.append(f'{i},"{cell}"' if "," in cell else f"{i},{cell}")
        return "\n".join(lines) + "\n"

    def files(self, epoch: int) -> Dict[str, str]:
        """The three collectData2 CSVs; like the reference, nothing after the first empty
        history (base.py:353-404 return early)."""
        out = {}
        for sub, name, col, rows in (
                ("DataRate", f"datarates_{epoch}.csv", "Data Rates", self.rates),
                ("UserEquipmentPosition", f"user_positions_{epoch}.csv", "Trajectory", self.traj),
                ("UserQoE", f"user_qoe_{epoch}.csv", "QoE", self.qoe)):
            if not rows:
                break
            out[os.path.join("collectData2", sub, name)] = self._csv(col, rows)
        return out


def write_files(root: str, files: Dict[str, str]) -> None:
    for rel, text in files.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(text)


class DatasetWriter:
    """Asynchronous collectData / collectData2 writer for envs of a StepEngine.

    ``record()`` after every ``engine.step(1)`` (the engine needs ``rate64`` and ``util64``,
    the exact float64 outputs). ``envs``: indices of the envs to dump (default: all).
    ``epoch_of(env_index, episode_index)`` names an env's episode in the file names (default:
    ``episode_index * len(envs) + position of the env in envs``, so one env gives the
    reference driver's numbering). The first recorded step of each env must be step 0 of an
    episode. ``close()`` drains the queue; files of an episode's CSVs appear after its last
    step has been recorded."""

    def __init__(self, engine, root: str, envs=None, epoch_of: Optional[Callable] = None,
                 depth: int = 8, station_positions: bool = True,
                 episode_steps: Optional[int] = None):
        import torch
        eng = getattr(engine, "engine", engine)
        if eng.rate64 is None or eng.util64 is None:
            raise ValueError("DatasetWriter needs an engine built with rate64=True, util64=True")
        self.eng = eng
        self.root = root
        E = eng.p.num_envs
        self.envs = np.arange(E) if envs is None else np.asarray(envs, dtype=np.int64)
        self._sel = torch.as_tensor(self.envs, device=eng.device)
        self.n = len(self.envs)
        self.epoch_of = epoch_of or (lambda e, k, _pos={int(v): i for i, v in
                                                         enumerate(self.envs)}, _n=self.n:
                                     k * _n + _pos[int(e)])
        self.station_positions = station_positions
        # the driver's save_epoch_data after this many steps (default: the episode length)
        self.episode_steps = episode_steps or eng.p.t_end
        self._stream = torch.cuda.Stream(device=eng.device)
        self._free = queue.Queue()
        for _ in range(depth):
            self._free.put(None)
        self._work = queue.Queue()
        self._episode = np.full(self.n, -1, dtype=np.int64)
        self._hist = [None] * self.n
        self._error = None
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()

    # -- producer (caller's thread) ----------------------------------------------------------
    def record(self) -> None:
        import torch
        if self._error is not None:
            raise RuntimeError("dataset writer failed") from self._error
        self._free.get()  # back-pressure: at most `depth` steps in flight
        eng, sel = self.eng, self._sel
        cur = torch.cuda.current_stream(eng.device)
        dev = {
            "state": eng.ue_state.index_select(0, sel),
            "serving": eng.serving.index_select(0, sel),
            "rate": eng.rate64.index_select(0, sel),
            "util": eng.util64.index_select(0, sel),
            "t": eng.t.index_select(0, sel),
        }
        if eng.bs_per_env:
            dev["bs"] = eng.bs_xy.index_select(0, sel)
            if eng.bs_count is not None:
                dev["bs_count"] = eng.bs_count.index_select(0, sel)
        else:
            dev["bs"] = eng.bs_xy
        self._stream.wait_stream(cur)
        host = {}
        with torch.cuda.stream(self._stream):
            for k, v in dev.items():
                h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                h.copy_(v, non_blocking=True)
                v.record_stream(self._stream)
                host[k] = h
            ev = torch.cuda.Event()
            ev.record(self._stream)
        self._work.put((ev, host))

    def close(self) -> None:
        self._work.put(None)
        self._thread.join()
        if self._error is not None:
            raise RuntimeError("dataset writer failed") from self._error

    # -- consumer (writer thread) -------------------------------------------------------------
    def _run(self):
        try:
            while True:
                item = self._work.get()
                if item is None:
                    return
                ev, host = item
                ev.synchronize()
                self._write_step({k: v.numpy() for k, v in host.items()})
                self._free.put(None)
        except BaseException as exc:  # surfaced by the next record() / close()
            self._error = exc
            self._free.put(None)

    def _write_step(self, h):
        p = self.eng.p
        for i in range(self.n):
            t = int(h["t"][i])  # time after the step: curr_step = t - 1
            step = t - 1
            if step == 0:
                self._episode[i] += 1
                self._hist[i] = EpisodeHistory(p.num_ues)
            if self._episode[i] < 0:
                raise RuntimeError("the first recorded step of an env must be step 0")
            epoch = int(self.epoch_of(int(self.envs[i]), int(self._episode[i])))
            bs = h["bs"][i] if self.eng.bs_per_env else h["bs"]
            if "bs_count" in h:
                bs = bs[: int(h["bs_count"][i])]
            st = h["state"][i].astype(np.int64)
            xy, wpx = st[:, :2], st[:, 2]
            util = h["util"][i]
            active = ~np.isnan(util)
            files = {}
            if step == 0 and self.station_positions:
                files.update(format_station_positions(epoch, bs))
            files.update(format_step_files(epoch, step, bs, xy, h["serving"][i], h["rate"][i],
                                           util, active))
            self._hist[i].add(xy, active & (wpx < 0), h["serving"][i], h["rate"][i], util,
                              active)
            if step == self.episode_steps - 1:
                files.update(self._hist[i].files(epoch))
            write_files(self.root, files)
