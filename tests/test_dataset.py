"""Dataset writer against the files the reference itself wrote
(tests/golden/dump_mcom_custom.json, made by tests/golden/make_dump_golden.py running the
collectData2.ipynb driver on MComCustom).

CPU: the oracle supplies each step's state, the formatting functions of
mobile_env.dataset render it -- every file must equal the reference's byte for byte
(data_rates: the same entries; within a station the reference's order is python-set order).
GPU: the asynchronous DatasetWriter on a StepEngine, and the MComCore facade's own dump."""
import json
import os
import random

import numpy as np
import pytest

from conftest import ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden", "dump_mcom_custom.json")


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def layout(files, epoch):
    rows = json.loads(files[f"collectData/BaseStationPosition/stations_info_{epoch}_0.json"])
    return [[int(r["x"]), int(r["y"])] for r in rows]


def assert_same_files(got: dict, want: dict):
    assert sorted(got) == sorted(want)
    for k in sorted(want):
        if "/DataRate/data_rates_" in k:
            key = lambda r: (r["bs_id"], r["ue_id"])  # noqa: E731
            assert sorted(json.loads(got[k]), key=key) == sorted(json.loads(want[k]), key=key), k
            # the reference groups the entries by station in station order
            assert [r["bs_id"] for r in json.loads(got[k])] == \
                [r["bs_id"] for r in json.loads(want[k])], k
        else:
            assert got[k] == want[k], k


def read_tree(root):
    out = {}
    for dirpath, _, names in os.walk(root):
        for n in names:
            p = os.path.join(dirpath, n)
            out[os.path.relpath(p, root)] = open(p).read()
    return out


def test_golden_layouts_are_mcom_custom_draws():
    """The layouts in the golden files are MComCustom's global-random draws (the driver's
    extra reset in cell 3 takes the first one)."""
    from mobile_env.scenarios.custom import MComCustom
    g = golden()
    for run in g["runs"]:
        random.seed(run["random_seed"])
        draws = [[[bs.x, bs.y] for bs in MComCustom.generate_base_stations(
            MComCustom.default_config())] for _ in range(g["epochs"] + 1)]
        for ep in range(g["epochs"]):
            assert layout(run["files"], ep) == draws[ep + 1]


def test_formatting_reproduces_reference_files():
    from mobile_env.dataset import EpisodeHistory, format_station_positions, format_step_files
    from mobile_env.scenarios.custom import MComCustom
    from oracle.vec import OracleBatch, OracleParams
    g = golden()
    seed = MComCustom.default_config()["seed"]
    for run in g["runs"]:
        want = run["files"]
        lay0 = np.full((1, 10, 2), -1)
        l0 = layout(want, 0)
        lay0[0, :len(l0)] = l0
        ob = OracleBatch(OracleParams(velocity=10.0), lay0, 7, [seed], bs_count=[len(l0)])
        got = {}
        for ep in range(g["epochs"]):
            lay = layout(want, ep)
            ob.set_bs(0, lay)
            got.update(format_station_positions(ep, lay))
            hist = EpisodeHistory(7)
            for s in range(g["steps"]):
                o = ob.step()
                util = o["util"][0]
                active = ~np.isnan(util)
                got.update(format_step_files(ep, s, lay, o["xy"][0], o["serving"][0],
                                             o["rate"][0], util, active))
                hist.add(o["xy"][0], active & ~ob.wvalid[0], o["serving"][0], o["rate"][0],
                         util, active)
            got.update(hist.files(ep))
        assert_same_files(got, want)


def test_episode_history_csv_quoting():
    from mobile_env.dataset import EpisodeHistory
    h = EpisodeHistory(3)
    h.add([[1, 2], [3, 4], [5, 6]], [False, True, False], [0, -1, 1], [1.5, 0.0, 2.25],
          [0.25, -1.0, 0.5], [True, True, False])
    f = h.files(7)
    assert f["collectData2/DataRate/datarates_7.csv"] == \
        "User ID,Data Rates\n0,[np.float64(1.5)]\n1,[0.0]\n2,[]\n"
    assert f["collectData2/UserEquipmentPosition/user_positions_7.csv"] == \
        'User ID,Trajectory\n0,"[(np.int64(1), np.int64(2))]"\n1,"[(3, 4)]"\n2,[]\n'
    assert f["collectData2/UserQoE/user_qoe_7.csv"] == \
        "User ID,QoE\n0,[np.float64(0.25)]\n1,[-1.0]\n2,[]\n"


@pytest.mark.gpu
def test_async_writer_on_engine_matches_reference(tmp_path):
    """DatasetWriter on a 2-env StepEngine (one env per golden run, per-env layouts switched
    at the episode boundary like MComCustom.reset), one writer per env."""
    import torch
    from mobile_env.core.engine import EngineParams, StepEngine
    from mobile_env.dataset import DatasetWriter
    from mobile_env.scenarios.custom import MComCustom
    g = golden()
    runs = g["runs"]
    E = len(runs)
    seed = MComCustom.default_config()["seed"]
    lays = [[layout(r["files"], ep) for ep in range(g["epochs"])] for r in runs]

    def padded(ep):
        xy = np.full((E, 10, 2), 0, dtype=np.int32)
        cnt = np.zeros(E, dtype=np.int32)
        for e in range(E):
            xy[e, :len(lays[e][ep])] = lays[e][ep]
            cnt[e] = len(lays[e][ep])
        return xy, cnt

    xy0, cnt0 = padded(0)
    p = EngineParams(num_envs=E, num_ues=7, num_bs=10, velocity=10.0)
    eng = StepEngine(p, xy0, np.full(E, seed), bs_count=cnt0, device="cuda", rate64=True,
                     util64=True)
    writers = [DatasetWriter(eng, str(tmp_path / f"env{e}"), envs=[e]) for e in range(E)]
    for ep in range(g["epochs"]):
        if ep:
            eng.set_bs_layout(*padded(ep))
        for s in range(g["steps"]):
            eng.step()
            for w in writers:
                w.record()
    for w in writers:
        w.close()
    torch.cuda.synchronize()
    eng.close()
    for e, run in enumerate(runs):
        assert_same_files(read_tree(str(tmp_path / f"env{e}")), run["files"])


@pytest.mark.gpu
def test_facade_dump_matches_reference(tmp_path):
    """The MComCustom facade driven like collectData2.ipynb writes the reference's files."""
    from mobile_env.scenarios.custom import MComCustom
    g = golden()
    for run in g["runs"]:
        root = tmp_path / f"seed{run['random_seed']}"
        random.seed(run["random_seed"])
        env = MComCustom({"dump_root": str(root)})
        env.reset()
        for ep in range(g["epochs"]):
            env.reset()
            env.save_base_station_positions(ep)
            for s in range(g["steps"]):
                env.step(ep, s)
            env.save_epoch_data(ep)
        env.close()
        assert_same_files(read_tree(str(root)), run["files"])


def test_draw_layouts_follow_the_reference_call_order():
    from mobile_env.collect import draw_layouts
    from mobile_env.scenarios.custom import MComCustom
    random.seed(11)
    want = [[[bs.x, bs.y] for bs in MComCustom.generate_base_stations(
        MComCustom.default_config())] for _ in range(5)]
    xy, cnt = draw_layouts(random.Random(11), 5)
    assert [xy[k, :cnt[k]].tolist() for k in range(5)] == want


@pytest.mark.gpu
def test_batched_collect_matches_reference_driver(tmp_path):
    """collect_data (every notebook epoch as one env of a batch) writes the files of the
    reference's sequential collectData2 driver, for the same random seed."""
    from mobile_env.collect import collect_data
    g = golden()
    for run in g["runs"]:
        root = tmp_path / f"seed{run['random_seed']}"
        collect_data(g["epochs"], str(root), random_seed=run["random_seed"], steps=g["steps"],
                     device="cuda", batch=1 if run["random_seed"] else 64)
        assert_same_files(read_tree(str(root)), run["files"])


def _golden_qoe(files, epoch):
    """{ue_id: [qoe, ...]} of a golden user_qoe_{epoch}.csv (the notebook eval()s the cells;
    here the numbers are parsed)."""
    import re
    text = files[f"collectData2/UserQoE/user_qoe_{epoch}.csv"]
    out = {}
    for line in text.strip().split("\n")[1:]:
        uid, cell = line.split(",", 1)
        out[int(uid)] = [float(v) for v in re.findall(r"-?\d+\.\d+(?:e-?\d+)?", cell)]
    return out


def test_layout_scores_formula_matches_notebook():
    from mobile_env.scoring import layout_scores, qoe_value_reference
    g = golden()
    for run in g["runs"]:
        for ep in range(g["epochs"]):
            q = _golden_qoe(run["files"], ep)
            allq = np.hstack(list(q.values()))
            stats = np.array([[len(allq), allq.sum(), (allq * allq).sum(),
                               (allq < 0.0).sum()]], dtype=np.float64)
            got = layout_scores(stats)
            want = qoe_value_reference(q)
            for k in want:
                np.testing.assert_allclose(got[k][0], want[k], rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
def test_gpu_layout_scores_match_notebook_on_reference_files():
    """qoe_stats accumulated by the step kernel score the reference's epochs like
    chooseBaseStation.ipynb does from the reference's CSV files."""
    from mobile_env.scoring import qoe_value_reference, score_layouts
    g = golden()
    lays = [layout(r["files"], ep) for r in g["runs"] for ep in range(g["epochs"])]
    want = [qoe_value_reference(_golden_qoe(r["files"], ep))
            for r in g["runs"] for ep in range(g["epochs"])]
    xy = np.zeros((len(lays), 10, 2), dtype=np.int32)
    cnt = np.array([len(l) for l in lays], dtype=np.int32)
    for i, l in enumerate(lays):
        xy[i, :len(l)] = l
    got = score_layouts(xy, cnt, device="cuda")
    for i, w in enumerate(want):
        for k in w:
            np.testing.assert_allclose(got[k][i], w[k], rtol=1e-12, atol=1e-14, err_msg=k)
    assert got["best"] == int(np.argmax([w["Score"] for w in want]))
