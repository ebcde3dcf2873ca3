"""CPU tests of the host side: the C-ABI library loads and exports every declared symbol,
numpy-compatible seeding, config lowering, the scenario registry, and the layouts the
reference-facing API builds. No GPU compute is called here."""
import os
import random
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mev.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mev_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from mobile_env.core import _native as N
    lib = N.lib()
    syms = declared_symbols()
    assert syms, "no declarations parsed"
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(N.EXPORTS) == syms
    assert lib.mev_abi_version() == N.ABI_VERSION


def test_struct_layout_matches_header():
    """ctypes mirrors of mev_params / mev_state / mev_outputs list the header's fields in
    order."""
    from mobile_env.core import _native as N
    text = open(HEADER).read()
    for cname, pyt in (("mev_params", N.MevParams), ("mev_state", N.MevState),
                       ("mev_outputs", N.MevOutputs)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), text, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            # "int32_t a, b" or "double x" or "const int32_t* p"
            typ_and_first, *rest = [d.strip() for d in decl.split(",")]
            names.append(re.split(r"[\s\*]+", typ_and_first)[-1])
            names += [re.sub(r"[\s\*]", "", r) for r in rest]
        assert names == [f[0] for f in pyt._fields_], (cname, names)


@pytest.mark.parametrize("seed", [0, 1, 4, 2028, 1004, 123456789, 2**32 - 1, 2**32 + 7,
                                  2**62 + 5])
def test_seeding_matches_numpy_pcg64(seed):
    from mobile_env.core import _native as N
    row = N.seed_pcg64([seed])[0]
    st = np.random.PCG64(seed).state["state"]
    assert int(row[0]) | (int(row[1]) << 64) == st["state"]
    assert int(row[2]) | (int(row[3]) << 64) == st["inc"]
    assert (row[4], row[5]) == (row[0], row[1])  # state0 = seeded state


def test_seeding_rejects_negative():
    from mobile_env.core import _native as N
    with pytest.raises(N.MevError):
        N.seed_pcg64(np.array([2**63], dtype=np.uint64))


def test_error_strings():
    from mobile_env.core import _native as N
    lib = N.lib()
    assert lib.mev_strerror(N.MEV_EINVAL) == b"invalid parameters"
    assert b"prefix" in lib.mev_strerror(N.MEV_ECHANNEL)


def test_create_rejects_bad_params_without_gpu():
    """Parameter validation happens before any device work."""
    import ctypes as C
    from mobile_env.core import _native as N
    from mobile_env.core.engine import EngineParams
    lib = N.lib()
    for bad in (dict(num_envs=0), dict(num_ues=0), dict(num_ues=1025), dict(num_bs=0),
                dict(width=2000), dict(stream_split=3)):
        kw = dict(num_envs=4, num_ues=5, num_bs=3)
        kw.update(bad)
        cp = EngineParams(**kw).to_c(False)
        ctx = C.c_void_p()
        assert lib.mev_create(C.byref(cp), C.byref(ctx)) == N.MEV_EINVAL


def test_registry():
    import mobile_env
    from mobile_env.scenarios.registry import spec
    ids = mobile_env.registered_ids()
    for size, (u, b) in {"small": (5, 3), "medium": (15, 7), "large": (30, 13)}.items():
        for mode in ("central", "ma"):
            sp = spec(f"mobile-{size}-{mode}-v0")
            assert (sp["num_ues"], sp["num_bs"], sp["mode"]) == (u, b, mode)
    assert "mobile-custom-128x1024-v0" in ids
    with pytest.raises(KeyError):
        spec("mobile-huge-central-v0")


def test_config_defaults_and_seeding_match_reference_schema():
    """default_config / seeding follow base.py:103-170 (movement seed = seed + 4)."""
    from mobile_env.core.base import MComCore
    from mobile_env.core.util import deep_dict_merge
    cfg = deep_dict_merge(MComCore.default_config(), {"seed": 10, "ue": {"velocity": 3}})
    cfg = MComCore.seeding(cfg)
    assert cfg["movement_params"]["seed"] == 14
    assert cfg["arrival_params"]["seed"] == 11
    assert cfg["utility_params"]["seed"] == 15
    assert cfg["ue"] == {"velocity": 3, "snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}
    assert cfg["bs"] == {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50}


def test_lowering_builtin_plugins_and_rejects_others():
    from mobile_env.core import lowering
    from mobile_env.core.arrival import NoDeparture
    from mobile_env.core.channels import OkumuraHata
    from mobile_env.core.entities import BaseStation, UserEquipment
    from mobile_env.core.movement import RandomWaypointMovement
    from mobile_env.core.schedules import RateFair, ResourceFair
    from mobile_env.core.utilities import BoundedLogUtility
    st = [BaseStation(i, (10 * i, 5), 9e6, 2500, 40, 50) for i in range(3)]
    us = [UserEquipment(i, 1.5, 2e-8, 1e-9, 1.6) for i in range(4)]
    plug = dict(arrival=NoDeparture(ep_time=20, seed=1, reset_rng_episode=False),
                channel=OkumuraHata(), scheduler=ResourceFair(),
                movement=RandomWaypointMovement(width=200, height=200, seed=5,
                                                reset_rng_episode=True),
                utility=BoundedLogUtility(lower=-20, upper=20, coeffs=(10, 0, 10)))
    p = lowering.lower(num_envs=1, stations=st, users=us, ep_max_time=20,
                       first_step_active=True, **plug)
    assert (p.num_ues, p.num_bs, p.velocity, p.arrival_exit, p.t_end) == (4, 3, 1.5, 20, 20)
    assert p.util_coeffs == (10.0, 0.0, 10.0)
    with pytest.raises(NotImplementedError):
        lowering.lower(num_envs=1, stations=st, users=us, ep_max_time=20,
                       first_step_active=True, **{**plug, "scheduler": RateFair()})

    class MyHata(OkumuraHata):
        pass
    with pytest.raises(NotImplementedError):
        lowering.check_plugins(plug["arrival"], MyHata(), plug["scheduler"], plug["movement"],
                               plug["utility"])
    us[2].velocity = 3.0
    with pytest.raises(NotImplementedError):
        lowering.lower(num_envs=1, stations=st, users=us, ep_max_time=20,
                       first_step_active=True, **plug)


def test_mcom_custom_layout_uses_global_random_like_reference():
    """MComCustom draws randint(5,10) stations at int(uniform(0,200)) from the global
    `random` (custom.py:68-77): the fixture layouts come out for random.seed(k)."""
    from helpers import load
    from mobile_env.scenarios.custom import MComCustom
    d = load("mcom_custom")
    for k in range(8):
        random.seed(int(d["random_seeds"][k]))
        for ep in range(2):
            lay = MComCustom.generate_base_stations(MComCustom.default_config())
            want = d["bs_xy"][k, ep, :d["bs_count"][k, ep]].tolist()
            assert [[bs.x, bs.y] for bs in lay] == want


def test_engine_refuses_cpu_device():
    from mobile_env.core.engine import EngineParams, StepEngine
    with pytest.raises(RuntimeError):
        StepEngine(EngineParams(num_envs=1, num_ues=5, num_bs=3), [[0, 0]] * 3, [1],
                   device="cpu")


def test_station_range_check():
    import torch
    from mobile_env.core.engine import _check_station_range
    _check_station_range(torch.tensor([[0, 0], [1023, 5]]))
    with pytest.raises(ValueError):
        _check_station_range(torch.tensor([[0, 0], [1024, 5]]))
    with pytest.raises(ValueError):
        _check_station_range(torch.tensor([[-1, 0]]))
    # per-env layouts: rows beyond bs_count are padding and are not checked
    lay = torch.tensor([[[5, 5], [-1, -1]], [[7, 7], [8, 8]]])
    _check_station_range(lay, [1, 2])
    with pytest.raises(ValueError):
        _check_station_range(lay, [2, 2])
