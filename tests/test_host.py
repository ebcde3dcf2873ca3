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
    # build provenance: the library was compiled from the sources beside it
    assert lib.mev_source_hash().decode() == N.source_hash() != "unknown"


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
                dict(width=4097), dict(height=5000), dict(stream_split=3)):
        kw = dict(num_envs=4, num_ues=5, num_bs=3)
        kw.update(bad)
        cp = EngineParams(**kw).to_c(False)
        ctx = C.c_void_p()
        assert lib.mev_create(C.byref(cp), C.byref(ctx)) == N.MEV_EINVAL
    # a caller's channel table longer than any squared distance on a 1024 x 1024 map
    cp = EngineParams(num_envs=4, num_ues=5, num_bs=3).to_c(False)
    cp.rate_table_len = 2 * 1023 * 1023 + 2
    cp.rate_table = C.c_void_p(8)  # not read: rejected first
    assert lib.mev_create(C.byref(cp), C.byref(C.c_void_p())) == N.MEV_EINVAL


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

    class MyHata(OkumuraHata):  # overrides nothing the kernel implements: lowers
        label = "mine"
    lowering.check_plugins(plug["arrival"], MyHata(), plug["scheduler"], plug["movement"],
                           plug["utility"])

    class LossyHata(OkumuraHata):  # its own path loss: no kernel
        def power_loss(self, bs, ue):
            return 1.0
    with pytest.raises(NotImplementedError):
        lowering.check_plugins(plug["arrival"], LossyHata(), plug["scheduler"],
                               plug["movement"], plug["utility"])
    # entities with their own parameters lower to parameter classes (entities.py:7-22,33-45)
    us[2].velocity = 3.0
    st[1].tx_power = 30
    p = lowering.lower(num_envs=1, stations=st, users=us, ep_max_time=20,
                       first_step_active=True, **plug)
    assert p.heterogeneous and p.bs_class == [0, 1, 0] and p.ue_class == [0, 0, 0, 0]
    assert [c["tx"] for c in p.bs_classes] == [40, 30]
    # the velocity goes per UE (movement only): no UE class for it
    assert p.ue_velocity == [1.5, 1.5, 3.0, 1.5] and len(p.ue_classes) == 1
    us[1].snr_threshold = 5e-8
    p = lowering.lower(num_envs=1, stations=st, users=us, ep_max_time=20,
                       first_step_active=True, **plug)
    assert p.ue_class == [0, 1, 0, 0] and [c["snr_tr"] for c in p.ue_classes] == [2e-8, 5e-8]
    tab, offs = p.rate_table()
    assert len(offs) == 2 * 2 + 1 and offs[-1] == len(tab)
    # any number of distinct velocities (the 16-class limit is on the channel tuples only)
    us2 = [UserEquipment(i, 1.0 + 0.5 * i, 2e-8, 1e-9, 1.6) for i in range(40)]
    p = lowering.lower(num_envs=1, stations=st, users=us2, ep_max_time=20,
                       first_step_active=True, **plug)
    assert p.ue_velocity == [1.0 + 0.5 * i for i in range(40)]


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
    # maps beyond 1024 (mev.h kMaxMap): stations anywhere in [0, 4096)
    from mobile_env.core.engine import station_limit
    assert station_limit(200, 1024) == 1024 and station_limit(1025, 30) == 4096
    _check_station_range(torch.tensor([[0, 0], [4095, 5]]), limit=station_limit(3000, 2000))
    with pytest.raises(ValueError):
        _check_station_range(torch.tensor([[4096, 0]]), limit=4096)


def test_wide_map_rate_tables():
    """Maps beyond 1024 x 1024: the Python (numpy) and C (libm) tables scan the squared
    distances up to D2_TOP and agree on the connectable range; a channel that still connects
    at D2_TOP is refused by both (the association keys hold the squared distance in 22 bits)."""
    import ctypes as C
    from mobile_env.core import _native as N
    from mobile_env.core.channels import D2_TOP, OkumuraHata
    from mobile_env.core.engine import EngineParams
    lib = N.lib()
    bs = {"bw": 9e6, "freq": 2500, "tx": 55, "height": 50}
    ue = {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6}
    tab = OkumuraHata().rate_table(bs, ue, 3000, 2000)
    cp = EngineParams(num_envs=1, num_ues=5, num_bs=3, width=3000, height=2000, bs=bs,
                      ue=ue).to_c(False)
    n = lib.mev_build_rate_table(C.byref(cp), None, 0)
    assert n == len(tab) and 19363 < n < D2_TOP
    ctab = np.zeros(n)
    assert lib.mev_build_rate_table(C.byref(cp), ctab.ctypes.data, n) == n
    np.testing.assert_allclose(ctab, tab, rtol=1e-13, atol=0)  # (libm vs numpy's log10 / pow)
    strong = dict(bs, tx=90)
    with pytest.raises(ValueError):
        OkumuraHata().rate_table(strong, ue, 3000, 2000)
    cp = EngineParams(num_envs=1, num_ues=5, num_bs=3, width=3000, height=2000, bs=strong,
                      ue=ue).to_c(False)
    assert lib.mev_build_rate_table(C.byref(cp), None, 0) == N.MEV_EINVAL


def test_bench_byte_models():
    """bench.py's byte models: SURVEY 8d's canonical 54 U + 61 B per env-step (1,681 B for
    mobile-large), and the rollout launch's algorithmic bytes (every step's outputs + the state
    read and written once) -- never above the canonical figure times the steps."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.algorithmic_bytes_per_env_step(30, False, 13) == 1681
    assert bench.algorithmic_bytes_per_env_step(1024, True, 128) == 56381
    for U in (5, 15, 30):
        for n in (1, 2, 20):
            r = bench.algorithmic_bytes_rollout(U, False, 3, n)
            assert r == n * (20 * U + 5) + 34 * U + 56
            assert r <= n * bench.algorithmic_bytes_per_env_step(U, False, 3)


def test_bench_dtype_names_the_state_form():
    """The bench line's dtype names the UE state form the kernels run (the compact uint8 x4
    rows on the registered 200 x 200 maps, int16 x4 beyond 255 per side) and the fixed-point
    reward sum."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    d4, d8 = bench.dtype_string(4), bench.dtype_string(8)
    assert "uint8x4" in d4 and "int16" not in d4
    assert "int16x4" in d8 and "uint8" not in d8
    for d in (d4, d8):
        assert "fixed-point reward" in d and "f64 rate" in d


def test_bench_cpu_baseline_follows_workload():
    """bench.py's cpu_baseline runs the CPU port on the --workload's sizes (shared and per-env
    layouts), one short sample per workload."""
    import importlib.util
    import os
    import sys
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    sys.modules["bench"] = bench  # (the worker function is pickled by module name)
    spec.loader.exec_module(bench)
    for wl, sizes in (("mobile-small-central-v0", "3 BS x 5 UE"),
                      ("mobile-large-perenv-v0", "13 BS x 30 UE")):
        r = bench.cpu_baseline(0.3, 1, wl)
        assert r["value"] > 0 and r["cores"] == 1 and r["kind"] == "port"
        assert wl in r["sample"] and sizes in r["sample"]


def test_sums_of_two_squares_rank_index():
    """The LDS tables index the float64 rates by the rank of d2 in S = {a^2 + b^2 <= d2max}
    (mev_step.hip build_lds_tables / k_lds_map): every squared integer distance is in S, and
    the {bits, prefix} words give consecutive ranks (restated here on the host)."""
    import numpy as np
    d2max = 19362
    s = set()
    a = 0
    while a * a <= d2max:
        b = a
        while a * a + b * b <= d2max:
            s.add(a * a + b * b)
            b += 1
        a += 1
    assert len(s) == 5101
    nw = d2max // 32 + 1
    bits = np.zeros(nw, np.uint64)
    for d in s:
        bits[d >> 5] |= np.uint64(1) << np.uint64(d & 31)
    prefix = np.concatenate([[0], np.cumsum([bin(int(w)).count("1") for w in bits])[:-1]])
    rank = lambda d: int(prefix[d >> 5]) + bin(int(bits[d >> 5]) & ((1 << (d & 31)) - 1)).count("1")
    assert [rank(d) for d in sorted(s)] == list(range(len(s)))
    rng = np.random.default_rng(0)
    for _ in range(1000):  # positions and stations anywhere on a 200 x 200 map
        dx, dy = rng.integers(-199, 200, 2)
        d2 = int(dx * dx + dy * dy)
        if d2 <= d2max:
            assert d2 in s


def test_store_hazard_check_on_generated_assembly():
    """Deterministic guard for the gfx950 wide-buffer-store hazard (mev_step.hip
    flush_pending): no buffer_store_dwordx3/x4 in the generated device assembly takes an SGPR
    soffset (LLVM places no wait state for those), checked on `make asm` output; the checker
    itself flags a register soffset."""
    import shutil
    import sys
    if shutil.which("/opt/rocm/bin/hipcc") is None:
        pytest.skip("hipcc not available")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_store_hazard as ch
    bad_line = "\tbuffer_store_dwordx4 v[0:3], v8, s[96:99], s4 offen"
    assert ch.violations("_Zk:\n" + bad_line) and not ch.violations(
        "_Zk:\n\tbuffer_store_dwordx4 v[0:3], v8, s[96:99], 0 offen")
    text = open(ch.build_asm()).read()
    assert ch.wide_store_count(text) > 0
    assert ch.violations(text) == []


def test_prefetch_registers_check_on_generated_assembly():
    """The two-group rollout kernel's one-pair-ahead input loads are inline assembly the
    compiler does not track (mev_step.hip, pf_b32 / pf_b64); the kernel waits for them itself.
    tools/check_prefetch_regs.py verifies on `make asm` output that every prefetched value stays
    in the register its load wrote, untouched, until the explicit wait -- no copy, no spill,
    no reuse -- in every kernel instance that has them; and the checker flags a copy."""
    import shutil
    import sys
    if shutil.which("/opt/rocm/bin/hipcc") is None:
        pytest.skip("hipcc not available")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_prefetch_regs as cp
    bad = ("_Zk:\n\tglobal_load_dword v5, v[2:3], off ; mev-prefetch\n"
           "\tv_mov_b32_e32 v9, v5\n\t; mev-prefetch-wait v9\n")
    assert cp.violations(bad)[0]
    good = ("_Zk:\n\tglobal_load_dword v5, v[2:3], off ; mev-prefetch\n"
            "\tv_add_u32_e32 v7, v8, v6\n\ts_waitcnt vmcnt(63)\n\t; mev-prefetch-wait v5\n"
            "\tds_write_b32 v1, v5\n")
    assert cp.violations(good) == ([], 1)
    # a 64-bit multiply-add that reads an in-flight register only as its addend's don't-care high
    # half (the result's high half dead: redefined, after an unconditional branch, before any
    # read on any path) is benign; with the high half read afterwards on some path, not
    head = ("_Zk:\n\tglobal_load_dword v43, v[2:3], off ; mev-prefetch\n"
            "\tv_mad_u64_u32 v[0:1], s[8:9], s35, v7, v[42:43]\n")
    tail = "\ts_waitcnt vmcnt(63)\n\t; mev-prefetch-wait v43\n"
    dead = head + "\ts_branch .LBB0_2\n.LBB0_2:\n\tds_read_u8 v1, v0\n" + tail
    assert cp.violations(dead) == ([], 1)
    used = head + "\tv_add_u32_e32 v4, v1, v0\n" + tail
    assert cp.violations(used)[0]
    cond = (head + "\ts_cbranch_scc1 .LBB0_2\n\tds_read_u8 v1, v0\n.LBB0_2:\n"
            "\tv_add_u32_e32 v4, v1, v0\n" + tail)  # (the taken branch reads the dead half)
    assert cp.violations(cond)[0]
    both = head + "\ts_cbranch_scc1 .LBB0_2\n\tds_read_u8 v1, v0\n.LBB0_2:\n" + tail
    assert cp.violations(both) == ([], 1)  # (no path reads it)
    # a call (the reward guard's out-of-line rare path) while a prefetch is in flight: flagged
    # unless an s_waitcnt vmcnt(0) precedes it in its block (the callee's register save /
    # restore would lose the landing data)
    call = ("_Zk:\n\tglobal_load_dword v5, v[2:3], off ; mev-prefetch\n; %bb.1:\n"
            "\ts_swappc_b64 s[30:31], s[0:1]\n\ts_waitcnt vmcnt(63)\n\t; mev-prefetch-wait v5\n")
    assert cp.violations(call)[0]
    waited = call.replace("; %bb.1:\n", "; %bb.1:\n\ts_waitcnt vmcnt(0)\n")
    assert cp.violations(waited) == ([], 1)
    # wait, THEN a new prefetch load, then the call in the same block: the earlier wait does not
    # cover the later load -- flagged
    late = ("_Zk:\n; %bb.1:\n\ts_waitcnt vmcnt(0)\n"
            "\tglobal_load_dword v5, v[2:3], off ; mev-prefetch\n"
            "\ts_swappc_b64 s[30:31], s[0:1]\n\ts_waitcnt vmcnt(63)\n\t; mev-prefetch-wait v5\n")
    assert cp.violations(late)[0]
    text = open(cp.build_asm()).read()
    v, n = cp.violations(text)
    assert n >= 8 and v == []


def test_host_code_under_asan(tmp_path, golden_dir):
    """The library's host code (argument checks, numpy-compatible seeding, the libm channel
    table, mev_create's validation and failure path) under AddressSanitizer + UBSan with leak
    detection: `make asan` builds libmev_asan.so (sanitizers on the host side only), and
    tests/asan/host_driver.c calls every entry point that needs no GPU with exactly sized
    buffers. Its printed seed rows must equal numpy's PCG64 seeding and its table the
    reference's channel table (channel_default.npz)."""
    import shutil
    import subprocess
    clang = "/opt/rocm/llvm/bin/clang"
    if not os.path.exists(clang) or shutil.which("make") is None:
        pytest.skip("ROCm clang / make not available")
    csrc = os.path.join(ROOT, "mobile-env-gan_amd", "csrc")
    subprocess.run(["make", "-s", "-C", csrc, "asan"], check=True, timeout=900)
    lib = os.path.join(ROOT, "mobile-env-gan_amd", "lib", "libmev_asan.so")
    drv = str(tmp_path / "host_driver")
    subprocess.run([clang, "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-g",
                    "-I", os.path.join(ROOT, "include"), "-o", drv,
                    os.path.join(ROOT, "tests", "asan", "host_driver.c"), lib,
                    "-Wl,-rpath," + os.path.dirname(lib)], check=True, timeout=120)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([drv], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    lines = r.stdout.split("\n")
    assert "ok" in lines
    for ln in (x for x in lines if x.startswith("seed ")):
        seed, slo, shi, ilo, ihi = (int(v) for v in ln.split()[1:])
        st = np.random.PCG64(seed).state["state"]
        assert (shi << 64 | slo) == st["state"] and (ihi << 64 | ilo) == st["inc"], seed
    n, t1, tmid, tlast = next(x for x in lines if x.startswith("table ")).split()[1:]
    c = np.load(f"{golden_dir}/channel_default.npz")
    rate = c["rate"]
    assert int(n) == int(c["d2max"]) + 1 == len(rate)
    # (the C library's log10 may differ from numpy's by an ulp: the Python host passes numpy's)
    np.testing.assert_allclose([float(t1), float(tmid), float(tlast)],
                               [rate[1], rate[int(n) // 2], rate[-1]], rtol=1e-14)


@pytest.mark.parametrize("v", [1.0, 3.0, 10.0, 25.0, 100.0])
def test_integer_velocity_axis_moves_take_the_fast_path(v):
    """An integer velocity has no axis-parallel branch (host_move_params sets axis_exact 0,
    mev_step.hip move_ue_p): an axis move is pos +- v in the reference (movement.py:58-62, the
    float64 p + v * a / |a| is exact and integral), and the float32 fast path -- q = a * (v_f *
    rsq(a^2)) with rsq within 2^-21 relative, accepted when |q - rint(q)| < 0.5 - 2^-16 max(1, v)
    -- must accept every such move and give exactly +-v. Checked for every axis distance on a
    1024 map beyond the arrival radius, at both ends of the rsq error bound."""
    a = np.arange(1, 1024, dtype=np.float64)
    a = a[a > v]  # |a| <= v: arrival (the snap), not a step
    ref = np.rint(0.0 + (v * a) / np.sqrt(a * a))  # the reference's float64 step from p = 0
    assert np.all(ref == v)
    lim = np.float32(0.5 - 2.0 ** -16 * max(1.0, v))
    for rel in (-(2.0 ** -21), 0.0, 2.0 ** -21):
        rsq = ((1.0 / a) * (1.0 + rel)).astype(np.float32)
        sc = np.float32(v) * rsq
        for sgn in (1.0, -1.0):
            q = (sgn * a).astype(np.float32) * sc
            r = np.rint(q)
            assert np.all(np.abs(q - r) < lim)
            assert np.all(r == sgn * v)
