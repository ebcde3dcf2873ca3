"""ctypes binding of libmev.so -- the C ABI declared in include/mev.h.

The library is built in-tree by ``make -C mobile-env-gan_amd/csrc`` (or
``__graft_entry__.build()``) into ``mobile-env-gan_amd/lib/libmev.so``. There is no CPU
fallback: if the library is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "MEV_LIB", os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libmev.so")))

ABI_VERSION = 23
MEV_OK = 0
MEV_EINVAL = -22
MEV_ENOMEM = -12
MEV_EHIP = -1000
MEV_ECHANNEL = -1001

# every symbol include/mev.h declares (tests check the library exports all of them)
EXPORTS = ("mev_abi_version", "mev_source_hash", "mev_create", "mev_destroy", "mev_d2max", "mev_launch_parts", "mev_step_shape", "mev_lds_tables_bytes", "mev_state_bytes_per_ue",
           "mev_rate_table", "mev_copy_rate_table", "mev_seed_pcg64", "mev_seed_pcg64_device",
           "mev_update_stations", "mev_update_layouts", "mev_build_rate_table", "mev_share_cents",
           "mev_rollout_instance", "mev_share_tie_free", "mev_last_launch_kind",
           "mev_reset", "mev_prepare_draws", "mev_sync_stream_state", "mev_restore_stream_state", "mev_step", "mev_rollout", "mev_rollout_timed", "mev_strerror", "mev_last_hip_error")


class MevParams(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("num_ues", C.c_int32), ("num_bs", C.c_int32),
        ("width", C.c_int32), ("height", C.c_int32), ("ep_max_time", C.c_int32),
        ("arrival_start", C.c_int32), ("arrival_exit", C.c_int32),
        ("bs_per_env", C.c_int32), ("first_step_active", C.c_int32),
        ("movement_reseed", C.c_int32), ("draw_table", C.c_int32), ("fuse_steps", C.c_int32),
        ("stream_split", C.c_int32),
        ("velocity", C.c_double),
        ("bs_bw", C.c_double), ("bs_freq", C.c_double), ("bs_tx", C.c_double),
        ("bs_height", C.c_double),
        ("ue_snr_tr", C.c_double), ("ue_noise", C.c_double), ("ue_height", C.c_double),
        ("util_lower", C.c_double), ("util_upper", C.c_double),
        ("util_w1", C.c_double), ("util_w2", C.c_double), ("util_w3", C.c_double),
        ("qoe_low", C.c_double),
        ("rate_table", C.c_void_p), ("rate_table_len", C.c_int64),
        ("num_bs_classes", C.c_int32), ("num_ue_classes", C.c_int32),
        ("bs_class", C.c_void_p), ("ue_class", C.c_void_p),
        ("bs_class_params", C.c_void_p), ("ue_class_params", C.c_void_p),
        ("rate_table_offsets", C.c_void_p),
        ("lds_tables", C.c_int32), ("two_groups", C.c_int32), ("stage_rows", C.c_int32),
        ("xcd_remap", C.c_int32), ("scenario_constants", C.c_int32),
        ("station_culling", C.c_int32),
        ("ues_per_lane", C.c_int32),
        ("ue_velocity", C.c_void_p),
        ("compact_state", C.c_int32),
        ("reward_exact", C.c_int32),
    ]


class MevState(C.Structure):
    _fields_ = [("ue_state", C.c_void_p), ("pcg", C.c_void_p), ("t", C.c_void_p),
                ("bs_xy", C.c_void_p), ("bs_count", C.c_void_p)]


class MevOutputs(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("serving", C.c_void_p), ("reward", C.c_void_p),
                ("done", C.c_void_p), ("rate64", C.c_void_p), ("util64", C.c_void_p),
                ("metrics", C.c_void_p), ("qoe_stats", C.c_void_p)]


class MevError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        msg = lib().mev_strerror(code).decode(errors="replace") if _LIB else str(code)
        super().__init__(f"{where} failed ({code}): {msg}")


_LIB = None
_LOCK = threading.Lock()
SOURCES = (os.path.normpath(os.path.join(_HERE, "..", "..", "csrc", "mev_step.hip")),
           os.path.normpath(os.path.join(_HERE, "..", "..", "..", "include", "mev.h")))


def source_hash():
    """First 16 hex digits of SHA-256(mev_step.hip + mev.h) -- the Makefile's MEV_SRC_HASH --
    or None when the sources are not beside the library (an installed copy)."""
    import hashlib
    h = hashlib.sha256()
    for path in SOURCES:
        try:
            with open(path, "rb") as f:
                h.update(f.read())
        except OSError:
            return None
    return h.hexdigest()[:16]


def lib():
    """Load libmev.so once; raise loudly if it is absent (no CPU fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libmev.so not found at {LIB_PATH}: build it with `make -C mobile-env-gan_amd/csrc`"
                " or __graft_entry__.build() -- the engine has no CPU fallback")
        L = C.CDLL(LIB_PATH)
        L.mev_abi_version.restype = C.c_int
        L.mev_create.argtypes = [C.POINTER(MevParams), C.POINTER(C.c_void_p)]
        L.mev_create.restype = C.c_int
        L.mev_destroy.argtypes = [C.c_void_p]
        L.mev_destroy.restype = None
        L.mev_d2max.argtypes = [C.c_void_p]
        L.mev_d2max.restype = C.c_int
        L.mev_launch_parts.argtypes = [C.c_void_p]
        L.mev_launch_parts.restype = C.c_int
        L.mev_step_shape.argtypes = [C.c_void_p]
        L.mev_step_shape.restype = C.c_int
        L.mev_lds_tables_bytes.argtypes = [C.c_void_p]
        L.mev_lds_tables_bytes.restype = C.c_int
        L.mev_state_bytes_per_ue.argtypes = [C.c_void_p]
        L.mev_state_bytes_per_ue.restype = C.c_int
        L.mev_rate_table.argtypes = [C.c_void_p]
        L.mev_rate_table.restype = C.c_void_p
        L.mev_copy_rate_table.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.mev_copy_rate_table.restype = C.c_int
        L.mev_seed_pcg64.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
        L.mev_seed_pcg64.restype = C.c_int
        L.mev_seed_pcg64_device.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        L.mev_seed_pcg64_device.restype = C.c_int
        L.mev_prepare_draws.argtypes = [C.c_void_p, C.POINTER(MevState), C.c_void_p, C.c_void_p]
        L.mev_prepare_draws.restype = C.c_int
        L.mev_sync_stream_state.argtypes = [C.c_void_p, C.POINTER(MevState), C.c_void_p]
        L.mev_sync_stream_state.restype = C.c_int
        L.mev_restore_stream_state.argtypes = [C.c_void_p, C.POINTER(MevState), C.c_void_p,
                                               C.c_void_p]
        L.mev_restore_stream_state.restype = C.c_int
        L.mev_update_stations.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.mev_update_stations.restype = C.c_int
        L.mev_update_layouts.argtypes = [C.c_void_p, C.POINTER(MevState), C.c_void_p, C.c_void_p]
        L.mev_update_layouts.restype = C.c_int
        L.mev_reset.argtypes = [C.c_void_p, C.POINTER(MevState), C.POINTER(MevOutputs),
                                C.c_void_p, C.c_void_p]
        L.mev_reset.restype = C.c_int
        L.mev_step.argtypes = [C.c_void_p, C.POINTER(MevState), C.POINTER(MevOutputs),
                               C.c_int32, C.c_void_p]
        L.mev_step.restype = C.c_int
        L.mev_rollout.argtypes = [C.c_void_p, C.POINTER(MevState), C.POINTER(MevOutputs),
                                  C.c_int32, C.c_void_p]
        L.mev_rollout.restype = C.c_int
        L.mev_rollout_timed.argtypes = [C.c_void_p, C.POINTER(MevState), C.POINTER(MevOutputs),
                                        C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mev_rollout_timed.restype = C.c_int
        L.mev_build_rate_table.argtypes = [C.POINTER(MevParams), C.c_void_p, C.c_int64]
        L.mev_build_rate_table.restype = C.c_int64
        L.mev_share_cents.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.mev_share_cents.restype = C.c_int
        L.mev_rollout_instance.argtypes = [C.c_void_p]
        L.mev_rollout_instance.restype = C.c_int
        L.mev_share_tie_free.argtypes = [C.c_void_p]
        L.mev_share_tie_free.restype = C.c_int
        L.mev_last_launch_kind.argtypes = [C.c_void_p]
        L.mev_last_launch_kind.restype = C.c_int
        L.mev_strerror.argtypes = [C.c_int]
        L.mev_strerror.restype = C.c_char_p
        L.mev_last_hip_error.restype = C.c_char_p
        # (MEV_LIB, dev A/B of library variants: a variant of the previous ABI is accepted -- the
        # ABI changes between neighbouring versions are additive)
        abi = L.mev_abi_version()
        if abi != ABI_VERSION and not (os.environ.get("MEV_LIB") and abi == ABI_VERSION - 1):
            raise ImportError(f"libmev ABI {abi} != expected {ABI_VERSION}")
        L.mev_source_hash.restype = C.c_char_p
        built, src = L.mev_source_hash().decode(), source_hash()
        if src is not None and built != src and not os.environ.get("MEV_LIB"):
            raise ImportError(
                f"stale libmev.so at {LIB_PATH}: compiled from sources {built}, the sources next "
                f"to it hash to {src} -- rebuild with `make -C mobile-env-gan_amd/csrc` or "
                "__graft_entry__.build()")
        _LIB = L
        return L


def check(code: int, where: str):
    if code != MEV_OK:
        raise MevError(code, where)


def seed_pcg64(seeds) -> "list[int]":
    """numpy-compatible PCG64 seeding (host C): rows of 6 uint64 per seed."""
    import numpy as np  # host-side buffer only

    s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(-1))
    rows = np.zeros((len(s), 6), dtype=np.uint64)
    check(lib().mev_seed_pcg64(s.ctypes.data, len(s), rows.ctypes.data), "mev_seed_pcg64")
    return rows
