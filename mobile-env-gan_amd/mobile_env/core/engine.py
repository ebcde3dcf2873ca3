"""StepEngine: batched env state as SoA device tensors + the libmev.so kernels.

This is the host side of the hot path. It owns (as torch tensors on one GPU) the state of
E independent mobile-env instances and drives the fused HIP step kernel through the C ABI
(include/mev.h). It replaces, for a whole batch at once, the per-object state the
reference keeps in entity/plugin objects:

=====================  ===================================  ============================
tensor                 reference state                      reference file:line
=====================  ===================================  ============================
``ue_state [E,U,4]``   ``UserEquipment.x/.y`` (cols 0-1)    entities.py:47-48, base.py:233
  ``i16``              ``RandomWaypointMovement``           movement.py:33,44-47,55
                       ``.userMoveDirection`` (cols 2-3,
                       wx<0: none)
``pcg [E,6] u64``      ``Movement.rng`` (numpy PCG64)       movement.py:16-18
``t [E] i32``          ``MComCore.time``                    base.py:175,280
``bs_xy [B,2]/[E,B,2]`` ``BaseStation.x/.y`` (int-truncated) entities.py:18,24-26
=====================  ===================================  ============================

Outputs per step: ``obs [E,U,4] f32`` = (x/W, y/H, data rate, scaled utility),
``serving [E,U] i32``, ``reward [E] f32`` (mean utility, metrics.py:25-28), ``done [E] u8``,
and optionally ``rate64``/``util64 [E,U] f64``, ``metrics [E,4] f32`` and ``qoe_stats [E,4] f64``
(per-episode {count, sum, sum of squares, count below qoe_low} of the rounded QoE values, the
input of the layout score, mobile_env.scoring).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import torch

from . import _native as N


@dataclass
class EngineParams:
    """Flattened scenario + plugin parameters (lowered from the MComCore config dict)."""
    num_envs: int
    num_ues: int
    num_bs: int
    width: int = 200
    height: int = 200
    ep_max_time: int = 20
    arrival_start: int = 0
    arrival_exit: int = 20
    first_step_active: bool = True
    movement_reseed: bool = True
    velocity: float = 1.5
    bs: dict = field(default_factory=lambda: {"bw": 9e6, "freq": 2500, "tx": 40, "height": 50})
    ue: dict = field(default_factory=lambda: {"snr_tr": 2e-8, "noise": 1e-9, "height": 1.6})
    util_lower: float = -20.0
    util_upper: float = 20.0
    util_coeffs: tuple = (10.0, 0.0, 10.0)
    stream_split: int = 0  # mev_params.stream_split: 0 auto, 1 single stream, 2 two halves
    draw_table: int = -1   # mev_params.draw_table: episode draw table pairs per env (-1 auto)
    fuse_steps: int = 0    # mev_params.fuse_steps: 0 step(n > 1) in one launch, -1 n launches
    qoe_low: float = 0.0   # low-QoE threshold of the per-episode QoE statistics
    # launch-shape overrides (mev_params; 0 = automatic, results identical for every setting):
    lds_tables: int = 0          # -1 L2 association map, 1..3 that LDS table mode
    two_groups: int = 0          # -1 packed one-group rollouts; 1 / 2 two-group kernel (2 / 1 groups
                                 # per wave); 3 / 4 pipelined one-group kernel, U = 15 in 16- / 32-
                                 # lane segments (mev.h)
    stage_rows: int = 0          # > 0: at most that many staged per-env rows per window
    xcd_remap: int = 0           # -1 blocks in dispatch order
    scenario_constants: int = 0  # -1 generic kernel instances only
    station_culling: int = 0     # -1 U > 64: scan every station (no per-cell candidate lists)
    ues_per_lane: int = 0        # U > 64: 1 / 2 UEs per lane (0: two in one-step launches, U > 512)
    # heterogeneous entities (entities.py:7-22,33-45): parameter classes and each station's /
    # UE's class (None: every entity has bs / ue / velocity above); see lowering.lower
    bs_classes: "list | None" = None   # [{bw, freq, tx, height}]
    ue_classes: "list | None" = None   # [{velocity, snr_tr, noise, height}]
    bs_class: "list | None" = None     # [B] class index per station
    ue_class: "list | None" = None     # [U] class index per UE
    # per-UE velocity (mev_params.ue_velocity; None: `velocity` / the UE's class's): velocity
    # drives only the movement, so any number of distinct values needs no class
    ue_velocity: "list | None" = None  # [U]
    # UE state form (mev_params.compact_state): 0 auto -- uint8 x4 per UE on maps <= 255 per
    # side (every registered scenario), else int16 x4; -1 always int16; 1 uint8 (maps <= 255)
    compact_state: int = 0
    # mev_params.reward_exact: 1 -- every float32 reward from the exact float64 utilities (the
    # lean kernels otherwise do that only where the float32 sum could miss 1e-5 relative)
    reward_exact: int = 0

    @property
    def state_u8(self) -> bool:
        if self.compact_state < 0:
            return False
        return self.compact_state > 0 or (int(self.width) <= 255 and int(self.height) <= 255)

    @property
    def heterogeneous(self) -> bool:
        """More than one channel class on a side (the per-pair tables; per-UE velocities alone
        need none: see ue_velocity)."""
        return len(self.bs_classes or ()) > 1 or len(self.ue_classes or ()) > 1

    def _classes(self):
        bsc = self.bs_classes or [dict(self.bs)]
        uec = self.ue_classes or [dict(self.ue, velocity=self.velocity)]
        return bsc, uec

    def rate_table(self):
        """The channel rate table(s) of these parameters (numpy, reference op order; see
        mobile_env.core.channels): float64 [d2max + 1]; heterogeneous entities: one table per
        (station class, UE class) pair concatenated, and the [NB * NU + 1] offsets."""
        import numpy as np
        from .channels import OkumuraHata
        W, H = int(self.width), int(self.height)
        if not self.heterogeneous:
            return OkumuraHata().rate_table(self.bs, self.ue, W, H)
        bsc, uec = self._classes()
        tabs = [OkumuraHata().rate_table(b, u, W, H) for b in bsc for u in uec]
        offs = np.concatenate([[0], np.cumsum([len(t) for t in tabs])]).astype(np.int64)
        return np.concatenate(tabs).astype(np.float64), offs

    def to_c(self, bs_per_env: bool, rate_table=None) -> N.MevParams:
        """mev_params; ``rate_table`` (rate_table()'s result) is passed as mev_params.rate_table.
        The host arrays the struct points to are kept on the returned struct (``_keep``) until
        it is dropped: keep it alive until mev_create returns."""
        import numpy as np
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(np.asarray(a, dtype=dt))
            keep.append(a)
            return C.c_void_p(a.ctypes.data)

        offs = None
        if isinstance(rate_table, tuple):
            rate_table, offs = rate_table
        tab = (arr(rate_table, np.float64), len(rate_table)) if rate_table is not None \
            else (C.c_void_p(None), 0)
        het = {}
        if self.heterogeneous:
            bsc, uec = self._classes()
            het = dict(
                num_bs_classes=len(bsc), num_ue_classes=len(uec),
                bs_class=arr(self.bs_class if self.bs_class is not None
                             else [0] * self.num_bs, np.int32),
                ue_class=arr(self.ue_class if self.ue_class is not None
                             else [0] * self.num_ues, np.int32),
                bs_class_params=arr([[b["bw"], b["freq"], b["tx"], b["height"]] for b in bsc],
                                    np.float64),
                ue_class_params=arr([[u["velocity"], u["snr_tr"], u["noise"], u["height"]]
                                     for u in uec], np.float64),
                rate_table_offsets=arr(offs, np.int64) if offs is not None else C.c_void_p(None))
        cp = N.MevParams(
            rate_table=tab[0], rate_table_len=tab[1], **het,
            num_envs=self.num_envs, num_ues=self.num_ues, num_bs=self.num_bs,
            width=int(self.width), height=int(self.height), ep_max_time=int(self.ep_max_time),
            arrival_start=int(self.arrival_start), arrival_exit=int(self.arrival_exit),
            bs_per_env=int(bs_per_env), first_step_active=int(bool(self.first_step_active)),
            movement_reseed=int(bool(self.movement_reseed)),
            draw_table=int(self.draw_table), fuse_steps=int(self.fuse_steps),
            stream_split=int(self.stream_split),
            velocity=float(self.velocity),
            bs_bw=float(self.bs["bw"]), bs_freq=float(self.bs["freq"]),
            bs_tx=float(self.bs["tx"]), bs_height=float(self.bs["height"]),
            ue_snr_tr=float(self.ue["snr_tr"]), ue_noise=float(self.ue["noise"]),
            ue_height=float(self.ue["height"]),
            util_lower=float(self.util_lower), util_upper=float(self.util_upper),
            util_w1=float(self.util_coeffs[0]), util_w2=float(self.util_coeffs[1]),
            util_w3=float(self.util_coeffs[2]), qoe_low=float(self.qoe_low),
            lds_tables=int(self.lds_tables), two_groups=int(self.two_groups),
            stage_rows=int(self.stage_rows), xcd_remap=int(self.xcd_remap),
            scenario_constants=int(self.scenario_constants),
            station_culling=int(self.station_culling), ues_per_lane=int(self.ues_per_lane),
            compact_state=int(self.state_u8), reward_exact=int(self.reward_exact),
            ue_velocity=(arr([float(v) for v in self.ue_velocity], np.float64)
                         if self.ue_velocity is not None else C.c_void_p(None)))
        cp._keep = keep
        return cp

    @property
    def t_end(self) -> int:
        return min(int(self.ep_max_time), int(self.arrival_exit))


@dataclass
class Trajectory:
    """Per-step outputs of a rollout, leading axis = step: obs [n,E,U,4] f32, serving [n,E,U]
    i32, reward [n,E] f32, done [n,E] u8, and optionally rate64/util64 [n,E,U] f64,
    metrics [n,E,4] f32."""
    obs: torch.Tensor
    serving: torch.Tensor
    reward: torch.Tensor
    done: torch.Tensor
    rate64: "torch.Tensor | None" = None
    util64: "torch.Tensor | None" = None
    metrics: "torch.Tensor | None" = None

    def rows(self, start: int, n: int) -> "Trajectory":
        """Rows [start, start + n) as a trajectory (views; for rollouts of n steps that fill a
        longer trajectory piece by piece)."""
        def v(t):
            return None if t is None else t[start:start + n]
        return Trajectory(v(self.obs), v(self.serving), v(self.reward), v(self.done),
                          v(self.rate64), v(self.util64), v(self.metrics))


def station_limit(width: int, height: int) -> int:
    """Station coordinates lie in [0, limit): 1024 on maps up to 1024 x 1024 (the association
    keys hold |p - q|^2 - |p|^2 in 32 bits), 4096 on larger maps (mev.h kMaxMap: the keys hold
    the clamped squared distance itself)."""
    return 1024 if width <= 1024 and height <= 1024 else 4096


def _check_station_range(bs, bs_count=None, limit: int = 1024):
    """Station coordinates must lie in [0, limit) (station_limit); per-env layouts with a
    station count: only the first bs_count[e] rows are stations."""
    if bs_count is not None and bs.dim() == 3:
        cnt = torch.as_tensor(bs_count, dtype=torch.int64, device=bs.device).reshape(-1, 1)
        keep = torch.arange(bs.shape[1], device=bs.device)[None, :] < cnt
        bs = bs[keep]
    if bs.numel() and (int(bs.min()) < 0 or int(bs.max()) > limit - 1):
        raise ValueError(f"base-station coordinates must lie in [0, {limit})")


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(None)


class StepEngine:
    """E envs on one GPU. ``seeds`` are config seeds (movement stream = seed + 4,
    base.py:156-168); ``bs_xy`` is [B,2] (shared layout) or [E,B,2] (+ ``bs_count`` [E])."""

    def __init__(self, params: EngineParams, bs_xy, seeds, bs_count=None, device=None,
                 rate64: bool = False, util64: bool = False, metrics: bool = False,
                 qoe_stats: bool = False):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("StepEngine runs on a ROCm GPU only (no CPU fallback)")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.p = params
        E, U = params.num_envs, params.num_ues
        bs = torch.as_tensor(bs_xy, dtype=torch.int32)
        self.bs_per_env = bs.dim() == 3
        if self.bs_per_env:
            if bs.shape[0] != E or bs.shape[2] != 2:
                raise ValueError(f"bs_xy must be [E,B,2], got {tuple(bs.shape)}")
        elif bs.dim() != 2 or bs.shape[1] != 2:
            raise ValueError(f"bs_xy must be [B,2] or [E,B,2], got {tuple(bs.shape)}")
        B = bs.shape[-2]
        if B != params.num_bs:
            raise ValueError(f"bs_xy has {B} stations, params say {params.num_bs}")
        _check_station_range(bs, bs_count, station_limit(params.width, params.height))
        L = N.lib()
        with torch.cuda.device(device):
            tab = params.rate_table()  # the reference's own values (numpy, host)
            cp = params.to_c(self.bs_per_env, tab)
            ctx = C.c_void_p()
            N.check(L.mev_create(C.byref(cp), C.byref(ctx)), "mev_create")
            del tab
            self._ctx = ctx
            self._lib = L
            kw = dict(device=device)
            self.bs_xy = bs.contiguous().to(**kw)
            self.bs_count = None
            if bs_count is not None:
                self.bs_count = torch.as_tensor(bs_count, dtype=torch.int32).reshape(E).to(**kw)
                if int(self.bs_count.max()) > B or int(self.bs_count.min()) < 0:
                    raise ValueError("bs_count out of range")
            # the kernels' UE state rows: uint8 x4 (compact form, 255 = -1) or int16 x4
            self._u8 = params.state_u8
            self._ue_raw = torch.full((E, U, 4), 255 if self._u8 else -1,
                                      dtype=torch.uint8 if self._u8 else torch.int16, **kw)
            self.t = torch.full((E,), params.t_end, dtype=torch.int32, **kw)
            self._pcg = torch.zeros((E, 6), dtype=torch.int64, **kw)
            self.obs = torch.zeros((E, U, 4), dtype=torch.float32, **kw)
            self.serving = torch.full((E, U), -1, dtype=torch.int32, **kw)
            self.reward = torch.zeros((E,), dtype=torch.float32, **kw)
            self.done = torch.zeros((E,), dtype=torch.uint8, **kw)
            self.rate64 = torch.zeros((E, U), dtype=torch.float64, **kw) if rate64 else None
            self.util64 = torch.zeros((E, U), dtype=torch.float64, **kw) if util64 else None
            self.metrics = torch.zeros((E, 4), dtype=torch.float32, **kw) if metrics else None
            self.qoe_stats = (torch.zeros((E, 4), dtype=torch.float64, **kw) if qoe_stats
                              else None)
        self._bind()
        self.seed(seeds)
        with torch.cuda.device(device):
            N.check(L.mev_update_stations(self._ctx, _ptr(self.bs_xy), self._stream()),
                    "mev_update_stations")
            N.check(L.mev_update_layouts(self._ctx, C.byref(self._st), None, self._stream()),
                    "mev_update_layouts")

    # -- plumbing -----------------------------------------------------------------------------
    def _bind(self):
        self._st = N.MevState(_ptr(self._ue_raw), _ptr(self._pcg), _ptr(self.t),
                              _ptr(self.bs_xy), _ptr(self.bs_count))
        self._out = N.MevOutputs(_ptr(self.obs), _ptr(self.serving), _ptr(self.reward),
                                 _ptr(self.done), _ptr(self.rate64), _ptr(self.util64),
                                 _ptr(self.metrics), _ptr(self.qoe_stats))

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def ue_state(self):
        """UE state rows [E,U,4] int16 {x, y, wx, wy} (wx < 0: no waypoint): the kernels' rows
        (mev_state.ue_state) in their int16 form -- a decoded COPY where the context keeps the
        compact uint8 form (255 = -1; maps <= 255 per side, the default there), so writes to it
        are not seen by the kernels. Write rows with restore_state (or through state_rows)."""
        if not self._u8:
            return self._ue_raw
        v = self._ue_raw.to(torch.int16)
        return torch.where(v == 255, torch.full_like(v, -1), v)

    @property
    def state_rows(self):
        """The kernels' own UE state buffer (mev_state.ue_state) in its own form -- uint8 [E,U,4]
        with 255 for -1 (compact_state) or int16 [E,U,4] -- a writable view: writes reach the
        next launch. After writing mid-episode rows, declare the stream states with
        restore_state if the envs' pcg rows changed too."""
        return self._ue_raw

    @property
    def state_bytes_per_ue(self) -> int:
        """4 (compact uint8 x4 rows) or 8 (int16 x4) -- mev_state_bytes_per_ue."""
        return int(self._lib.mev_state_bytes_per_ue(self._ctx))

    @property
    def ue_xy(self):
        """UE positions [E,U,2] int16: a view of the rows in the int16 form, a decoded copy in
        the compact form (see ue_state)."""
        return self._ue_raw[..., :2] if not self._u8 else self._ue_raw[..., :2].to(torch.int16)

    @property
    def wp_xy(self):
        """RandomWaypoint targets [E,U,2] (int16; x < 0: none)."""
        return self.ue_state[..., 2:]

    @property
    def d2max(self) -> int:
        return int(self._lib.mev_d2max(self._ctx))

    @property
    def fused_steps(self) -> bool:
        """step(n > 1) / rollout(n) run as one fused launch (fuse_steps >= 0)."""
        return self.p.fuse_steps >= 0

    @property
    def launch_parts(self) -> int:
        """Env halves per step launch (1, or 2 on two streams)."""
        return int(self._lib.mev_launch_parts(self._ctx))

    @property
    def step_shape(self) -> str:
        """"packed" (one lane per UE, several envs per wavefront) or "block" (one workgroup
        per env) -- mev_step_shape."""
        return {1: "packed", 2: "block"}[int(self._lib.mev_step_shape(self._ctx))]

    @property
    def lds_tables_bytes(self) -> int:
        """Bytes of the LDS association tables of rollout launches (0: L2 map gather)."""
        return int(self._lib.mev_lds_tables_bytes(self._ctx))

    @property
    def rollout_instance(self) -> int:
        """Rollout kernel instance: 0 generic, s > 0 registered scenario s with constants."""
        code = int(self._lib.mev_rollout_instance(self._ctx))
        N.check(min(code, 0), "mev_rollout_instance")  # (negative: a null or closed context)
        return code

    #: mev_last_launch_kind codes (include/mev.h MEV_KIND_*)
    LAUNCH_KINDS = {0: None, 1: "packed_step", 2: "packed_fused", 3: "lds2_two_groups",
                    4: "lds2_one_group", 5: "lds2_pipelined", 6: "lds2_per_env", 7: "block",
                    8: "lds2_pipelined_seg32", 9: "lds2_het"}

    @property
    def last_launch_kind(self) -> "str | None":
        """The step kernel the last step() / rollout() launched (mev_last_launch_kind): every
        kind computes the same results; tests use it to pin which kernel they checked."""
        code = int(self._lib.mev_last_launch_kind(self._ctx))
        if code < 0:  # MEV_EINVAL: a null or closed context
            N.check(code, "mev_last_launch_kind")
        if code not in self.LAUNCH_KINDS:
            raise N.MevError(N.MEV_EINVAL, f"mev_last_launch_kind: unknown kind {code}")
        return self.LAUNCH_KINDS[code]

    @property
    def share_tie_free(self) -> bool:
        """The rate table needs no tie test in the LDS rollouts' share (mev_share_tie_free)."""
        return bool(self._lib.mev_share_tie_free(self._ctx))

    def share_cents(self, nmax: int, path: int = 0):
        """Device rounded shares rint((rate_full[d2] / n) * 100) for n in [1, nmax] as the
        kernels form them (path 0: reciprocal form; 1: 100/n table form, nmax <= 64):
        float64 [nmax, d2max + 1] on the device (tests)."""
        out = torch.empty((int(nmax), self.d2max + 1), dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_share_cents(self._ctx, int(nmax), int(path), _ptr(out),
                                              self._stream()), "mev_share_cents")
        return out

    def rate_table(self):
        """Host copy (numpy float64) of the device channel table rate_full[0..d2max]."""
        import numpy as np
        host = np.zeros(self.d2max + 1, dtype=np.float64)
        N.check(self._lib.mev_copy_rate_table(self._ctx, host.ctypes.data, len(host)),
                "mev_copy_rate_table")
        return host

    # -- API ----------------------------------------------------------------------------------
    def seed(self, seeds):
        """Set per-env config seeds (movement stream = seed + 4); takes effect at reset."""
        import numpy as np
        s = np.asarray(seeds, dtype=np.int64).reshape(-1)
        if len(s) == 1 and self.p.num_envs > 1:
            s = s[0] + np.arange(self.p.num_envs, dtype=np.int64)
        if len(s) != self.p.num_envs:
            raise ValueError(f"need {self.p.num_envs} seeds, got {len(s)}")
        if (s < 0).any() or (s > np.iinfo(np.int64).max - 4).any():
            raise ValueError("seeds must lie in [0, 2^63 - 5]")
        if len(s) >= 4096:  # SeedSequence hashing on the device for large batches
            d_seeds = torch.from_numpy(s + 4).to(self.device)
            with torch.cuda.device(self.device):
                N.check(self._lib.mev_seed_pcg64_device(_ptr(d_seeds), len(s), _ptr(self._pcg),
                                                        self._stream()),
                        "mev_seed_pcg64_device")
        else:
            rows = N.seed_pcg64((s + 4).astype(np.uint64))
            self._pcg.copy_(torch.from_numpy(rows.view(np.int64)).to(self.device))
        self.t.fill_(self.p.t_end)
        with torch.cuda.device(self.device):  # the episode draw tables follow the new streams
            N.check(self._lib.mev_prepare_draws(self._ctx, C.byref(self._st), None,
                                                self._stream()), "mev_prepare_draws")

    def sync_stream_state(self):
        """Materialise every env's movement stream state in the pcg rows (mev_sync_stream_state):
        with the episode draw table the kernels leave the state column as it is while an
        episode's draws stay inside the table. (``pcg`` does this on every read.)"""
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_sync_stream_state(self._ctx, C.byref(self._st), self._stream()),
                    "mev_sync_stream_state")

    @property
    def pcg(self):
        """The movement streams [E, 6] int64 {state, inc, state0} (u128 each, numpy PCG64,
        movement.py:16-18), every state current: reading it synchronises the state column first
        (mev_sync_stream_state), so a saved copy is a valid checkpoint. Writes to the returned
        tensor reach the engine's rows; after writing mid-episode states call
        ``restore_state`` (or use it to write them)."""
        self.sync_stream_state()
        return self._pcg

    def restore_state(self, ue_state, pcg, t, mask=None, declare=True):
        """Load a checkpoint {ue_state [E,U,4] int16, pcg [E,6] (as read from ``pcg``), t [E]}
        taken at any step of an episode (all envs, or those with mask[e]) and continue from it:
        the envs' waypoint draws continue from the saved stream states until their next reset
        (mev_restore_stream_state), exactly as the saving engine would have continued."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.bool)
        src = [torch.as_tensor(x, device=self.device) for x in (ue_state, pcg, t)]
        if self._u8:  # the compact form: -1 -> 255
            v = src[0].to(torch.int16)
            src[0] = torch.where(v < 0, torch.full_like(v, 255), v)
        for dst, x in zip((self._ue_raw, self._pcg, self.t), src):
            x = x.to(dst.dtype).reshape(dst.shape)
            if m is None:
                dst.copy_(x)
            else:
                dst[m] = x[m]
        mk = m.to(torch.uint8).contiguous() if m is not None else None
        if not declare:  # (tests: the rows alone, as a caller forgetting the call would)
            return
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_restore_stream_state(self._ctx, C.byref(self._st), _ptr(mk),
                                                       self._stream()),
                    "mev_restore_stream_state")
        self._keep = mk

    def set_bs_layout(self, bs_xy, bs_count=None):
        bs = torch.as_tensor(bs_xy, dtype=torch.int32, device=self.device)
        if tuple(bs.shape) != tuple(self.bs_xy.shape):
            raise ValueError("layout shape mismatch")
        _check_station_range(bs, bs_count, station_limit(self.p.width, self.p.height))
        if bs_count is not None and self.bs_count is None:
            raise ValueError("engine was built without bs_count")
        self.bs_xy.copy_(bs)
        if bs_count is not None:
            self.bs_count.copy_(torch.as_tensor(bs_count, dtype=torch.int32))
        with torch.cuda.device(self.device):  # re-derive the station keys / culling records
            N.check(self._lib.mev_update_stations(self._ctx, _ptr(self.bs_xy), self._stream()),
                    "mev_update_stations")
            N.check(self._lib.mev_update_layouts(self._ctx, C.byref(self._st), None,
                                                 self._stream()), "mev_update_layouts")

    def reset(self, mask=None):
        """MComCore.reset for all envs (mask None) or envs where mask[e] != 0."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_reset(self._ctx, C.byref(self._st), C.byref(self._out),
                                        _ptr(m), self._stream()), "mev_reset")
        self._keep = m  # keep mask alive until the launch is consumed

    def step(self, nsteps: int = 1):
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_step(self._ctx, C.byref(self._st), C.byref(self._out),
                                       int(nsteps), self._stream()), "mev_step")

    def trajectory(self, nsteps: int) -> "Trajectory":
        """Allocate trajectory buffers for rollout(nsteps): every per-step output with a
        leading step axis (the optional float64 / metrics outputs as the engine was built)."""
        E, U = self.p.num_envs, self.p.num_ues
        kw = dict(device=self.device)
        n = int(nsteps)
        return Trajectory(
            obs=torch.empty((n, E, U, 4), dtype=torch.float32, **kw),
            serving=torch.empty((n, E, U), dtype=torch.int32, **kw),
            reward=torch.empty((n, E), dtype=torch.float32, **kw),
            done=torch.empty((n, E), dtype=torch.uint8, **kw),
            rate64=(torch.empty((n, E, U), dtype=torch.float64, **kw)
                    if self.rate64 is not None else None),
            util64=(torch.empty((n, E, U), dtype=torch.float64, **kw)
                    if self.util64 is not None else None),
            metrics=(torch.empty((n, E, 4), dtype=torch.float32, **kw)
                     if self.metrics is not None else None))

    def rollout(self, nsteps: int, traj: "Trajectory | None" = None) -> "Trajectory":
        """mev_rollout: ``nsteps`` steps (as step(nsteps): one launch) keeping
        every step's outputs -- row i of the returned trajectory is step i. ``traj`` (from
        trajectory(n), n >= nsteps) is reused when given. The engine's own one-step output
        tensors (obs, serving, ...) are not written; qoe_stats accumulates as in step()."""
        n = int(nsteps)
        if traj is None:
            traj = self.trajectory(n)
        if traj.obs.shape[0] < n or tuple(traj.obs.shape[1:]) != tuple(self.obs.shape):
            raise ValueError("trajectory buffers do not fit this engine / nsteps")
        if (traj.rate64 is None) != (self.rate64 is None) or \
                (traj.util64 is None) != (self.util64 is None) or \
                (traj.metrics is None) != (self.metrics is None):
            raise ValueError("trajectory outputs differ from the engine's output set")
        if n == 0:
            return traj
        out = N.MevOutputs(_ptr(traj.obs), _ptr(traj.serving), _ptr(traj.reward),
                           _ptr(traj.done), _ptr(traj.rate64), _ptr(traj.util64),
                           _ptr(traj.metrics), _ptr(self.qoe_stats))
        with torch.cuda.device(self.device):
            N.check(self._lib.mev_rollout(self._ctx, C.byref(self._st), C.byref(out), n,
                                          self._stream()), "mev_rollout")
        return traj

    def launcher(self, nsteps: int, traj: "Trajectory | None" = None, events=None):
        """A zero-argument callable that issues ``rollout(nsteps, traj)`` (traj given) or
        ``step(nsteps)`` with every ctypes argument prebuilt: the per-call host cost is one
        foreign call (the benchmark's timed loop). ``events`` (rollouts only): a (start, stop)
        pair of HIP event handles the launch records from its own dispatch
        (mev_rollout_timed). Checks like rollout(): the trajectory must fit and carry the
        engine's output set; the launch runs on the engine's device."""
        n = int(nsteps)
        st = C.byref(self._st)
        with torch.cuda.device(self.device):
            stream = self._stream()
        if traj is None:
            if events is not None:
                raise ValueError("timing events need a trajectory launch (rollout)")
            fn, out, where = self._lib.mev_step, C.byref(self._out), "mev_step"
        else:
            if traj.obs.shape[0] < n or tuple(traj.obs.shape[1:]) != tuple(self.obs.shape):
                raise ValueError("trajectory buffers do not fit this engine / nsteps")
            if (traj.rate64 is None) != (self.rate64 is None) or \
                    (traj.util64 is None) != (self.util64 is None) or \
                    (traj.metrics is None) != (self.metrics is None):
                raise ValueError("trajectory outputs differ from the engine's output set")
            o = N.MevOutputs(_ptr(traj.obs), _ptr(traj.serving), _ptr(traj.reward),
                             _ptr(traj.done), _ptr(traj.rate64), _ptr(traj.util64),
                             _ptr(traj.metrics), _ptr(self.qoe_stats))
            fn, out, where = self._lib.mev_rollout, C.byref(o), "mev_rollout"
        ctx = self._ctx
        dev = self.device.index
        if events is not None:
            fn, where = self._lib.mev_rollout_timed, "mev_rollout_timed"
            ev0, ev1 = (C.c_void_p(int(e) if e else 0) for e in events)

            def go():
                if torch.cuda.current_device() != dev:
                    raise RuntimeError(f"launcher of cuda:{dev} called with another device current")
                rc = fn(ctx, st, out, n, stream, ev0, ev1)
                if rc:
                    N.check(rc, where)
        else:
            def go():
                if torch.cuda.current_device() != dev:
                    raise RuntimeError(f"launcher of cuda:{dev} called with another device current")
                rc = fn(ctx, st, out, n, stream)
                if rc:
                    N.check(rc, where)
        go.keep = (out, traj, events)
        return go

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            torch.cuda.synchronize(self.device)
            self._lib.mev_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
