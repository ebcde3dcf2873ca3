/*
 * mev.h -- C ABI of the MI355X-native mobile-env step engine (libmev.so).
 *
 * The reference (yang-peilin/mobile-env-gan) is pure Python: its hot path is
 * MComCore.step() (mobile_env/core/base.py:230-296) calling the plugin objects
 * RandomWaypointMovement.move (core/movement.py:42-62), OkumuraHata via
 * Channel.calculateSNR / Channel.datarate (core/channels.py:24-27,78-83,133-146),
 * ResourceFair.share (core/schedules.py:20-22), BoundedLogUtility
 * (core/utilities.py:44-58), NoDeparture (core/arrival.py:28-36) and the metrics
 * (core/metrics.py:5-28). The reference has no FFI; this header is the boundary
 * the Python host (mobile-env-gan_amd/mobile_env/core/_native.py, ctypes) binds.
 * Each entry point names the reference interface it replaces.
 *
 * Conventions
 *   - Return 0 on success, a negative MEV_E* code on error (mev_strerror()).
 *   - All state / output buffers are DEVICE pointers owned by the caller (the
 *     Python host allocates them as torch tensors); the context owns only the
 *     read-only tables it builds (channel rate table, PCG64 jump table).
 *   - Launches are asynchronous and stream-ordered on the hipStream_t passed as
 *     `stream` (NULL = default stream). A context is not thread-safe; use one
 *     context per (device, stream).
 *   - Layout (SoA, row-major, E envs, U UEs, B base stations per env):
 *       ue_state int16 [E][U][4]  {x, y, wx, wy}: UE position (integer grid,
 *                                 entities.py:52-54) and RandomWaypoint target
 *                                 (movement.py:44-47); wx < 0 means "no waypoint";
 *                                 or uint8 [E][U][4] with 255 for -1 (compact_state,
 *                                 maps <= 255 per side; mev_state_bytes_per_ue)
 *       pcg     uint64[E][6]      numpy-PCG64 stream of the movement model:
 *                                 {state_lo, state_hi, inc_lo, inc_hi,
 *                                  state0_lo, state0_hi}; state0 = state right after
 *                                 seeding (movement re-seeds each episode,
 *                                 movement.py:16-18 with reset_rng_episode=True).
 *                                 With the episode draw table (draw_table) the
 *                                 step kernels leave {state} as it is while the
 *                                 episode's draws stay inside the table -- the
 *                                 table holds the state then -- and write it
 *                                 only after draws past it; mev_sync_stream_state
 *                                 materialises it (checkpoints, comparisons)
 *       t       int32 [E]         episode time (base.py:175,280)
 *       bs_xy   int32 [B][2] (shared; the step kernel uses the keys derived from it by
 *                                 mev_reset / mev_update_stations) or [E][B][2] (per env);
 *                                 coordinates in [0, 1024), or [0, 4096) on a map
 *                                 beyond 1024 per side
 *       bs_count int32 [E]        per-env number of valid BSs (NULL: all B)
 *     outputs
 *       obs     f32  [E][U][4]    {x/W, y/H, data rate, scaled utility}
 *       serving i32  [E][U]       serving BS index, -1 = not connected
 *       reward  f32  [E]          mean scaled utility (metrics.py:25-28)
 *       done    u8   [E]          episode over after this step (base.py:407-409)
 *       rate64  f64  [E][U]       optional (NULL): data rate in float64
 *       util64  f64  [E][U]       optional (NULL): scaled utility in float64 (NaN if inactive)
 *       metrics f32  [E][4]       optional (NULL): number connections, number
 *                                 connected, mean utility, mean datarate
 */
#ifndef MEV_H_
#define MEV_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MEV_ABI_VERSION 23

#define MEV_OK 0
#define MEV_EINVAL (-22)   /* bad parameters / shapes */
#define MEV_ENOMEM (-12)   /* device allocation failed */
#define MEV_EHIP (-1000)   /* HIP runtime error (see mev_last_hip_error) */
#define MEV_ECHANNEL (-1001) /* channel connectivity is not a prefix of d2 */

/* Scenario / plugin parameters. Mirrors MComCore.default_config() (base.py:103-153):
 * "bs" -> bs_*, "ue" -> ue_*, "utility_params" -> util_*, "arrival_params" ep_time ->
 * arrival_exit, EP_MAX_TIME -> ep_max_time, "movement_params" width/height. */
typedef struct mev_params {
  int32_t num_envs;       /* E; E * U < 2^28 per context (shard larger batches) */
  int32_t num_ues;        /* U, 1..1024 */
  int32_t num_bs;         /* B (max per env), 1..1024 */
  int32_t width, height;  /* map size (base.py:104), 1..4096 per side. Beyond 1024 the
                             association keys hold the squared distance itself (<= 2 x 1023^2:
                             a channel that connects farther is refused), per-env layouts with
                             U <= 64 run on the block kernel, and no LDS tables / culling */
  int32_t ep_max_time;    /* EP_MAX_TIME (base.py:109) */
  int32_t arrival_start;  /* NoDeparture arrival time, 0 (arrival.py:32-33) */
  int32_t arrival_exit;   /* NoDeparture departure time = ep_time (arrival.py:35-36) */
  int32_t bs_per_env;     /* 0: bs_xy is [B][2]; 1: bs_xy is [E][B][2] */
  int32_t first_step_active; /* 1: activeUsers filled at reset (custom.py:53-54);
                                0: bare MComCore quirk, first step of an episode is a no-op */
  int32_t movement_reseed;   /* 1: movement RNG re-seeded every episode (movement_params
                                reset_rng_episode=True, base.py:133, movement.py:16-18);
                                0: one stream continued across episodes */
  int32_t draw_table;        /* episode draw table (U <= 64, movement_reseed = 1): pairs per
                                env precomputed from state0 by mev_reset / mev_prepare_draws
                                (every episode of an env draws the same sequence); -1 auto
                                (3U + 8), 0 off */
  int32_t fuse_steps;        /* mev_step(n > 1), U <= 64: 0 (auto) -> the n steps run in ONE
                                launch with the env state in registers between them (outputs
                                written every step, identical results); -1: n launches */
  int32_t stream_split;      /* mev_step launch shape: 0 (auto) or 1: one kernel per step on
                                the caller's stream; 2: the env batch in two halves on the
                                caller's stream and a context-owned stream (joined before
                                return), so one half's tail overlaps the other half's start */
  double velocity;        /* UE velocity (base.py:119, custom.py:16-18) */
  double bs_bw, bs_freq, bs_tx, bs_height;        /* base.py:117 */
  double ue_snr_tr, ue_noise, ue_height;          /* base.py:118-123 */
  double util_lower, util_upper;                  /* base.py:136 */
  double util_w1, util_w2, util_w3;               /* coeffs (10, 0, 10) */
  double qoe_low;         /* low-QoE threshold of the layout score (chooseBaseStation.ipynb
                             cell 5: low_qoe_threshold = 0.0) */
  /* Channel rate table (optional, HOST memory, read by mev_create only): rate_table[d2] =
   * Channel.datarate(bs, ue, Channel.calculateSNR(bs, ue)) for a pair at integer squared
   * distance d2 (channels.py:24-27,78-83,133-146), for d2 in [0, rate_table_len); the pairs at
   * d2 >= rate_table_len are not connectable (snr <= snr_tr). The Python host builds it with
   * numpy in the reference's operation order (mobile_env.core.channels), which makes it the
   * reference's own values on the host that runs it. NULL: mev_create builds it on the host
   * with the C library's log10 / pow / log2 in the same order (mev_build_rate_table). */
  const double* rate_table;
  int64_t rate_table_len;
  /* Heterogeneous entities (entities.py:7-22,33-45: every BaseStation / UserEquipment carries
   * its own parameters; the channel is evaluated per pair, channels.py:133-146). 0 or 1 classes
   * on both sides: every station / UE has the bs_* / ue_* / velocity values above. Otherwise
   * (HOST arrays, read by mev_create only) station j belongs to class bs_class[j] <
   * num_bs_classes with {bw, freq, tx, height} = bs_class_params[4 c ..], UE u to class
   * ue_class[u] < num_ue_classes with {velocity, snr_tr, noise, height} = ue_class_params[4 c ..]
   * (at most 16 classes each); a UE connects to the closest station whose pair SNR exceeds its
   * snr_tr (base.py:236-241). rate_table then holds one table per class pair
   * p = cb * num_ue_classes + cu at [rate_table_offsets[p], rate_table_offsets[p + 1]) (NULL
   * rate_table: built with libm). With a shared layout and U <= 64 heterogeneous contexts run the
   * packed kernels (one association map per UE class, [num_ue_classes][H][W] x 16 B); with
   * per-env layouts or U > 64, the block kernel. */
  int32_t num_bs_classes, num_ue_classes;
  const int32_t* bs_class;
  const int32_t* ue_class;
  const double* bs_class_params;
  const double* ue_class_params;
  const int64_t* rate_table_offsets;
  /* Launch-shape overrides, for tests and A/B measurements (0 everywhere = automatic: the
   * fastest shape the context qualifies for). Results are identical for every setting.
   *   lds_tables: rollouts of a shared layout read the association from LDS tables of mode
   *     1..3 (KTables::lds_blob in mev_step.hip), -1: from the L2 association map;
   *   two_groups: -1: one env group per wavefront in rollout launches (the packed kernel);
   *     0: two groups per wavefront where the batch fills the GPU with pairs, else the
   *     software-pipelined one-group kernel for the registered U = 15 / 30 scenarios, else
   *     the packed kernel; 1 / 2: the two-group kernel with two / one groups per wavefront at
   *     any batch size; 3 / 4: the pipelined one-group kernel at any batch size (where it
   *     applies), U = 15 in 16- / 32-lane segments. Heterogeneous entities on a shared layout
   *     (lds_mode 5 tables, when they fit in LDS): 0 / 2 one group per wavefront, 1 two;
   *   stage_rows: > 0: at most that many staged rows of per-env outputs per window;
   *   xcd_remap: -1: blocks in dispatch order (else XCD-contiguous env ranges; 2..8: the
   *     ranges rotated by xcd_remap - 1 XCDs, a placement experiment);
   *   scenario_constants: -1: the generic kernel instances only (else a registered scenario's
   *     parameters are compiled in when every value matches);
   *   station_culling: -1: the U > 64 kernel scans every station per UE (else per-cell
   *     candidate lists where the layout qualifies: 32..255 stations, map <= 512 x 512);
   *   ues_per_lane: U > 64 kernel, 1 / 2 UEs per lane (0: two in one-step launches for
   *     U > 512 with homogeneous entities -- half the waves per env, so that 1,024 envs of
   *     1,024 UEs are resident in one round of the chip's wave slots instead of two -- and one
   *     in multi-step launches). */
  int32_t lds_tables, two_groups, stage_rows, xcd_remap, scenario_constants, station_culling;
  int32_t ues_per_lane;
  /* Per-UE velocity (optional, HOST [num_ues], read by mev_create only): UserEquipment u moves
   * with ue_velocity[u] (entities.py:33-45, movement.py:42-62) instead of `velocity` / its
   * class's velocity. Velocity drives only the movement, so distinct velocities need no
   * parameter class: any number of them (one per UE) with the channel classes above limited
   * to the (snr_tr, noise, height) tuples that differ. All equal: the same as `velocity`. */
  const double* ue_velocity;
  /* 1: the compact UE state form, ue_state = uint8 [E][U][4] {x, y, wx, wy} with 255 for -1
   * (no waypoint) -- half the state bytes, which one-step launches move every step; maps up to
   * 255 per side only (every registered scenario is 200 x 200). 0: int16 [E][U][4]. */
  int32_t compact_state;
  /* Reward precision. The lean kernels (no float64 outputs) form the float32 reward from
   * float32 utilities; wherever that sum could miss the reference's float64 mean by more than
   * 1e-5 relative (mean utilities near zero: cancellation), the env's reward is re-formed from
   * the exact float64 utilities (reward_risky in mev_step.hip). 1: every reward that way (the
   * float32 reward of the float64 mean -- slower; tests pin the exact path with it). k <= -2
   * (tests): the risk band k times wider, so that a subset of rows takes the exact path. Every
   * kernel shape decides with the same test (the 2^-25 fixed-point sum against nact r_thr25),
   * so one env-step's reward has the same bits whichever shape ran it. */
  int32_t reward_exact;
} mev_params;

typedef struct mev_state {
  int16_t* ue_state;      /* (uint8_t* with compact_state) */
  uint64_t* pcg;
  int32_t* t;
  const int32_t* bs_xy;
  const int32_t* bs_count; /* may be NULL */
} mev_state;

typedef struct mev_outputs {
  float* obs;
  int32_t* serving;
  float* reward;
  uint8_t* done;
  double* rate64;   /* may be NULL */
  double* util64;   /* may be NULL */
  float* metrics;   /* may be NULL */
  double* qoe_stats; /* may be NULL: [E][4] per-episode statistics of the rounded QoE values
                        round(u, 2) of the active UEs (the values save_epoch_data writes,
                        base.py:269): {count, sum, sum of squares, count below qoe_low};
                        restarted at every episode's first step */
} mev_outputs;

typedef struct mev_ctx mev_ctx;

/* Library ABI version (MEV_ABI_VERSION). */
int mev_abi_version(void);

/* Hash of the sources this library was compiled from (the first 16 hex digits of the SHA-256
 * of csrc/mev_step.hip followed by include/mev.h; "unknown" for a build without the Makefile's
 * -DMEV_SRC_HASH). The Python host compares it with the sources next to the library and refuses
 * a stale build. No reference counterpart (build provenance). */
const char* mev_source_hash(void);

/* Build a context on the current HIP device: validates params, uploads the channel table
 * (Okumura-Hata -> SNR -> Shannon rate at every integer squared distance,
 * channels.py:24-27,78-83,133-146; replaces the per-pair Channel.calculateSNR/datarate calls
 * of base.py:212-214,427-431; params->rate_table, or built on the host) and builds the PCG64
 * jump-ahead table. Replaces MComCore.__init__'s plugin construction (base.py:57-61).
 * Synchronous. */
int mev_create(const mev_params* params, mev_ctx** out);
void mev_destroy(mev_ctx* ctx);

/* Largest connectable squared distance (snr > snr_tr <=> d2 <= d2max); -1 if none. */
int mev_d2max(const mev_ctx* ctx);
/* Number of env halves mev_step launches per step (1, or 2 on two streams; stream_split). */
int mev_launch_parts(const mev_ctx* ctx);
/* Kernel shape of the context's steps: 1 = packed (one lane per UE, U <= 64: several envs per
 * wavefront), 2 = block (one workgroup per env: U > 64, or heterogeneous entities with per-env
 * layouts). */
int mev_step_shape(const mev_ctx* ctx);
/* Bytes of the compact association tables rollout launches copy into LDS (shared layouts whose
 * tables fit); 0: rollouts gather from the L2 association map. */
int mev_lds_tables_bytes(const mev_ctx* ctx);
/* Bytes of one UE's ue_state row: 4 (compact_state, uint8 x4) or 8 (int16 x4). */
int mev_state_bytes_per_ue(const mev_ctx* ctx);
/* Device pointer to the channel rate table (float64 [d2max+1]) -- for tests. */
const double* mev_rate_table(const mev_ctx* ctx);
/* Copy the first n entries of the channel rate table to dst (host or device memory,
 * hipMemcpyDefault). Synchronous. */
int mev_copy_rate_table(const mev_ctx* ctx, double* dst, int64_t n);

/* Host: the channel rate table of params' bs_* / ue_* values with the C library's float64
 * log10 / pow / log2 in the reference's operation order (OkumuraHata.power_loss
 * channels.py:133-146, calculateSNR channels.py:24-27, datarate channels.py:78-83; the
 * distance is sqrt(d2), correctly rounded, like shapely's). Returns n = d2max + 1 (the
 * connectable squared distances are exactly [0, n)) and writes min(n, cap) entries to dst
 * (may be NULL with cap 0: query); MEV_ECHANNEL if connectivity is not a prefix of d2.
 * numpy's log10 (SIMD loops on AVX-512 hosts) can differ from the C library's by one ulp
 * on a few d2: the Python host passes numpy's table in params->rate_table instead. */
int64_t mev_build_rate_table(const mev_params* params, double* dst, int64_t cap);

/* Diagnostic (tests): the device's rounded ResourceFair shares, cents(n, d2) =
 * rint((rate_full[d2] / n) * 100) as the step kernels compute them (base.py:427-435,
 * schedules.py:20-22), for n in [1, nmax] and d2 in [0, d2max]: dst is a DEVICE buffer
 * [nmax][d2max + 1] of float64. path 0: the reciprocal form (one-step and block kernels),
 * path 1: the 100/n table form (n <= 64, LDS-table rollouts). Stream-ordered. */
int mev_share_cents(const mev_ctx* ctx, int32_t nmax, int32_t path, double* dst, void* stream);

/* The rollout kernel instance mev_rollout runs for this context: 0 generic, s > 0 the
 * registered scenario s compiled with its parameters as constants (chosen when every value
 * matches; mev_params.scenario_constants = -1 forces the generic instance). */
int mev_rollout_instance(const mev_ctx* ctx);

/* Diagnostic (tests, A/B tools): the step kernel the context's last mev_step / mev_rollout call
 * launched (0 before any). Every kind computes the same results; the choice depends on the
 * batch, the launch length, the output set and the layout. */
#define MEV_KIND_PACKED_STEP 1   /* one launch per step, one lane per UE (k_step_packed) */
#define MEV_KIND_PACKED_FUSED 2  /* fused steps, one env group per wavefront (k_steps_packed) */
#define MEV_KIND_LDS2_TWO 3      /* fused, two env groups per wavefront (k_steps_lds2, R = 2) */
#define MEV_KIND_LDS2_ONE 4      /* fused, one group per wavefront (k_steps_lds2, R = 1) */
#define MEV_KIND_LDS2_PIPE 5     /* fused, software-pipelined one-group loop (k_steps_lds2 PIPE) */
#define MEV_KIND_LDS2_PERENV 6   /* fused, per-env layouts, two groups per wavefront */
#define MEV_KIND_BLOCK 7         /* one workgroup per env (k_steps_block) */
#define MEV_KIND_LDS2_PIPE32 8   /* the pipelined loop with U <= 16 in 32-lane segments (two envs
                                    per wavefront; two_groups = 4) */
#define MEV_KIND_LDS2_HET 9      /* fused, heterogeneous entities on a shared layout, LDS tables
                                    (k_steps_lds2 HET) */
int mev_last_launch_kind(const mev_ctx* ctx);

/* 1 when the context's rate table needs no tie test in the ResourceFair share of the kernels
 * that form it from a 100/n table: for every entry and every share count n <= num_ues,
 * rint(full * fl(100 / n)) equals the reference's rint(fl(full / n) * 100) (checked
 * exhaustively at mev_create when entries x num_ues <= 10^8; 0 beyond); the scenario-constant
 * two-group and block kernels then skip the test and its exact fallback. */
int mev_share_tie_free(const mev_ctx* ctx);

/* Host helper: numpy-compatible seeding, np.random.default_rng(seed) ->
 * SeedSequence(seed) -> PCG64 (movement seed = config seed + 4, base.py:156-168).
 * Writes n rows of {state_lo, state_hi, inc_lo, inc_hi, state0_lo, state0_hi}
 * (host memory) for non-negative seeds[i] < 2^63. */
int mev_seed_pcg64(const uint64_t* seeds, int64_t n, uint64_t* pcg_rows);
/* The same rows computed on the device: seeds and rows are DEVICE pointers, stream-ordered;
 * a seed >= 2^63 yields an all-zero row (inc = 0) instead of an error. */
int mev_seed_pcg64_device(const uint64_t* seeds, int64_t n, uint64_t* rows, void* stream);

/* Reset envs: MComCore.reset + MComCustom.reset bookkeeping (base.py:172-209,
 * custom.py:53-54) -- re-seed the movement stream, draw initial positions
 * (movement.py:64-72), clear waypoints, t = 0. env_mask: device u8 [E] (NULL = all).
 * Writes obs (positions, rate 0, utility 0), serving = -1. */
int mev_reset(const mev_ctx* ctx, const mev_state* st, const mev_outputs* out,
              const uint8_t* env_mask, void* stream);
/* Rebuild the episode draw tables of the envs with env_mask[e] (all if NULL) from their
 * pcg rows' state0 (mev_reset does it; call it after changing pcg rows without a reset). */
int mev_prepare_draws(const mev_ctx* ctx, const mev_state* state, const uint8_t* env_mask,
                      void* stream);

/* Write every env's movement stream state (numpy PCG64 state after the env's draws so far,
 * movement.py:44-47,64-72) into its pcg row: the step kernels skip that write while an
 * episode's draws stay inside the episode draw table (mev_state.pcg). Stream-ordered. */
int mev_sync_stream_state(const mev_ctx* ctx, const mev_state* st, void* stream);

/* Restore a checkpoint mid-episode: after writing saved {ue_state, pcg, t} rows (pcg saved
 * after mev_sync_stream_state) into this context's state buffers, declare that the pcg rows of
 * the envs with env_mask[e] (all if NULL) hold their CURRENT stream states. Their waypoint
 * draws (movement.py:44-47) then continue from those rows -- not from the episode draw table,
 * whose position in the episode this context does not know -- until each env's next reset,
 * which returns it to the table (rebuilt here from the rows' state0, as mev_prepare_draws).
 * Without it a restored env would re-read the episode's first table pairs. No-op without a draw
 * table. Stream-ordered. */
int mev_restore_stream_state(const mev_ctx* ctx, const mev_state* st, const uint8_t* env_mask,
                             void* stream);

/* Shared station layout (bs_per_env = 0): (re)derive the association keys the step kernel
 * uses from bs_xy (device int32 [B][2]). Called by mev_reset; call it after changing the
 * shared layout between resets. No-op for per-env layouts. Stream-ordered; with the compact
 * LDS tables (mode 3) it then waits for the stream once: the host reads back how many distinct
 * serving distances the layout has (the rollout kernels' choice and LDS sizes depend on it). */
int mev_update_stations(const mev_ctx* ctx, const int32_t* bs_xy, void* stream);

/* Per-env station layouts (bs_per_env = 1): rebuild what the step kernels keep per env from
 * bs_xy / bs_count for the envs with env_mask[e] (all if NULL) -- the block shape's station
 * culling records (per map cell the stations that can be closest), which its short launches
 * (mev_step, rollouts < 32 steps) read instead of scanning every station. Called by mev_reset;
 * call it after changing an env's layout between resets. Envs whose records were never built
 * are scanned in full (same results). No-op for shared layouts (mev_update_stations) and for
 * the packed shape. Stream-ordered. */
int mev_update_layouts(const mev_ctx* ctx, const mev_state* st, const uint8_t* env_mask,
                       void* stream);

/* Advance every env by `nsteps` steps of MComCore.step (base.py:230-296). An env whose
 * episode is over (t >= min(EP_MAX_TIME, departure)) is reset at the start of its next step
 * (lazy auto-reset), so a sequence of steps reproduces the reference driver loop
 * `reset(); step() x20; reset(); ...` (collectData2.ipynb cells 3-4). nsteps > 1 with U <= 64
 * runs as ONE launch (fuse_steps). Outputs hold the last step's results. */
int mev_step(const mev_ctx* ctx, const mev_state* st, const mev_outputs* out,
             int32_t nsteps, void* stream);

/* mev_step keeping every step's outputs (one episode of the collectData2.ipynb loop, whose
 * per-step dump base.py:261,298-349 consumes each step): the buffers of `traj` hold nsteps
 * rows -- obs [n][E][U][4], serving [n][E][U], reward [n][E], done [n][E], rate64 / util64
 * [n][E][U], metrics [n][E][4] -- and step i writes row i. qoe_stats stays [E][4]
 * (per-episode, accumulated as in mev_step). Same results as nsteps mev_step calls. */
int mev_rollout(const mev_ctx* ctx, const mev_state* st, const mev_outputs* traj,
                int32_t nsteps, void* stream);

/* mev_rollout with timing events (hipEvent_t, created by the caller; either may be NULL): a
 * launch of one kernel records them from its own dispatch (hipExtLaunchKernelGGL: the kernel's
 * start and end; no marker packets and no system-scope fence of separate event records around
 * it); launches of several kernels record them before the first and after the last. */
int mev_rollout_timed(const mev_ctx* ctx, const mev_state* st, const mev_outputs* traj,
                      int32_t nsteps, void* stream, void* start_event, void* stop_event);

/* Error text for a return code; last HIP error string for MEV_EHIP. */
const char* mev_strerror(int code);
const char* mev_last_hip_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MEV_H_ */
