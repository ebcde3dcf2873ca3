// mev_step.hip -- MI355X (gfx950) kernels + C ABI of the vectorised mobile-env step engine.
//
// One fused kernel per env-step implements MComCore.step (reference
// mobile_env/core/base.py:230-296) for every env of the batch:
//   move (RandomWaypointMovement.move, movement.py:42-62)
//   -> associate (closest connectable BS, base.py:236-241; Channel.calculateSNR
//      channels.py:24-27 + OkumuraHata channels.py:133-146 folded into the integer
//      test d2 <= d2max)
//   -> per-BS connected-UE counts (ResourceFair.share, schedules.py:20-22)
//   -> rate = round(datarate / n, 2) (base.py:421-435, channels.py:78-83)
//   -> scaled BoundedLogUtility (utilities.py:44-58), reward = mean utility
//      (metrics.py:25-28), the other metrics (metrics.py:5-21)
//   -> time / done bookkeeping (base.py:280-291,407-409; arrival.py:28-36).
//
// Launch shapes:
//   * packed: U <= 64. A wavefront holds floor(64/U) envs, one lane per UE; per-env
//     reductions are ballot/popcount/DPP over the env's lane segment. k_step_packed runs one
//     step per launch (state loaded and stored every step); k_steps_packed runs n steps per
//     launch with the state in registers (mev_step(n), mev_rollout), rollouts reading the
//     association from LDS copies of compact tables in a persistent grid.
//   * block:  64 < U <= 1024. One workgroup (ceil(U/64) waves) per env; per-BS counts
//     with LDS atomics, RNG offsets by a workgroup scan.
// One-step launches are HBM-streaming (per UE 8+8 B state, 16 B obs + 4 B serving); rollout
// launches are bound by their instruction stream.
// Numerics: the reference computes in float64 with numpy; every float64 op here keeps
// the reference's operation order, the file is compiled with -ffp-contract=off, and
// HIP's float64 '/', sqrt and rint are IEEE correctly rounded, so positions, serving
// indices and the rounded rates match the reference exactly (tests/ check it).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <type_traits>
#include <new>
#include <vector>

#include "mev.h"

typedef unsigned __int128 u128;
typedef short s16x2 __attribute__((ext_vector_type(2)));

// numpy PCG64 = PCG XSL-RR 128/64 (numpy/random/src/pcg64/pcg64.h)
#define PCG_MULT_HI 0x2360ED051FC65DA4ULL
#define PCG_MULT_LO 0x4385DF649FCCF645ULL

namespace {

constexpr int kMaxU = 1024;
constexpr int kMaxB = 1024;
constexpr int kMaxClasses = 16;  // station / UE parameter classes (heterogeneous entities)
// largest squared distance of a UE (inside the map) to a station (coordinates < 1024): also
// the longest connectable distance on the larger maps (kMaxMap), whose association keys hold
// the squared distance clamped to 22 bits
constexpr int64_t kD2Top = 2 * 1023 * 1023;
// map side limit: int16 UE state, and on maps beyond 1024 ("wide") coordinates < 4096, so that a
// station-to-UE difference fits int16 and its squared length int32
constexpr int kMaxMap = 4096;
constexpr int kKeyBits = 10;
// (d2, bs) association key: BS index in the low kKeyBits bits

struct KParams {
  int E, U, B, W, H;
  int t_end, arr_start, arr_exit;
  int first_step_active;
  int movement_reseed;
  int d2max;
  int envs_per_wave;  // packed shape only
  int srv_bits;       // bits of a serving-BS index (ceil(log2(B))), for the ballot match
  int util_kmax;      // utility table covers rounded rates k/100 for k in [0, util_kmax]
  int util_direct;    // 1: evaluate the utility in-kernel (no monotone saturation point)
  float u_err;        // bound on |float32 utility (utility_f32r) - float64 utility| (reward_risky)
  float r_thr;        // reward_risky as a bound on the fast mean: |mean| <= r_thr (host, from u_err)
  int r_thr25;        // ... on the 2^-25 fixed-point sum: |isum| <= nact r_thr25
  int hist_lds;       // packed shape: per-env BS counts in an LDS histogram ([G][B] per wave)
  int tab_m;          // episode draw table: pairs per env (0: off)
  float inv_w, inv_h; // obs normalisation
  int d2snap;         // largest integer d2 with sqrt(d2) <= velocity (arrival test)
  float move_band;    // tie band of the float32 movement fast path
  float move_lim;     // 0.5 - move_band (exact)
  float u_log2_coef, u_w2f, u_lowerf, u_upperf, u_scale, u_offset;  // float32 utility
  int axis_exact;     // 1: (velocity * a) / a == velocity for every axis distance a and the
                      // velocity not an integer (axis moves = pos +- velocity, ties for the
                      // fast path: a float64 add instead); 2: velocity 1.5 on a map <= 1024
                      // (the exact integer step, step_v15); 0: neither (integer velocities)
  float vel_f;
  int xcd_remap;      // 1: blocks sharing an XCD (blockIdx % 8) take one contiguous env range
  // LDS association tables of a shared layout (fused launches; 0: off, see KTables::lds_blob)
  int lds_assoc;      // bytes of the blob (multiple of 16)
  int lds_mode;       // 1: station map + rank index; 2: + per-cell rank map; 3: per-cell
                      // {station, rank in the layout's own d2 set} (see KTables::lds_blob)
  int lds_st_off, lds_rank_off, lds_rate_off, lds_r100_off, lds_r16_off;  // byte offsets
  double Wd, Hd, vel, lower, upper, w1, w2, log_w3, util_sat;
  double qoe_low;
  int lbs;            // fused per-env-layout launches: station slots per env staged in LDS (0: off)
  int het;            // heterogeneous entities: nb_cls station classes, nu_cls UE classes
  int nb_cls, nu_cls, bperm;
  // block kernel station culling (0: off): cells of 2^cull_log x 2^cull_log, cull_nx per row,
  // cull_nc in all (block_cull_params)
  int cull_log, cull_nx, cull_nc;
  int st8;            // compact UE state: uint8 x4 per UE (maps <= 255 per side; 255 = -1)
  // 1: the float32 utility cannot hold 1e-5 relative near zero (a nonzero scaled offset or w2:
  // ur * scale + offset / log2(w2 + r) cancel) -- the utility comes from the exact table instead
  // (non-lean kernels); 0 for the reference's default parameters (offset 0, w2 0)
  int util_exact;
};

struct KState {
  int2* ue_state;  // [E][U] {x, y, wx, wy} as int16x4 (8 B per UE; coordinates < 4096, -1), or
                   // with KParams::st8 as uint8 x4 (4 B per UE; 255 = -1: no waypoint)
  uint64_t* pcg;
  int* t;
  const int2* bs_xy;
  const int* bs_count;
};

struct KOut {
  float4* obs;
  int* serving;
  float* reward;
  uint8_t* done;
  double* rate64;
  double* util64;
  float4* metrics;
  double4* qoe_stats;  // [E] {count, sum, sum of squares, count below qoe_low}
};

// Outputs of row i of a trajectory (mev_rollout): every per-step output holds one row per
// step; qoe_stats is per episode and not shifted.
__host__ __device__ __forceinline__ KOut out_row(KOut o, int E, int U, int i) {
  const size_t eu = (size_t)E * U * i, ee = (size_t)E * i;
  o.obs += eu;
  o.serving += eu;
  o.reward += ee;
  o.done += ee;
  if (o.rate64) o.rate64 += eu;
  if (o.util64) o.util64 += eu;
  if (o.metrics) o.metrics += ee;
  return o;
}

// Movement parameters of one UE (velocity and the values derived from it on the host).
struct MoveP {
  double vel;
  float vel_f, move_lim;
  int d2snap, axis_exact;
};

struct KTables {
  const double* rate_full;  // [d2max + 1]
  const u128* jump;         // [2*(jmax+1)]: {a^k, G(k)} with G(k) = sum_{i<k} a^i
  const double* util;       // [util_kmax + 1]: scaled utility of rate k/100
  const int4* assoc;        // [H][W] shared layout: {serving BS or -1, d2, full rate (f64)}
  // episode draw table (movement re-seeded every episode => each env's draws of an episode
  // are a fixed sequence): pair k = the (x, y) of draws 2k, 2k+1 from state0 and the stream
  // state after them; `drawn` = pairs of the current episode consumed so far
  const int* tab_xy;        // [E][M] int16x2
  const u128* tab_st;       // [E][M]
  int* drawn;               // [E]
  // Compact form of `assoc` that fits in LDS (copied once per workgroup by the fused launch):
  //   [0, lds_st_off)          serving station per grid cell, 4 bits (15 = none), 2 per byte
  //   [lds_st_off, +64)        station coordinates x | y << 16 (16 slots)
  //   [lds_rank_off, ...)      uint2 {bits, prefix} per 32 squared distances: bit d of the
  //                            set S of sums of two squares <= d2max, prefix = |S below word|
  //   [lds_r100_off, +576)     100 / n for n in [0, 64] (ResourceFair share, share_cents_r)
  //   [lds_rate_off, ...)      rate_full[d] for d in S, in increasing d (rank of d in S)
  // so full = rate[rank(d2)] with d2 to the serving station: the same float64 values as
  // `assoc`, from four LDS reads instead of one 16-byte gather from L2 per UE and step.
  // Mode 2 adds a per-cell u16 rank at lds_r16_off (two parallel reads, then the rate). Mode 3
  // (the default; cells <= 65536): ONE u16 per cell at offset 0, (station << 12) | k with k the
  // rank of the cell's d2 in D, the set of squared distances that occur between a cell and its
  // serving station in this layout (|D| is ~900 for mobile-large, ~3,300 for mobile-small);
  // 0xF000 = no station in reach, 0xFFFF = k beyond 4094 (such cells take the L2 map);
  // [lds_r100_off, +576) 100 / n; [lds_rate_off, +32 KB) rate_full[d] for d in D, in increasing d.
  const int4* lds_blob;
  // mode 3: |D|, the rates over D in use (k_d2_prefix, per layout): the copies into LDS stop
  // at lds_rate_off + 8 |D| instead of the 4,096 rate slots reserved (113 -> 88 KB for
  // mobile-large); null for the other modes
  const int* dcount;
  // heterogeneous entities (KParams::het): per station class cb / UE class cu
  const uint8_t* bs_cls;    // [B] class of station j
  const uint8_t* ue_cls;    // [U] class of UE u
  const int2* pair;         // [NB * NU] {offset into rate_full, d2max} of class pair cb * NU + cu
  const MoveP* mv;          // [U] movement parameters per UE (its velocity: ue_velocity, else its class's)
  const int16_t* perm;      // [kp.bperm] stations grouped by class (segments of even length,
                            // padded with -1)
  const int* seg;           // [NB + 1] segment bounds in perm
  // station culling records of per-env layouts kept across launches (mev_update_layouts):
  // [E][cull_nc] 16-byte records (see block_cull_params), and per env 1 if they are valid
  const unsigned char* crec_g;
  const uint8_t* crec_ok;
};

// Element at a 32-bit byte offset from a wave-uniform base: addresses become
// `global_load v, v_off, s_base` (no 64-bit address arithmetic per lane). The packed kernel
// uses it for every per-env / per-UE access; mev_create bounds the buffers below 4 GiB.
template <class T>
__device__ __forceinline__ T& at(T* base, uint32_t byte_off) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off);
}

// UE state row {x, y, wx, wy} packed as int16x4: one 8-byte load / store per UE.
__device__ __forceinline__ int4 load_ue(const int2* p) {
  const int2 v = *p;
  return make_int4((int)(short)v.x, v.x >> 16, (int)(short)v.y, v.y >> 16);
}

__device__ __forceinline__ void store_ue(int2* p, int2 pos, int2 wp) {
  *p = make_int2((int)(((unsigned)pos.x & 0xffffu) | ((unsigned)pos.y << 16)),
                 (int)(((unsigned)wp.x & 0xffffu) | ((unsigned)wp.y << 16)));
}

// Compact UE state (KParams::st8, maps <= 255 per side): {x, y, wx, wy} as uint8 x4, one 4-byte
// load / store per UE (half the state bytes of the int16 form: the one-step launches move the
// state every step); 255 encodes -1 (no waypoint).
__device__ __forceinline__ int dec8(unsigned b) { return b == 255u ? -1 : (int)b; }
__device__ __forceinline__ unsigned pack8(int2 pos, int2 wp) {
  return ((unsigned)pos.x & 255u) | (((unsigned)pos.y & 255u) << 8) |
         (((unsigned)wp.x & 255u) << 16) | ((unsigned)wp.y << 24);
}
__device__ __forceinline__ int4 unpack8(unsigned v) {
  return make_int4((int)(v & 255u), (int)((v >> 8) & 255u), dec8((v >> 16) & 255u),
                   dec8(v >> 24));
}
// UE ui's state row in either form (`st8` wave-uniform, a compile-time constant in the
// scenario instances)
__device__ __forceinline__ int4 load_ue_at(int2* base, uint32_t ui, bool st8) {
  if (st8) return unpack8(at(reinterpret_cast<unsigned*>(base), 4u * ui));
  return load_ue(&at(base, 8u * ui));
}
__device__ __forceinline__ void store_ue_at(int2* base, uint32_t ui, int2 pos, int2 wp, bool st8) {
  if (st8) at(reinterpret_cast<unsigned*>(base), 4u * ui) = pack8(pos, wp);
  else store_ue(&at(base, 8u * ui), pos, wp);
}

// ------------------------------------------------------------------------------------
// PCG64 helpers (device)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ u128 mk128(uint64_t lo, uint64_t hi) {
  return ((u128)hi << 64) | (u128)lo;
}

__device__ __forceinline__ uint64_t pcg_output(u128 s) {
  const uint64_t hi = (uint64_t)(s >> 64);
  const uint64_t lo = (uint64_t)s;
  const unsigned rot = (unsigned)(hi >> 58);
  const uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64u - rot) & 63u));
}


// numpy Generator.uniform(0, span) is off + scale * next_double with next_double =
// (next_uint64 >> 11) * 2^-53 (numpy/random/src/distributions/distributions.c); the reference
// then truncates with int() (movement.py:45-46,67-68). PCG64 advances, then outputs.
// The two draws (x then y) of a waypoint / initial position at stream offsets k+1, k+2:
// jump straight to offset k+1 with the table, then one step with the constant multiplier.
// Returns the stream state after both draws.
__device__ __forceinline__ u128 pcg_draw_pair(u128 s, u128 inc, int k, const u128* jump,
                                              double w, double h, int& x, int& y) {
  const u128 s1 = jump[2 * (k + 1)] * s + jump[2 * (k + 1) + 1] * inc;
  x = (int)(0.0 + w * ((double)(pcg_output(s1) >> 11) * (1.0 / 9007199254740992.0)));
  const u128 s2 = s1 * mk128(PCG_MULT_LO, PCG_MULT_HI) + inc;
  y = (int)(0.0 + h * ((double)(pcg_output(s2) >> 11) * (1.0 / 9007199254740992.0)));
  return s2;
}

// The same pair at stream offsets 1, 2 (two steps of the constant multiplier).
__device__ __forceinline__ u128 pcg_draw_pair_next(u128 s, u128 inc, double w, double h, int& x,
                                                   int& y) {
  const u128 a = mk128(PCG_MULT_LO, PCG_MULT_HI);
  const u128 s1 = s * a + inc;
  x = (int)(0.0 + w * ((double)(pcg_output(s1) >> 11) * (1.0 / 9007199254740992.0)));
  const u128 s2 = s1 * a + inc;
  y = (int)(0.0 + h * ((double)(pcg_output(s2) >> 11) * (1.0 / 9007199254740992.0)));
  return s2;
}

// Registered scenarios with default parameters (medium, large; 200 x 200 map, default channel,
// NoDeparture, draw table 3U + 8, the LDS tables of mode 3): their rollout launches run
// an instance with these values as constants (SCN > 0; fewer kernel arguments held in
// SGPRs: -3 % time per step), chosen on the host only when every value matches the context's.
struct ScnConst {
  int U, B, W, H, tab_m, hist_lds, t_end, arr_start, arr_exit, first_step_active;
  int lds_r16_off, lds_r100_off, lds_rate_off, lds_assoc;
  // velocity 1.5, default utility: float32 values as bit patterns
  int d2snap, axis_exact;
  unsigned vel_f, move_lim, inv_w, inv_h, u_log2_coef, u_w2f, u_lowerf, u_upperf, u_scale,
      u_offset;
  int d2max;
  int cull_log, cull_nx, cull_nc;
};
__host__ __device__ constexpr ScnConst scn_const(int scn) {
#define MEV_SCN_F32 2, 2, 0x3fc00000u, 0x3efffd00u, 0x3ba3d70au, 0x3ba3d70au, 0x4040a8c1u, \
                    0x00000000u, 0xc1a00000u, 0x41a00000u, 0x3d4ccccdu, 0x00000000u, 19362
  // (LDS tables of mode 3 for 200 x 200: cell entries [0, 80000), 100/n at 80000, rates at
  // 80576, 113344 bytes in all)
  return scn == 1 ? ScnConst{15, 7, 200, 200, 53, 1, 20, 0, 20, 1, 0, 80000, 80576, 113344,
                             MEV_SCN_F32}
       : scn == 2 ? ScnConst{30, 13, 200, 200, 98, 1, 20, 0, 20, 1, 0, 80000, 80576, 113344,
                             MEV_SCN_F32}
       // mobile-large-perenv-v0: per-env layouts, mode-4 tables of the default channel (rank
       // index of S at 0, 100/n at 4848, rates at 5424, 46240 bytes)
       : scn == 3 ? ScnConst{30, 13, 200, 200, 98, 1, 20, 0, 20, 1, 0, 4848, 5424, 46240,
                             MEV_SCN_F32}
       // mobile-custom-128x1024-v0 (block kernel): velocity 10 (d2snap 100, float32 10, tie
       // band 2^-16 x 10), draw table 3U + 8, no LDS tables, default channel and utility
       : scn == 4 ? ScnConst{1024, 128, 200, 200, 3080, 0, 20, 0, 20, 1, 0, 0, 0, 0, 100, 0,
                             0x41200000u, 0x3effec00u, 0x3ba3d70au, 0x3ba3d70au, 0x4040a8c1u,
                             0x00000000u, 0xc1a00000u, 0x41a00000u, 0x3d4ccccdu, 0x00000000u,
                             19362, 2, 50, 2500}
                  : ScnConst{};
}
// every registered scenario is a 200 x 200 map: compact state (the host sets st8 there)
__host__ __device__ constexpr bool scn_st8(int scn) { return scn >= 1 && scn <= 4; }
#define KPS(f) (SCN ? scn_const(SCN).f : kp.f)
#define KST8 (SCN ? scn_st8(SCN) : kp.st8 != 0)
#define KPSF(f) (SCN ? __builtin_bit_cast(float, scn_const(SCN).f) : kp.f)

// Per-UE movement (movement.py:42-62), exact float64 form: the reference computes
// position + velocity * v / |v| in float64, then np.round (half-to-even) and astype(int).
__device__ __forceinline__ int2 move_exact(int2 pos, int dx, int dy, double vel) {
  const double nrm = sqrt((double)(dx * dx + dy * dy));  // np.linalg.norm of the int vector
  return make_int2((int)rint((double)pos.x + (vel * (double)dx) / nrm),
                   (int)rint((double)pos.y + (vel * (double)dy) / nrm));
}


// Velocity 1.5 (the registered scenarios' and mobile-env's default) in integers, exactly
// (MoveP::axis_exact == 2, or the scenario instances' constants): off the axes
// |q| = 1.5 |dx| / |v| lies strictly between 0 and 1.5, and |q| > 1/2 <=> 8 dx^2 > dy^2
// (equality has no integer solution but 0, and |q| stays > 1e-7 away from 1/2 for coordinates
// < 1024, far beyond float64's rounding of the reference's expression), so the step is
// sgn(dx) [8 dx^2 > dy^2]; on an axis q = +-1.5 exactly, and np.round's half-to-even gives
// |step| 2 from an even coordinate, 1 from an odd one. (Arrival, d2 <= 2, is the caller's;
// tests/test_oracle.py checks the formula against the reference expression for every
// displacement of a 200 x 200 map.)
__device__ __forceinline__ int2 step_v15(int2 pos, int dx, int dy, int ax2, int ay2) {
  const int sx = (ax2 << 3 > ay2 ? 1 : 0) + (dy == 0 && !(pos.x & 1) ? 1 : 0);
  const int sy = (ay2 << 3 > ax2 ? 1 : 0) + (dx == 0 && !(pos.y & 1) ? 1 : 0);
  return make_int2(pos.x + (dx < 0 ? -sx : sx), pos.y + (dy < 0 ? -sy : sy));
}
// step_v15 in fewer VALU: [8 dx^2 > dy^2] as the sign bit of dy^2 - 8 dx^2 (one 24-bit
// multiply-add and a shift), and x + sgn(dx) sx as one 24-bit multiply-add with sgn(dx) =
// med3(dx, -1, 1): 24 instead of 29 VALU per UE and step with the selects. (The two as inline
// assembly: written in C, the compiler turned the multiply by -8 into a shift pair and the clamp
// of wp.x - x into two compares and two selects against the coordinates.) dx = 0 gives sgn 0
// and, off the arrival radius, sx = 0 as well, so the product is the step either way. Taken by
// the software-pipelined loop (4,096 medium envs, one wave per SIMD: 90.4 vs 95.6 us per
// 200-step launch, interleaved); in the two-group loop it measured slower (20-step 163.8 vs
// 162.6 us, 200-step 1.54 vs 1.49 ms -- as for every step shortened there) and the
// Gym step() unchanged, so those keep step_v15.
__device__ __forceinline__ int mad_m8_i24(int a, int c) {  // c - 8 a (|a| < 2^23)
  int r;
  asm("v_mad_i32_i24 %0, %1, -8, %2" : "=v"(r) : "v"(a), "v"(c));
  return r;
}
__device__ __forceinline__ int sgn_i32(int x) {  // med3(x, -1, 1)
  int r;
  asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ int2 step_v15_mad(int2 pos, int dx, int dy, int ax2, int ay2) {
  const int gx = (int)((uint32_t)mad_m8_i24(ax2, ay2) >> 31);  // 8 dx^2 > dy^2
  const int gy = (int)((uint32_t)mad_m8_i24(ay2, ax2) >> 31);  // 8 dy^2 > dx^2
  const int sx = gx + (((pos.x & 1) | dy) == 0 ? 1 : 0);  // (dy == 0 and x even: |step| 2)
  const int sy = gy + (((pos.y & 1) | dx) == 0 ? 1 : 0);
  return make_int2(__mul24(sgn_i32(dx), sx) + pos.x, __mul24(sgn_i32(dy), sy) + pos.y);
}
// Movement step. Arrival (|v| <= velocity) is the integer test d2 <= d2snap (sqrt is
// correctly rounded and monotone). Otherwise the new coordinate is x + rint(q) with
// q = velocity * dx / |v| (x is an integer, so rint(x + q) = x + rint(q) unless x + q is a
// tie). q is evaluated in float32 with a relative error < 5e-7 (|q| <= velocity, so the
// absolute error is < 5e-7 * max(1, velocity)); only when q lies within move_band =
// 2^-16 * max(1, velocity) (30x wider) of a half-integer -- where float32 could pick the
// other integer, or half-to-even needs the exact value -- is the exact float64 form used. Axis-parallel
// moves at a non-integer velocity (q = +-velocity exactly, often a tie) are done exactly in
// float64 (no division needed); at an integer velocity the fast path gives them.
__device__ __forceinline__ void move_ue_p(int2& pos, int2& wp, const MoveP& mp) {
  const int dx = wp.x - pos.x;
  const int dy = wp.y - pos.y;
  // |dx|, |dy| <= map size < 2^23: 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate)
  const int d2 = __mul24(dx, dx) + __mul24(dy, dy);
  if (d2 <= mp.d2snap) {  // arrived: snap to waypoint and pop it
    pos = wp;
    wp = make_int2(-1, -1);
    return;
  }
  if (mp.axis_exact == 2) {  // velocity 1.5: integers (step_v15)
    pos = step_v15(pos, dx, dy, __mul24(dx, dx), __mul24(dy, dy));
    return;
  }
  if (mp.axis_exact && (dx == 0 || dy == 0)) {
    const double q = mp.vel;
    if (dy == 0) pos.x = (int)rint((double)pos.x + (dx > 0 ? q : -q));
    else pos.y = (int)rint((double)pos.y + (dy > 0 ? q : -q));
    return;
  }
  const float sc = mp.vel_f * __builtin_amdgcn_rsqf((float)d2);  // velocity / |v|
  const float qx = (float)dx * sc;
  const float qy = (float)dy * sc;
  // clear of a tie: |q - rint(q)| < 0.5 - move_band (<=> |frac(q) - 0.5| > move_band, with the
  // rounding shared with the result; q - rint(q) is exact)
  const float rx = rintf(qx), ry = rintf(qy);
  if (fmaxf(fabsf(qx - rx), fabsf(qy - ry)) < mp.move_lim) {
    pos.x += (int)rx;
    pos.y += (int)ry;
  } else {
    pos = move_exact(pos, dx, dy, mp.vel);
  }
}

// move_ue_p with the parameters held compactly (the heterogeneous two-group rollout keeps them
// per lane for the launch): {vel_f, move_lim} and hpk = d2snap << 8 | axis_exact << 4 | class;
// the float64 velocity of the exact paths (axis moves, ties) read from `mvu` there (rare).
__device__ __forceinline__ void move_ue_pc(int2& pos, int2& wp, float vel_f, float move_lim,
                                           uint32_t hpk, const MoveP* mvu) {
  const int dx = wp.x - pos.x;
  const int dy = wp.y - pos.y;
  const int d2 = __mul24(dx, dx) + __mul24(dy, dy);
  if (d2 <= (int)(hpk >> 8)) {
    pos = wp;
    wp = make_int2(-1, -1);
    return;
  }
  const uint32_t axis = (hpk >> 4) & 3u;
  if (axis == 2u) {
    pos = step_v15(pos, dx, dy, __mul24(dx, dx), __mul24(dy, dy));
    return;
  }
  if (axis && (dx == 0 || dy == 0)) {
    const double q = mvu->vel;
    if (dy == 0) pos.x = (int)rint((double)pos.x + (dx > 0 ? q : -q));
    else pos.y = (int)rint((double)pos.y + (dy > 0 ? q : -q));
    return;
  }
  const float sc = vel_f * __builtin_amdgcn_rsqf((float)d2);
  const float qx = (float)dx * sc;
  const float qy = (float)dy * sc;
  const float rx = rintf(qx), ry = rintf(qy);
  if (fmaxf(fabsf(qx - rx), fabsf(qy - ry)) < move_lim) {
    pos.x += (int)rx;
    pos.y += (int)ry;
  } else {
    pos = move_exact(pos, dx, dy, mvu->vel);
  }
}

// The context's movement parameters (compile-time constants in a scenario instance).
template <int SCN>
constexpr bool scn_v15() { return SCN != 0 && scn_const(SCN).vel_f == 0x3fc00000u; }
// Every UE active at every step (a scenario with arrival at 0, no departure before the episode
// end, the first step active): after the lazy reset 0 <= t < t_end, so the activity test of
// base.py:288-291 is constant -- active = valid, no compares, no ballot.
template <int SCN>
constexpr bool scn_all_active() {
  return SCN != 0 && scn_const(SCN).arr_start == 0 &&
         scn_const(SCN).arr_exit >= scn_const(SCN).t_end && scn_const(SCN).first_step_active;
}

template <int SCN = 0>
__device__ __forceinline__ void move_ue(int2& pos, int2& wp, const KParams& kp) {
  if constexpr (scn_v15<SCN>()) {
    const int dx = wp.x - pos.x, dy = wp.y - pos.y;
    const int ax2 = __mul24(dx, dx), ay2 = __mul24(dy, dy);
    if (ax2 + ay2 <= 2) {  // arrived (sqrt(d2) <= 1.5): snap to the waypoint and pop it
      pos = wp;
      wp = make_int2(-1, -1);
    } else {
      pos = step_v15(pos, dx, dy, ax2, ay2);
    }
    return;
  }
  move_ue_p(pos, wp, MoveP{kp.vel, KPSF(vel_f), KPSF(move_lim), KPS(d2snap), KPS(axis_exact)});
}

// BoundedLogUtility.calculateUtility + scaleUtility (utilities.py:44-55).
__device__ __forceinline__ double scaled_utility(double rate, const KParams& kp) {
  double ur;
  if (rate <= 0.0) {
    ur = kp.lower;
  } else {
    ur = kp.w1 * log(kp.w2 + rate) / kp.log_w3;
    ur = fmin(fmax(ur, kp.lower), kp.upper);  // np.clip
  }
  return 2.0 * (ur - kp.lower) / (kp.upper - kp.lower) - 1.0;
}

// ResourceFair share of the full-rate entry and numpy round(., 2) (base.py:435): the
// reference value is cents = rint(fl(fl(full / n) * 100)), rate = cents / 100. The fast path
// forms c = full * (100 / n) (within 2^-50 relative of the exact product) and rounds it
// directly; only when c lies within 2^-46 relative of a half-integer are the two exact
// float64 operations evaluated. Returns cents (an integer-valued double).
// Rounding of c = full * (100 / n) with the tie test in float32: d = c - rint(c) is exact in
// float64 and its float32 conversion is within 2^-26, so 0.5 - |(float)d| > c 2^-46 + 2^-25
// implies c is more than c 2^-46 away from a half-integer (the old bound) -- two float64
// operations (rint, subtract) and two conversions instead of floor / fract / scale / compare in
// float64. `cf` = (float)cents, the value the obs rate and the float32 utility use.
__device__ __forceinline__ double cents_of(double c, double full, int n, float& cf) {
  const double r = rint(c);
  const float d = (float)(c - r);
  const float rf = (float)r;
  if (0.5f - fabsf(d) > __builtin_fmaf(rf, 0x1p-46f, 0x1p-25f)) {
    cf = rf;
    return r;
  }
  const double e = rint((full / (double)n) * 100.0);
  cf = (float)e;
  return e;
}

// The same with r100 = 100 / n correctly rounded (from a table: no reciprocal on the device).
__device__ __forceinline__ double share_cents_r(double full, double r100, int n, float& cf) {
  return cents_of(full * r100, full, n, cf);
}

__device__ __forceinline__ double share_cents(double full, int n, float& cf) {
  // 100 / n to within 2 ulp: hardware reciprocal + two Newton steps (no table, no division)
  const double dn = (double)n;
  double r = __builtin_amdgcn_rcp(dn);
  r = fma(r, fma(-dn, r, 1.0), r);
  r = fma(r, fma(-dn, r, 1.0), r);
  return cents_of(full * (100.0 * r), full, n, cf);
}

// Scaled utility of a rounded rate. The utility depends on the rate only, and the rate is
// cents/100 for an integer `cents`, so below the saturation point (rate where the clip at
// `upper` engages) it is read from a table the device built with scaled_utility() itself
// (identical values); above it, it is the scaled upper bound.
__device__ __forceinline__ double utility_of(double rate, double cents, const KParams& kp,
                                             const double* __restrict__ tab) {
  if (kp.util_direct) return scaled_utility(rate, kp);
  if (cents <= (double)kp.util_kmax) return tab[(int)cents];
  return kp.util_sat;
}

constexpr int kPackedBlock = 256;
constexpr int kWavesPerBlock = kPackedBlock / 64;
// fused launches with the LDS association tables: 8-wave workgroups, two per CU (one LDS copy
// of the <= ~65 KB tables per 8 waves; LDS-limited to 4 waves per SIMD). Measured at 65,536
// mobile-large envs (us per rollout step): 8 waves 15.7; 12 waves with <= 80 VGPRs (6 per
// SIMD) 16.5 -- 6,144 resident waves do not divide the 32,768 env groups, and the extra
// occupancy bought little; 10 waves 18.2 (two workgroups do not fit beside each other).
#ifndef MEV_LDS_WAVES
#define MEV_LDS_WAVES 8
#endif
constexpr int kLdsWaves = MEV_LDS_WAVES;
// the two-read tables (LDSM 2: + a 2-byte rank per cell, ~141 KB for 200 x 200) take one
// 16-wave workgroup per CU, the whole LDS
#ifndef MEV_LDS2_WAVES
#define MEV_LDS2_WAVES 16
#endif
constexpr int kLds2Waves = MEV_LDS2_WAVES;
constexpr int kLds2BytesPerWG = 160 * 1024;
constexpr int kLds2Window = 3;  // staged rows per window of the two-group rollout (see its launch)
constexpr int kStage2Bytes = 8;  // bytes per env of a k_steps_lds2 staged row: {isum, nact | done << 7}
__host__ __device__ constexpr int lds_waves(int ldsm) {
  return ldsm >= 2 ? kLds2Waves : ldsm == 1 ? kLdsWaves : 4;
}
constexpr int kLdsBytesPerWG = 80 * 1024;


// Sum of `v` over the lanes of one env segment that have `take` set (segment = lanes
// base..base+U-1, u = lane - base): a shift-down tree in float64 with partners restricted to
// the segment; the result is valid in lane `base`. (numpy's np.mean sums in pairwise order;
// the two float64 sums differ by a few ulps at most, far below the float32 output.)
__device__ __forceinline__ double seg_sum(double v, bool take, int U, int u) {
  double x = take ? v : 0.0;
  for (int off = 1; off < U; off <<= 1) {
    const double y = __shfl_down(x, (unsigned)off);
    if (u + off < U) x += y;
  }
  return x;
}

// Inclusive prefix sum within each 16-lane DPP row (all lanes active).
__device__ __forceinline__ int row_scan_i32(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  return x;
}

// float64 DPP move (both halves), invalid source lanes / masked rows read 0.0
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWMASK, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWMASK, 0xf, true);
  return __hiloint2double(hi, lo);
}

// Sum of `v` over the lanes of an aligned segment of P = 16 or 32 lanes with `take` set
// (all 64 lanes must be active): row prefix sums by row_shr 1/2/4/8, then (P = 32) the lower
// row's total added into the upper row by row_bcast15. The result is valid in the segment's
// last lane (u = P - 1).
template <int P>
__device__ __forceinline__ double seg_sum_rows(double v, bool take) {
  double x = take ? v : 0.0;
  x += dpp_f64<0x111>(x);  // row_shr:1
  x += dpp_f64<0x112>(x);  // row_shr:2
  x += dpp_f64<0x114>(x);  // row_shr:4
  x += dpp_f64<0x118>(x);  // row_shr:8
  if (P == 32) x += dpp_f64<0x142, 0xa>(x);  // row_bcast:15 into rows 1 and 3
  return x;
}

// int32 sum over an aligned segment of P = 16 or 32 lanes (all 64 lanes active), valid in the
// segment's last lane; DPP-modified adds (row_shr 1/2/4/8, then row_bcast:15 for P = 32)
template <int P>
__device__ __forceinline__ int seg_isum_rows(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  if (P == 32) x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, true);
  return x;
}

// ---- Reward exactness guard --------------------------------------------------------------------
// north_star holds the float32 reward to 1e-5 relative of the reference's float64 mean utility
// (metrics.py:25-28). The lean kernels sum float32 utilities, each within kp.u_err of the
// float64 value (the host's bound for the utility parameters), as fixed point (quantum q per
// UE); that mean is within 1e-5 unless the sum is small against its error bound --
// nact (u_err + q) >= 9.5e-6 |sum|, tested as |mean| <= kp.r_thr or |isum| <= nact kp.r_thr25
// (host-computed: one compare where the sum is formed): mean utilities near zero, cancellation
// (none in the registered large / medium / mixed workloads; ~1 % of small's env-steps). Such an
// env's reward comes from the exact float64 utilities (the device table tb.util by rounded rate,
// the non-lean kernels' values) summed as 2^-50 fixed point in int64: associative, so every
// kernel shape forms the same bits.
// The rare path's constants are held in LDS where a kernel's scalar registers are scarce:
// {utility table, util_sat, util_kmax, u_err | r_thr25} as four 8-byte slots -- the r100 table's
// slots 66..69 of the LDS blobs (kRewardCSlot), or a static array of the block kernel (kernel
// arguments used there were kept in SGPRs across the step loops and spilled others to VGPR
// lanes: +9 % at 4,096 medium envs).
constexpr int kRewardCSlot = 66;
struct RewardC {
  const double* tab;
  double sat;
  double kmax;
  float u_err;
  int thr25;  // KParams::r_thr25
};
__device__ __forceinline__ RewardC reward_c(const char* p) {  // (p: 8-byte aligned LDS)
  RewardC c;
  c.tab = *reinterpret_cast<const double* const*>(p);
  c.sat = *reinterpret_cast<const double*>(p + 8);
  c.kmax = *reinterpret_cast<const double*>(p + 16);
  c.u_err = *reinterpret_cast<const float*>(p + 24);
  c.thr25 = *reinterpret_cast<const int*>(p + 28);
  return c;
}
__device__ __forceinline__ long long util_fix50c(double cents, const RewardC& c) {
  const double uu = cents <= c.kmax ? c.tab[(int)cents] : c.sat;
  return (long long)(uu * 0x1p50);
}
__device__ __forceinline__ float exact_mean50(long long s, int nact) {
  return (float)((double)s * 0x1p-50 / (double)nact);
}
// The guard's rare work out of line: one copy of the code, whose scalars then do not compete
// with the step loops' (inlined into a loop, they kept kernel arguments live across it and
// spilled others to VGPR lanes).
// (default; -DMEV_GUARD_INLINE for the A/B: at 4,096 medium envs 92.8 vs 99.4 us per 200-step
// launch, interleaved on one box)
#ifndef MEV_GUARD_INLINE
#define MEV_GUARD_FN __device__ __attribute__((noinline))
#else
#define MEV_GUARD_FN __device__ __forceinline__
#endif
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ long long dpp_i64(long long v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(unsigned long long)v, CTRL, ROWMASK, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((unsigned long long)v >> 32), CTRL,
                                             ROWMASK, 0xf, true);
  return (long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
// int64 sum over an aligned segment of P = 16 / 32 / 64 lanes (all lanes active), valid in the
// segment's last lane (seg_sum_rows' pattern; P = 64: + row_bcast:31 into rows 2 and 3)
template <int P>
__device__ __forceinline__ long long seg_lsum_rows(long long x) {
  x += dpp_i64<0x111>(x);
  x += dpp_i64<0x112>(x);
  x += dpp_i64<0x114>(x);
  x += dpp_i64<0x118>(x);
  if (P >= 32) x += dpp_i64<0x142, 0xa>(x);
  if (P == 64) x += dpp_i64<0x143, 0xc>(x);
  return x;
}
// ... over U consecutive lanes (seg_sum's pattern), valid in the segment's first lane
__device__ __forceinline__ long long seg_lsum(long long x, int U, int u) {
  for (int off = 1; off < U; off <<= 1) {
    const long long y = __shfl_down(x, (unsigned)off);
    if (u + off < U) x += y;
  }
  return x;
}

// ResourceFair's n_b without LDS for 16-lane segments (P = 16: one DPP row per env) with at
// most 15 UEs and 8 stations: every lane adds 1 << 4 srv into a row-wide sum (butterfly over
// row_ror 8 / 4 / 2 / 1: the total in every lane of the row), i.e. 8 packed 4-bit counts, and
// reads its own station's field. No LDS round trips (zero, atomic add, read back) on the step's
// dependency chain -- which is what bounds a wave alone on its SIMD (small batches).
__host__ __device__ constexpr bool packed_counts_ok(int UC, int B) {
  return UC >= 1 && UC <= 15 && B >= 1 && B <= 8;
}
__device__ __forceinline__ int row_count_same(int srv) {
  int v = srv >= 0 ? 1 << (4 * srv) : 0;
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x122, 0xf, 0xf, false);  // row_ror:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x121, 0xf, 0xf, false);  // row_ror:1
  return srv >= 0 ? (int)__builtin_amdgcn_ubfe((uint32_t)v, (uint32_t)(4 * srv), 4u) : 0;
}

// Float32 form of the scaled BoundedLogUtility (used when no float64 utility output is
// requested): clip(w1 log(w2 + r) / log(w3), lower, upper) with log via v_log_f32, then the
// affine scale to [-1, 1]; r = (float)cents * 0.01f is the obs rate. Relative error ~1e-7 of
// the float64 value.
template <int SCN = 0>
__device__ __forceinline__ double utility_f32r(float cents, float r, const KParams& kp) {
  if (cents <= 0.f) return -1.0;  // rate <= 0 -> lower -> scaled -1
  // a scenario's zero w2 / offset is not added (r > 0 and ur * scale != -0: the same bits)
  constexpr bool no_w2 = SCN && scn_const(SCN).u_w2f == 0u;
  constexpr bool no_off = SCN && scn_const(SCN).u_offset == 0u;
  float ur = KPSF(u_log2_coef) * __log2f(no_w2 ? r : KPSF(u_w2f) + r);
  ur = __builtin_amdgcn_fmed3f(ur, KPSF(u_lowerf), KPSF(u_upperf));  // np.clip (ur is not NaN)
  return (double)(no_off ? ur * KPSF(u_scale) : ur * KPSF(u_scale) + KPSF(u_offset));
}

// ------------------------------------------------------------------------------------
// Packed shape: U <= 64, G = floor(64/U) envs per wavefront, one lane per UE.
// ------------------------------------------------------------------------------------
// An env occupies a segment of P >= U consecutive lanes (the segment pitch): lanes
// base .. base+U-1 hold its UEs, base+U .. base+P-1 are padding. P = U, or the next power of
// two where that costs no envs per wavefront (U = 15 -> 16, U = 30 -> 32): then segments are
// whole DPP rows / row pairs and per-env sums need no cross-row shuffles.
struct LaneMap {
  int seg, u, base;
  uint64_t segmask, lt;
};

// k_steps_lds2's compile-time U may carry kSeg32: UC = kSeg32 + U puts U <= 16 UEs in 32-lane
// segments (two envs per wavefront instead of four: twice the wavefronts for a small batch)
constexpr int kSeg32 = 1000;
__host__ __device__ constexpr int ue_of(int UC) { return UC >= kSeg32 ? UC - kSeg32 : UC; }
__host__ __device__ constexpr int pitch_of(int U) {
  return U >= kSeg32 ? 32
         : (U > 8 && U <= 16 && 64 / 16 == 64 / U) ? 16
         : (U > 16 && U <= 32 && 64 / 32 == 64 / U) ? 32 : U;
}

template <int PC>
__device__ __forceinline__ LaneMap lane_map(int lane, int P) {
  LaneMap m;
  if (PC == 16 || PC == 32) {
    m.seg = lane / PC;
  } else {
    // lane / P through float: (lane + 0.5) / P is >= 0.5/P away from an integer
    m.seg = (int)(((float)lane + 0.5f) * (1.0f / (float)P));
  }
  m.u = lane - m.seg * P;
  m.base = m.seg * P;
  m.segmask = (P >= 64) ? ~0ull : (((1ull << P) - 1ull) << m.base);
  m.lt = (1ull << lane) - 1ull;
  return m;
}

// The env's bits of a wavefront ballot, at bit 0, for aligned segments (P = 16 or 32): one
// 32-bit half of the ballot (a select between two scalar halves) or a 16-bit field of it --
// cheaper than masking the 64-bit ballot with the lane's segment mask.
template <int PC>
__device__ __forceinline__ uint32_t seg_field(uint64_t b, const LaneMap& m) {
  const uint32_t half = (m.base & 32) ? (uint32_t)(b >> 32) : (uint32_t)b;
  return PC == 32 ? half : __builtin_amdgcn_ubfe(half, (uint32_t)(m.base & 16), 16u);
}

// Per-lane inputs of one env group. The loads are unconditional (env index clamped to a
// valid env): a guarded load would make the compiler wait for it at the merge point.
struct GroupIn {
  int t;
  int drawn;           // draw-table mode: pairs of the episode consumed so far
  bool s_ok;           // fused + draw table: pa holds the state after pair drawn - 1
  int4 s;              // {x, y, wx, wy}
  ulonglong2 pa, pb;   // PCG64 state, increment of the env's movement stream
  double r100l;        // (one-step TF instances) 100 / lane, correctly rounded: the lane's entry
                       // of the host's table, read by the lanes through ds_bpermute
};

template <int SCN = 0>
__device__ __forceinline__ GroupIn load_group(const KParams& kp, const KState& st,
                                              const KTables& tb, int e, int u, int U,
                                              bool fused) {
  const int ec = min(e, kp.E - 1);
  GroupIn g;
  const uint32_t ue = (uint32_t)(ec * U + u);
  g.r100l = 0.0;
  g.t = at(st.t, 4u * (uint32_t)ec);
  g.s = load_ue_at(st.ue_state, ue, KST8);
  if (fused || kp.tab_m) {  // the stream state is read only where a draw needs it (fused:
    g.drawn = kp.tab_m ? at(tb.drawn, 4u * (uint32_t)ec) : 0;  // the caller's LDS slot)
    // the state row is the stream state without a table, or after draws past it
    g.s_ok = !kp.tab_m || g.drawn > kp.tab_m;
    g.pa = g.pb = make_ulonglong2(0, 0);
  } else {
    ulonglong2* pr = reinterpret_cast<ulonglong2*>(st.pcg);
    g.drawn = kp.tab_m ? at(tb.drawn, 4u * (uint32_t)ec) : 0;
    g.s_ok = true;
    g.pa = at(pr, 48u * (uint32_t)ec);
    g.pb = at(pr, 48u * (uint32_t)ec + 16u);
  }
  return g;
}

// Reset kernel: MComCore.reset (base.py:172-209) for envs with mask[e] != 0 (all if NULL):
// movement RNG re-seeded (movement.py:16-18), initial positions in ue_id order, 2 draws per
// UE (movement.py:64-72), waypoints cleared, t = 0.
__global__ __launch_bounds__(kPackedBlock) void k_reset_packed(KParams kp, KState st, KOut out,
                                                              KTables tb,
                                                              const uint8_t* __restrict__ mask) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const LaneMap m = lane_map<0>(lane, kp.U);
  const int e = wave * kp.envs_per_wave + m.seg;
  if (m.seg >= kp.envs_per_wave || e >= kp.E) return;
  if (mask != nullptr && !mask[e]) return;
  const ulonglong2* pr = reinterpret_cast<const ulonglong2*>(st.pcg + (size_t)6 * e);
  const ulonglong2 pa = pr[0], pb = pr[1], pc = pr[2];
  const u128 inc = mk128(pb.x, pb.y);
  const u128 s0 = kp.movement_reseed ? mk128(pc.x, pc.y) : mk128(pa.x, pa.y);
  int x, y;
  const u128 s_fin = pcg_draw_pair(s0, inc, 2 * m.u, tb.jump, kp.Wd, kp.Hd, x, y);
  const size_t idx = (size_t)e * kp.U + m.u;
  store_ue_at(st.ue_state, (uint32_t)idx, make_int2(x, y), make_int2(-1, -1), kp.st8 != 0);
  out.serving[idx] = -1;
  out.obs[idx] = make_float4((float)x * kp.inv_w, (float)y * kp.inv_h, 0.f, 0.f);
  if (out.rate64) out.rate64[idx] = 0.0;
  if (out.util64) out.util64[idx] = 0.0;
  if (m.u == kp.U - 1)  // the state after the env's 2U initial draws
    *reinterpret_cast<ulonglong2*>(st.pcg + (size_t)6 * e) =
        make_ulonglong2((uint64_t)s_fin, (uint64_t)(s_fin >> 64));
  if (m.u == 0) {
    if (kp.tab_m) tb.drawn[e] = kp.U;  // the U initial pairs of the episode
    st.t[e] = 0;
    out.reward[e] = 0.f;
    out.done[e] = 0;
    if (out.metrics) out.metrics[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Outputs of one fused step held back until the next step's association gather is issued
// (k_steps_packed): the global stores of step i then come after that load in program order,
// so waiting for the gather (vmcnt counts loads and stores in issue order) does not also wait
// for step i's stores to be acknowledged -- with trajectory rows every store allocates a new
// L2 line and that wait is long.
struct Pending {
  int srv;
  float4 obs;
  double rate, util;
  float reward;
  float4 met;
  uint32_t ui;
  int e;
  bool valid, lead, done;
};

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));

// s_waitcnt vmcnt(0) only (gfx9 encoding: expcnt 7, lgkmcnt 15 = no wait on those)
__device__ __forceinline__ void wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// int16x2 view of a 32-bit word by explicit halves. (__builtin_bit_cast(s16x2, v.z) of an element
// of a 4 x u32 ext_vector_type load is miscompiled by this LLVM (ROCm 7.2, gfx950): the dot
// products of both halves of a ds_read_b128 read kv.x -- checked in the generated assembly.)
__device__ __forceinline__ s16x2 as_s16x2(unsigned v) {
  s16x2 r;
  r.x = (short)(v & 0xffffu);
  r.y = (short)(v >> 16);
  return r;
}

// Lane mask of a bool: the ballot builtin on the i1 itself (HIP's __ballot takes an int, and
// the compiler then materialises compound conditions as v_cndmask + v_cmp before the ballot)
__device__ __forceinline__ uint64_t bal(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// LDS-DMA: this lane's element `src` to lds_base + lane * sizeof(T) (lds_base wave-uniform);
// complete after vmcnt(0)
typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
__device__ __forceinline__ void glds(const int* src, int* lds_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_base, 4, 0, 0);
}
__device__ __forceinline__ void glds(const int4* src, int4* lds_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_base, 16, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// The stores of a Pending step into row `row` of the output buffers (row 0 when the outputs
// are overwritten every step), branch-free: raw buffer stores through one descriptor per row
// (its base moves with the row, so a trajectory of any length needs no 32-bit offset range),
// whose lanes without data (padding lanes; non-leaders for the per-env rows) take the offset
// one past the row's end, which the buffer range check drops. Without branches every path
// issues the same VMEM ops, so the compiler's wait for the next gather can leave these stores
// in flight. The scalar offset stays the constant 0: with an SGPR soffset LLVM omits the wait
// state between a > 8-byte buffer store and a VALU write of its data registers, and on gfx950
// that write then corrupts the stored data (seen as other values in a few obs rows;
// tools/check_store_hazard.py checks the generated assembly for such stores).
// Cache policy of the per-UE trajectory stores (dev A/B knob: 0 default, 2 nt, 16 sc1)
#ifndef MEV_TRAJ_AUX
#define MEV_TRAJ_AUX 0
#endif
template <bool LEAN, bool SMALL = true>
__device__ __forceinline__ void flush_pending(const KOut& out, const Pending& p, uint32_t E,
                                              uint32_t EU, uint32_t row) {
  const uint32_t robs = 16u * EU, rsrv = 4u * EU, rrew = 4u * E;  // row bytes
  const v4u32 ob = {__float_as_uint(p.obs.x), __float_as_uint(p.obs.y),
                    __float_as_uint(p.obs.z), __float_as_uint(p.obs.w)};
  const size_t ru = (size_t)row * EU, re = (size_t)row * E;
  __builtin_amdgcn_raw_buffer_store_b32((uint32_t)p.srv, out_rsrc(out.serving + ru, rsrv),
                                        p.valid ? 4u * p.ui : rsrv, 0, MEV_TRAJ_AUX);
  __builtin_amdgcn_raw_buffer_store_b128(ob, out_rsrc(out.obs + ru, robs),
                                         p.valid ? 16u * p.ui : robs, 0, MEV_TRAJ_AUX);
  if (SMALL) {  // (else staged in LDS by the caller: k_steps_packed, STG)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(p.reward), out_rsrc(out.reward + re, rrew),
                                          p.lead ? 4u * (uint32_t)p.e : rrew, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)p.done, out_rsrc(out.done + re, E),
                                         p.lead ? (uint32_t)p.e : E, 0, 0);
  }
  if (!LEAN) {
    const KOut o = out_row(out, (int)E, (int)(EU / E), (int)row);
    if (p.valid) {
      if (o.rate64) o.rate64[p.ui] = p.rate;
      if (o.util64) o.util64[p.ui] = p.util;
    }
    if (p.lead && o.metrics) o.metrics[p.e] = p.met;
  }
}


// One env group (floor(64/U) envs, one lane per UE) of the packed step kernel.
//   UC:   U as a compile-time constant (0: runtime kp.U) -- folds the lane map, the segment
//         reductions and the env indexing for the registered scenario sizes;
//   LEAN: no float64 rate / utility / metrics outputs and the utility in its float32 form
//         (the Gym surface's default), so none of the optional work is even branched over.
//   FUSED: one of several steps of a launch (mev_step(n), n > 1): the env state stays in
//         registers between the steps (`cur` is updated; the caller stores it after the last
//         step), the per-step outputs are written every step as in separate launches.
//   FUSED steps write row `row` of the output rows (`out` is the base, row 0); without
//   LDSA they defer their stores (Pending): `pend` holds the previous step's outputs (for row
//   row - 1; nothing valid before the first step) and receives this step's.
//   LDSM: (fused, shared layout) association from the LDS copy of the compact tables at
//         `lblob` (KTables::lds_blob) instead of the L2 gather: 1 = station map + rank index
//         (four dependent reads), 2 = station map + per-cell rank map (two parallel reads and
//         the rate).
// packed_group's rare exact mean (wave-wide; valid in the env's leader lane): cents < 0 for a
// lane that does not count
template <bool ROWS, int PC>
MEV_GUARD_FN float packed_fix(double cents, int U, int u, const double* tab, double kmax,
                              double sat, int nact) {
  const long long v = cents < 0.0 ? 0 : util_fix50c(cents, RewardC{tab, sat, kmax, 0.f, 0});
  const long long se = ROWS ? seg_lsum_rows<PC>(v) : seg_lsum(v, U, u);
  return exact_mean50(se, nact);
}

template <bool PER_ENV_BS, bool LEAN, int UC, bool FUSED, int LDSM = 0, int SCN = 0,
          bool STG = false, bool TF = false>
__device__ __forceinline__ bool packed_group(const KParams& kp, const KState& st,
                                             const KOut& out, const KTables& tb,
                                             const LaneMap& m, GroupIn& cur, int e,
                                             bool env_ok, int* __restrict__ hist,
                                             const int* __restrict__ ltab = nullptr,
                                             Pending* pend = nullptr, int row = 0,
                                             const char* __restrict__ lblob = nullptr,
                                             u128* __restrict__ lpcg = nullptr,
                                             float* __restrict__ srew = nullptr,
                                             uint8_t* __restrict__ sdone = nullptr,
                                             uint64_t envok_wf = 0, uint64_t valid_wf = 0,
                                             const int* __restrict__ lbs = nullptr,
                                             int nb_f = 0) {
  constexpr int PC = UC ? pitch_of(UC) : 0;
  constexpr bool ROWS = PC == 16 || PC == 32;  // aligned segments (DPP row reductions)
  constexpr bool LDSA = LDSM != 0;
  const int U = UC ? UC : kp.U;
  const int P = PC ? PC : kp.U;
  const int u = m.u;
  const bool valid = env_ok && u < U;             // a lane holding a UE
  const bool leader = ROWS ? u == P - 1 : u == 0;  // the lane of the per-env stores
  const uint64_t segmask = m.segmask, lt = m.lt;
  const bool want_metrics = !LEAN && out.metrics != nullptr;
  const bool want_qoe = !LEAN && out.qoe_stats != nullptr;
  const bool exact_util =
      !LEAN && (out.util64 != nullptr || kp.util_direct || kp.util_exact || want_qoe);
  const bool want_rate = !LEAN && (out.rate64 != nullptr || want_metrics || exact_util);
  const size_t idx = (size_t)e * U + u;
  int t = cur.t;
  int2 pos = make_int2(cur.s.x, cur.s.y);
  int2 wp = make_int2(cur.s.z, cur.s.w);
  // fused: the env's stream {state, increment} lives in the wavefront's LDS slot lpcg[seg]
  // (read only where a draw needs it, written by the owner of a new state), not in registers
  u128* const slot = FUSED ? lpcg + 2 * m.seg : nullptr;
  u128 inc = FUSED ? (u128)0 : mk128(cur.pb.x, cur.pb.y);
  u128 s = FUSED ? (u128)0 : mk128(cur.pa.x, cur.pa.y);
  const int M = KPS(tab_m);  // wave-uniform
  int drawn = cur.drawn;
  bool s_ok = cur.s_ok;
  // heterogeneous entities (shared layout, L2 association maps only): this UE's class selects
  // its movement parameters and its class's association map (wave-uniform flag)
  constexpr bool HETOK = !LDSA && SCN == 0 && !PER_ENV_BS;
  const bool het = HETOK && kp.het;
  const int cu = het ? (int)tb.ue_cls[min(u, U - 1)] : 0;

  // Stream bookkeeping without cross-lane moves: the step's waypoint draws start at offset
  // koff of stream state `s` (koff = 2U right after a reset: the initial positions took the
  // first 2U draws), and the lane that made the env's LAST draw of the step writes the new
  // stream state back.
  int koff = 0;
  u128 s_fin = s;  // stream state after this lane's last draw

  // ---- lazy auto-reset at the start of the step after the episode ended ---------------
  // (wave masks: the ballot of one compare, ANDed in SALU with a loop-invariant mask -- the
  // ballot of a compound condition costs a v_cndmask + v_cmp)
  // (fused: the caller's, from before its step loop -- ballots are not hoisted out of it)
  const uint64_t envok_w = FUSED ? envok_wf : bal(env_ok);
  const uint64_t valid_w = FUSED ? valid_wf : bal(valid);
  const bool reset_env = env_ok && t >= KPS(t_end);  // every lane of the env, padding too
  const bool do_reset = reset_env && valid;
  if (bal(t >= KPS(t_end)) & envok_w) {
    if (reset_env) t = 0;
    if (M) {  // initial positions = the episode's first U pairs (draw table)
      if (reset_env) drawn = U;
      if (do_reset) {
        const uint32_t row = (uint32_t)e * (uint32_t)M;
        const int p = FUSED ? ltab[m.seg * M + u]
                            : at(const_cast<int*>(tb.tab_xy), 4u * (row + (uint32_t)u));
        pos = make_int2((int)(short)p, p >> 16);
        wp = make_int2(-1, -1);
      }
    } else if (do_reset) {  // MComCore.reset (base.py:172-209), see k_reset_packed
      const ulonglong2 pc = at(reinterpret_cast<ulonglong2*>(st.pcg), 48u * (uint32_t)e + 32u);
      if (FUSED) {
        inc = slot[1];
        if (!kp.movement_reseed) s = slot[0];
      }
      if (kp.movement_reseed) s = mk128(pc.x, pc.y);
      s_fin = pcg_draw_pair(s, inc, 2 * u, tb.jump, kp.Wd, kp.Hd, pos.x, pos.y);
      koff = 2 * U;
      wp = make_int2(-1, -1);
      if (FUSED) wait_vmem();  // in the loads' own block (see the fallback path below)
    }
  }

  // activeUsers during step t: startTime <= t < exitTime (base.py:288-291, custom.py:53-54)
  const bool active = valid && (scn_all_active<SCN>() ||
                                (t >= KPS(arr_start) && t < KPS(arr_exit) &&
                                 (KPS(first_step_active) || t != 0)));

  // ---- 1. movement: lazy waypoint draws in ue_id order (movement.py:44-47) ------------
  const uint64_t act_w =
      scn_all_active<SCN>()
          ? valid_w
          : bal(t >= KPS(arr_start) && t < KPS(arr_exit) && (KPS(first_step_active) || t != 0)) &
                valid_w;
  const bool nowp = wp.x == -1;  // (no waypoint: see lds2_step)
  const bool need = active && nowp;
  const uint64_t mneed_w = bal(nowp) & act_w;
  int tot, rank;  // draws of this env this step (2 per waypoint); this lane's rank among them
  if constexpr (ROWS) {
    const uint32_t f = seg_field<PC>(mneed_w, m);
    tot = __popc(f);
    rank = __popc(__builtin_amdgcn_ubfe(f, 0u, (uint32_t)u));
  } else {
    tot = __popcll(mneed_w & segmask);
    rank = __popcll(mneed_w & segmask & lt);
  }
  bool fell_back = false;  // wave-uniform: this step's draws came from the stream state
  if (mneed_w) {
    const int k = drawn + rank;  // this draw's pair index in the episode
    if (M && (bal(k >= M) & mneed_w) == 0) {
      // draw table: every drawing lane of the wavefront finds its pair precomputed (fused
      // launches read the wavefront's copy in LDS and track only `drawn`)
      // (the stream state is not written back: with the table it is the entry of pair
      // drawn - 1 -- see mev.h, mev_state.pcg)
      if (need) {
        const uint32_t row = (uint32_t)e * (uint32_t)M;
        const int p = FUSED ? ltab[m.seg * M + k]
                            : at(const_cast<int*>(tb.tab_xy), 4u * (row + (uint32_t)k));
        wp = make_int2((int)(short)p, p >> 16);
      }
    } else {
      fell_back = true;
      if (M) {  // beyond the table: from the stream state
        if (!FUSED) {  // loaded only on this path: the state row holds the stream state only
          // after draws past the table (drawn > M); before, the table's entry of pair drawn - 1
          ulonglong2* pr = reinterpret_cast<ulonglong2*>(st.pcg);
          const ulonglong2 pb = at(pr, 48u * (uint32_t)e + 16u);
          inc = mk128(pb.x, pb.y);
          if (drawn > 0 && drawn <= M) {
            s = at(const_cast<u128*>(tb.tab_st), 16u * ((uint32_t)e * (uint32_t)M + (uint32_t)(drawn - 1)));
          } else {
            const ulonglong2 pa = at(pr, 48u * (uint32_t)e);
            s = mk128(pa.x, pa.y);
          }
        } else {  // fused: the slot holds the state after a fallback draw, else the table
          inc = slot[1];
          if (!s_ok && drawn > 0) {
            s = at(const_cast<u128*>(tb.tab_st),
                   16u * ((uint32_t)e * (uint32_t)M + (uint32_t)(min(drawn, M) - 1)));
            wait_vmem();  // in the load's own block (see the wait below)
          } else {
            s = slot[0];
          }
        }
        if (reset_env) {  // the state after this episode's U initial pairs
          const u128 su = at(const_cast<u128*>(tb.tab_st),
                             16u * ((uint32_t)e * (uint32_t)M + (uint32_t)(U - 1)));
          s = su;
          if (FUSED) wait_vmem();
        }
      } else if (FUSED) {  // no table: the slot (after a reset this step: the reset's state)
        inc = slot[1];
        if (!do_reset) s = slot[0];
      }
      // common case: every drawing lane of the wave is the first of its env and no reset
      // came before -> two steps of the constant multiplier instead of a table jump
      if ((bal((rank | koff) != 0) & mneed_w) == 0) {
        if (need) s_fin = pcg_draw_pair_next(s, inc, kp.Wd, kp.Hd, wp.x, wp.y);
      } else {
        if (need)
          s_fin = pcg_draw_pair(s, inc, koff + 2 * rank, tb.jump, kp.Wd, kp.Hd, wp.x, wp.y);
      }
      // fused: the loads of this rare path land here, so the compiler's merged wait state
      // after it has nothing pending from them (it would otherwise wait, on the common path
      // too, for every store still in flight)
      if (FUSED) wait_vmem();
    }
  }
  // owner of the env's new stream state: the last drawing lane, else (reset without draws)
  // the last UE's lane, else nobody (the stream did not move)
  const bool own_fin = (need && rank == tot - 1) || (do_reset && tot == 0 && u == U - 1);
  if (FUSED) {
    if ((!M || fell_back) && own_fin) slot[0] = s_fin;  // the env's new stream state
    if (M) {  // with the table, the slot holds the state only after a fallback draw
      if (fell_back && tot > 0) s_ok = true;
      else if (tot > 0 || reset_env) s_ok = false;
    }
  }
  if (active) {
    if (het) move_ue_p(pos, wp, tb.mv[min(u, U - 1)]);
    else move_ue<SCN>(pos, wp, kp);
  }

  // ---- 2. association: closest BS with snr > snr_tr <=> d2 <= d2max (base.py:236-241)
  int srv = -1;
  double full = 0.0;
  if (PER_ENV_BS) {
    // per-env layout: key = (d2 << 10) | j, min over the env's stations (ties keep the lower
    // index, as python's min() over the station dict)
    unsigned best = UINT_MAX;
    const s16x2 pu = {(short)pos.x, (short)pos.y};
    const bool staged = FUSED && (SCN ? 0 : kp.lbs) != 0;  // (uniform)
    const int nb = staged ? nb_f : st.bs_count ? (valid ? st.bs_count[e] : 0) : KPS(B);
    const int2* bs = st.bs_xy + (size_t)e * KPS(B);
    int d2s;
    if (staged) {
      // the env's station keys from its LDS slots (staged once per launch, two stations per
      // ds_read_b128): one v_dot2 per station and a v_min3 per two, branch-free over 8 or 16
      // slots (the never-winning padding keys fill the rest)
      (void)nb;
      const s16x2 p2 = {(short)(pos.x << 1), (short)(pos.y << 1)};
      const v4u32* sv = reinterpret_cast<const v4u32*>(lbs + m.seg * 32);
      auto scan = [&](auto npair) {
#pragma unroll
        for (int q = 0; q < decltype(npair)::value; ++q) {
          const v4u32 w = sv[q];
          const unsigned k0 = (unsigned)__builtin_amdgcn_sdot2(p2, as_s16x2(w.x), (int)w.y, false);
          const unsigned k1 = (unsigned)__builtin_amdgcn_sdot2(p2, as_s16x2(w.z), (int)w.w, false);
          best = min(best, min(k0, k1));
        }
      };
      if (KPS(B) <= 8) scan(std::integral_constant<int, 4>());
      else scan(std::integral_constant<int, 8>());
      if (!active) best = UINT_MAX;
      d2s = (int)(best >> 4) - (1 << 21) + __mul24(pos.x, pos.x) + __mul24(pos.y, pos.y);
      if (best != UINT_MAX && d2s <= kp.d2max) srv = (int)(best & 15u);
    } else if (active && nb > 0) {
      const int nb8 = (KPS(B) + 7) & ~7;  // wave-uniform trip count; j clamped to the last
      for (int b0 = 0; b0 < nb8; b0 += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int j = min(b0 + k, nb - 1);
          const int2 p = bs[j];
          const s16x2 d = pu - s16x2{(short)p.x, (short)p.y};  // coordinates < 1024
          const unsigned d2 = (unsigned)__builtin_amdgcn_sdot2(d, d, 0, false);
          best = min(best, (d2 << kKeyBits) | (unsigned)j);
        }
      }
    }
    if (!staged) {
      d2s = (int)(best >> kKeyBits);
      if (best != UINT_MAX && d2s <= kp.d2max) srv = (int)(best & ((1u << kKeyBits) - 1));
    }
    // full-rate entry of the serving pair (index clamped: lanes without a server read a
    // valid entry)
    full = tb.rate_full[max(0, min(d2s, kp.d2max))];
  } else {
    // shared layout: the association map holds, for every grid position of the map, the
    // serving station (or -1) and the full rate of that pair -- one 16-byte gather from an
    // L2-resident table replaces the per-station loop and the rate-table read
    if (LDSA) {
      // the same association from LDS: station of the cell (4 bits), d2 to it, and the full
      // rate at the rank of d2 in the set of sums of two squares (KTables::lds_blob). UE
      // positions stay on the map (uniform draws in [0, W) x [0, H), moves toward waypoints
      // there), so the cell index is only bounded, not clamped per coordinate
      const uint32_t cell = min((uint32_t)(__mul24(pos.y, KPS(W)) + pos.x), (uint32_t)(KPS(W) * KPS(H) - 1));
      const uint32_t nib = LDSM == 3 ? 0u :
          ((uint32_t)*reinterpret_cast<const uint8_t*>(lblob + (cell >> 1)) >> ((cell & 1u) << 2)) &
          15u;
      if (LDSM == 3) {
        // one u16 per cell: {station, rank of d2 in the layout's set D}, then the rate (read
        // for every lane: entries without a station index a valid slot)
        const uint32_t ent = *reinterpret_cast<const uint16_t*>(lblob + 2u * cell);
        const double fr = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * (ent & 4095u));
        if (active && ent < 0xF000u) {
          srv = (int)(ent >> 12);
          full = fr;
        }
        if (bal(ent == 0xFFFFu) & act_w) {  // cells whose rank lies beyond the table: L2 map
          if (active && ent == 0xFFFFu) {
            const int4 r = at(const_cast<int4*>(tb.assoc), 16u * cell);
            srv = r.x;
            full = __hiloint2double(r.w, r.z);
          }
          wait_vmem();  // in the load's own block (see the fallback draws)
        }
      } else if (LDSM == 2) {  // rank of the cell's d2 from the per-cell map, read beside the nibble
        const uint32_t k = *reinterpret_cast<const uint16_t*>(lblob + KPS(lds_r16_off) + 2u * cell);
        if (active && nib != 15u) {
          srv = (int)nib;
          full = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * k);
        }
      } else if (active && nib != 15u) {
        srv = (int)nib;
        const int sp = *reinterpret_cast<const int*>(lblob + kp.lds_st_off + 4u * nib);
        const int dx = pos.x - (int)(short)sp, dy = pos.y - (sp >> 16);
        const uint32_t d2 = (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
        const uint2 w = *reinterpret_cast<const uint2*>(lblob + kp.lds_rank_off + 8u * (d2 >> 5));
        const uint32_t k = w.y + (uint32_t)__popc(w.x & ((1u << (d2 & 31u)) - 1u));
        full = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * k);
      }
    } else {
      // (heterogeneous entities: the map of this UE's class, [NU][H][W])
      const int xi = min(max(pos.x, 0), KPS(W) - 1), yi = min(max(pos.y, 0), KPS(H) - 1);
      const uint32_t moff = het ? (uint32_t)cu * (uint32_t)(KPS(W) * KPS(H)) : 0u;
      const int4 r = at(const_cast<int4*>(tb.assoc), 16u * ((uint32_t)(yi * KPS(W) + xi) + moff));
      if (active) {
        srv = r.x;
        full = __hiloint2double(r.w, r.z);
      }
    }
  }
  // the previous fused step's stores, after this step's gather; then the gather is waited for
  // on every path (an empty asm reading its registers): a lane or wave that never reads
  // `full` (no server) would otherwise carry the load as pending around the loop, and the
  // compiler's merged wait before its register is reused is vmcnt(0) -- which also waits for
  // every store just issued
  // (LDSA: no gather, nothing to defer -- the step's own stores go out at its end)
  constexpr bool DEFER = FUSED && !LDSA;
  if (DEFER) {
    flush_pending<LEAN>(out, *pend, (uint32_t)kp.E, (uint32_t)(kp.E * U),
                        (uint32_t)max(row - 1, 0));
    asm volatile("" ::"v"(srv), "v"(full));
  }

  // ---- 3. n_b of the own serving BS ---------------------------------------------------
  const uint64_t mcon = bal(srv >= 0) & segmask;
  int n;
  if (PC == 16 && SCN && packed_counts_ok(UC, KPS(B))) {
    n = row_count_same(srv);  // (registered scenarios: B is a compile-time constant)
  } else if (KPS(hist_lds)) {
    // per-env histogram in the wavefront's own LDS slice [G][B]: zero, count, read back
    // (one wavefront's LDS instructions execute in order: no barrier)
    int* h = hist + m.seg * KPS(B);
    if (env_ok)
      for (int k = u; k < KPS(B); k += P) h[k] = 0;
    __builtin_amdgcn_wave_barrier();
    if (srv >= 0) __hip_atomic_fetch_add(h + srv, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __builtin_amdgcn_wave_barrier();
    n = srv >= 0 ? h[srv] : 0;
  } else {
    // lanes of the segment with the same index, matched bit by bit with ballots
    uint64_t match = mcon;
    for (int bit = 0; bit < kp.srv_bits; ++bit) {
      const bool on = (srv >> bit) & 1;
      const uint64_t mb = bal(on);
      match &= on ? mb : ~mb;
    }
    n = (int)__popcll(match);
  }

  // ---- 4. rate (ResourceFair share, rounded to cents) + utility -----------------------
  double cents = 0.0, rate = 0.0;
  float cents_f = 0.f;
  double r100b = 0.0;
  if constexpr (!LDSA && TF) {  // (one-step launches) 100 / n from lane n's table entry (all
    // lanes active here: ds_bpermute reads the source lanes' registers)
    const int src = (srv >= 0 ? n : 0) << 2;
    const int lo = __builtin_amdgcn_ds_bpermute(src, __double2loint(cur.r100l));
    const int hi = __builtin_amdgcn_ds_bpermute(src, __double2hiint(cur.r100l));
    r100b = __hiloint2double(hi, lo);
  }
  if (srv >= 0) {
    if (LDSA && TF) {  // tie-free table (share_tie_free): the product rounds like the reference
      cents = rint(full * *reinterpret_cast<const double*>(lblob + KPS(lds_r100_off) + 8u * (uint32_t)n));
      cents_f = (float)cents;
    } else if (!LDSA && TF) {
      cents = rint(full * r100b);
      cents_f = (float)cents;
    } else {
      cents = LDSA ? share_cents_r(full, *reinterpret_cast<const double*>(
                                             lblob + KPS(lds_r100_off) + 8u * (uint32_t)n), n, cents_f)
                   : share_cents(full, n, cents_f);
    }
  }
  if (want_rate) rate = cents / 100.0;  // exact float64 rate (base.py:435)
  const float rate_f = cents_f * 0.01f;  // the obs value
  double util = 0.0;
  if (active) {
    // exact float64 utility (table) when the caller asks for it, else the float32 form
    util = exact_util ? utility_of(rate, cents, kp, tb.util) : utility_f32r<SCN>(cents_f, rate_f, kp);
  }

  // ---- 5. reward = np.mean(utilities of active UEs, id order) (metrics.py:25-28) ------
  // (not the constant U of an all-active scenario: the reward's hardware reciprocal of a
  // constant would be folded at compile time, correctly rounded, one ulp off the other shapes')
  const int nact = ROWS ? __popc(seg_field<PC>(act_w, m)) : __popcll(act_w & segmask);
  // lean path, aligned segments: the utilities (float32 values in [-1, 1]) summed as 2^-25
  // fixed point in int32 -- one DPP add per level instead of two moves and a float64 add;
  // error <= 2^-25 per UE, 1e-8 on the mean, below the float32 reward's own rounding
  constexpr bool ISUM = LEAN && ROWS;
  const double sum_u = ISUM ? 0.0
                            : ROWS ? seg_sum_rows<PC>(util, active) : seg_sum(util, active, U, u);
  const int isum_u = ISUM ? seg_isum_rows<PC>(active ? (int)((float)util * 0x1p25f) : 0) : 0;
  // reward_risky (rare): the env's mean from the exact utilities
  bool use_exact = false;
  float exact_r = 0.f;
  if constexpr (LEAN) {
    // (the rare path's constants from the LDS blob's RewardC where there is one)
    const char* rcp = LDSA ? lblob + KPS(lds_r100_off) + 8 * kRewardCSlot : nullptr;
    // (every UE active, aligned segments: the test as one unsigned compare, its ballot ANDed in
    // SALU with the env leaders' lanes -- see lds2_step)
    uint64_t risk_w;
    if constexpr (ISUM && scn_all_active<SCN>()) {
      constexpr uint64_t kLeadPat = [] {
        uint64_t v = 0;
        for (int q = 0; q < 64 / (PC ? PC : 64); ++q) v |= 1ull << (q * PC + PC - 1);
        return v;
      }();
      const uint32_t T = (uint32_t)U * (uint32_t)kp.r_thr25;
      risk_w = bal((uint32_t)isum_u + T <= 2u * T) & (envok_w & kLeadPat);
    } else {
      risk_w = bal(env_ok && leader && nact > 0 &&
                   (ISUM ? (uint32_t)abs(isum_u) <= (uint32_t)nact * (uint32_t)kp.r_thr25
                         : fabsf((float)sum_u) <= (float)nact * kp.r_thr));
    }
    if (risk_w) {
      wait_vmem();  // (no load in flight across the call)
      const RewardC c = LDSA ? reward_c(rcp)
                             : RewardC{tb.util, kp.util_sat, (double)kp.util_kmax, kp.u_err, 0};
      const float ex = packed_fix<ROWS, PC>(active ? cents : -1.0, U, u, c.tab, c.kmax, c.sat, nact);
      use_exact = (risk_w >> __lane_id()) & 1ull;
      exact_r = ex;
    }
  }
  double sum_r = 0.0;
  if (want_metrics)
    sum_r = ROWS ? seg_sum_rows<PC>(rate, srv >= 0) : seg_sum(rate, srv >= 0, U, u);
  // per-episode statistics of the rounded QoE values (numpy round(u, 2) = rint(100 u) / 100)
  double sum_q = 0.0, sum_q2 = 0.0;
  int nlow = 0;
  if (want_qoe) {
    const double q = rint(util * 100.0) / 100.0;
    sum_q = ROWS ? seg_sum_rows<PC>(q, active) : seg_sum(q, active, U, u);
    sum_q2 = ROWS ? seg_sum_rows<PC>(q * q, active) : seg_sum(q * q, active, U, u);
    nlow = (int)__popcll(bal(active && q < kp.qoe_low) & segmask);
  }

  // ---- 6. stores ----------------------------------------------------------------------
  const float4 obs = make_float4((float)pos.x * KPSF(inv_w), (float)pos.y * KPSF(inv_h), rate_f,
                                 (float)util);
  const double util_out = active ? util : __builtin_nan("");
  if (valid && !FUSED) {
    const uint32_t ui = (uint32_t)idx;
    store_ue_at(st.ue_state, ui, pos, wp, KST8);
    at(out.serving, 4u * ui) = srv;
    at(out.obs, 16u * ui) = obs;
    if (own_fin && (!M || fell_back))  // the stream moved: write the new state back (with the
                                       // table only after draws past it, mev_state.pcg)
      at(reinterpret_cast<ulonglong2*>(st.pcg), 48u * (uint32_t)e) =
          make_ulonglong2((uint64_t)s_fin, (uint64_t)(s_fin >> 64));
    if (!LEAN && out.rate64) out.rate64[idx] = rate;
    if (!LEAN && out.util64) out.util64[idx] = util_out;
  }
  if (FUSED && STG) {  // the per-UE rows now, before the leaders' reward branch (issued after
    // it, the compiler duplicates the stores into both sides: twice the store instructions,
    // each half a row)
    Pending up;
    up.srv = srv;
    up.obs = obs;
    up.ui = (uint32_t)idx;
    up.valid = valid;
    up.lead = up.done = false;
    up.e = 0;
    up.reward = 0.f;
    flush_pending<LEAN, false>(out, up, (uint32_t)kp.E, (uint32_t)(kp.E * U), (uint32_t)row);
  }
  const bool lead = env_ok && leader;
  float reward_out = 0.f;
  float4 met = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lead) {
    // np.mean; the lean path divides in float32 (the reward output is float32)
    const double mean_u =
        ISUM ? (nact > 0 ? (double)((float)isum_u * 0x1p-25f *
                                    __builtin_amdgcn_rcpf((float)nact))
                         : kp.lower)
        : LEAN ? (nact > 0 ? (double)((float)sum_u * __builtin_amdgcn_rcpf((float)nact))
                           : kp.lower)
               : (nact > 0 ? sum_u / (double)nact : kp.lower);
    reward_out = use_exact ? exact_r : (float)mean_u;
    if (want_metrics) {
      const int ncon = __popcll(mcon);
      const double mean_r = ncon > 0 ? sum_r / (double)ncon : 0.0;
      met = make_float4((float)ncon, (float)ncon, (float)mean_u, (float)mean_r);
    }
    if (!FUSED) {
      at(st.t, 4u * (uint32_t)e) = t + 1;
      if (M && (tot || reset_env)) at(tb.drawn, 4u * (uint32_t)e) = drawn + tot;
      if (STG) {  // staged: the block writes its envs' rows together (k_step_packed)
        srew[m.seg] = reward_out;
        sdone[m.seg] = (uint8_t)(t + 1 >= KPS(t_end));
      } else {
        at(out.reward, 4u * (uint32_t)e) = reward_out;
        at(out.done, (uint32_t)e) = (uint8_t)(t + 1 >= KPS(t_end));
      }
      if (want_metrics) out.metrics[e] = met;
    }
    if (want_qoe) {
      double4 a = t == 0 ? make_double4(0.0, 0.0, 0.0, 0.0) : out.qoe_stats[e];
      a.x += (double)nact;
      a.y += sum_q;
      a.z += sum_q2;
      a.w += (double)nlow;
      out.qoe_stats[e] = a;
    }
  }
  if (FUSED) {  // DEFER: held back until the next step's gather (or the end of the launch)
    Pending cp;
    cp.srv = srv;
    cp.obs = obs;
    cp.rate = rate;
    cp.util = util_out;
    cp.reward = reward_out;
    cp.met = met;
    cp.ui = (uint32_t)idx;
    cp.e = e;
    cp.valid = valid;
    cp.lead = lead;
    cp.done = t + 1 >= KPS(t_end);
    if (DEFER) {
      *pend = cp;
    } else {
      if (!STG)
        flush_pending<LEAN>(out, cp, (uint32_t)kp.E, (uint32_t)(kp.E * U), (uint32_t)row);
      if (STG && lead) {  // this step's row slot of the workgroup's staged per-env rows
        srew[m.seg] = reward_out;
        sdone[m.seg] = (uint8_t)cp.done;
      }
    }
  }
  if (FUSED) {
    cur.t = t + 1;
    cur.s = make_int4(pos.x, pos.y, wp.x, wp.y);
    cur.drawn = drawn + tot;
    cur.s_ok = s_ok;
  }
  return own_fin;  // this lane holds a new stream state of its env (the caller reduces)
}

// Block -> env-range slot. Blocks are dealt round-robin over the 8 XCDs (observed placement,
// MI355X_MICROARCH.md "Workgroup dispatch"); with the remap the blocks that share an XCD
// (equal blockIdx % 8) cover one contiguous range, so the per-env rows that several blocks
// write partially (t, reward, done, pcg) are merged in one L2 instead of eight. Bijective
// for any grid size. Speed only: any block order is correct. remap > 1 (dev): the slots are
// shifted cyclically by the start of range remap - 1, so XCD x covers the range XCD
// x + remap - 1 would (whole ranges when 8 divides the grid) -- still a bijection.
__device__ __forceinline__ int block_slot(int remap) {
  const int orig = blockIdx.x;
  if (!remap) return orig;
  const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7;
  auto base = [&](int x) { return x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q; };
  const int s = base(orig & 7) + (orig >> 3);
  if (remap == 1) return s;
  const int t = s + base(remap - 1);
  return t >= nwg ? t - nwg : t;
}

// 16-byte pieces of the LDS blob a rollout copies: all of it, or (mode 3) up to the rates over D
// in use (KTables::dcount)
template <int SCN>
__device__ __forceinline__ int blob_copy_n16(const KParams& kp, const KTables& tb) {
  const int all = KPS(lds_assoc) >> 4;
  if (!tb.dcount) return all;
  return min(all, (KPS(lds_rate_off) + 8 * *tb.dcount + 15) >> 4);
}

// Step kernel: one env group per wavefront (latency hidden by occupancy).
// Groups [g0, ngroups) of the batch (g0 > 0: second half of the two-stream shape).
// TF (scenario instances, share_tie_free, a context with the LDS blob): the share as the
// product with the host's correctly rounded 100 / n (no reciprocal iterations, no tie test).
template <bool PER_ENV_BS, bool LEAN, int UC, int SCN = 0, bool TF = false>
__global__ __launch_bounds__(kPackedBlock) void k_step_packed(KParams kp, KState st, KOut out,
                                                             KTables tb, int g0, int ngroups) {
  extern __shared__ int lds_hist[];  // [waves][G][B] when KPS(hist_lds)
  const int lane = threadIdx.x & 63;
  const int gb = g0 + block_slot(kp.xcd_remap) * kWavesPerBlock;
  const int g = gb + (threadIdx.x >> 6);
  // STG (lean, compile-time U): the block's per-env rows (reward float32, done byte) are
  // staged in LDS and written together after a barrier -- one 4 NW G-byte reward piece per
  // block instead of one 4 G-byte piece per wavefront (the rollout kernel's measurement:
  // such small pieces cost 12 % there); waves without a group only take part in the barrier
  constexpr bool STG = LEAN && UC != 0 && !PER_ENV_BS;
  constexpr int GC = UC ? 64 / pitch_of(UC ? UC : 1) : 1;
  __shared__ float srw[STG ? kWavesPerBlock * GC : 1];
  __shared__ uint8_t sdn[STG ? kWavesPerBlock * GC : 1];
  if (!STG && g >= ngroups) return;
  constexpr int PC = UC ? pitch_of(UC) : 0;
  const int U = UC ? UC : kp.U;
  const int P = PC ? PC : kp.U;
  const int G = PC ? 64 / (PC ? PC : 1) : kp.envs_per_wave;
  const LaneMap m = lane_map<PC>(lane, P);
  const int e = g * G + m.seg;
  const bool env_ok = (m.seg < G) && (e < kp.E);
  if (g < ngroups) {
    GroupIn a = load_group<SCN>(kp, st, tb, e, min(m.u, U - 1), U, false);
    a.r100l = TF ? *reinterpret_cast<const double*>(reinterpret_cast<const char*>(tb.lds_blob) +
                                                    KPS(lds_r100_off) + 8u * (uint32_t)lane)
                 : 0.0;
    packed_group<PER_ENV_BS, LEAN, UC, false, 0, SCN, STG, TF>(
        kp, st, out, tb, m, a, e, env_ok, lds_hist + (threadIdx.x >> 6) * G * kp.B, nullptr,
        nullptr, 0, nullptr, nullptr, srw + (threadIdx.x >> 6) * GC,
        sdn + (threadIdx.x >> 6) * GC);
  }
  if (STG) {
    __syncthreads();
    const int j = (int)threadIdx.x, eo = gb * GC + j;
    if (j < kWavesPerBlock * GC && eo < kp.E && gb + j / GC < ngroups) {
      at(out.reward, 4u * (uint32_t)eo) = srw[j];
      at(out.done, (uint32_t)eo) = sdn[j];
    }
  }
}

// nsteps fused steps per launch (mev_step / mev_rollout with n > 1): each wavefront advances
// its env group n steps with the state in registers -- loaded once, stored once -- and writes
// the outputs of every step: into row i of the trajectory buffers (traj != 0, mev_rollout),
// or over the previous step's (mev_step; the caller sees the last step's, as with n launches). One launch
// instead of n removes n - 1 kernel boundaries and the fill / drain of every launch.
//   LDSA: workgroups of kLdsWaves waves share one LDS copy of the compact association tables
//   (shared layouts whose tables fit, KParams::lds_assoc), copied once; the grid is then sized
//   to the resident workgroups (persistent: each wave takes groups g, g + T, g + 2T, ... of the
//   T waves of the grid), so the copy is made once per workgroup slot, not once per group.
// STG: the workgroup writes its staged per-env rows [row0, row0 + nr) x [e0, e0 + NWG) (reward
// float32, done byte) with consecutive threads on consecutive envs, between two barriers (the
// slots are complete before, and free for the next steps after).
__device__ __forceinline__ void flush_staged(const KOut& out, const float* srew,
                                             const uint8_t* sdone, int E, int e0, int row0,
                                             int nr, int NWG) {
  __syncthreads();
  for (int q = threadIdx.x; q < nr * NWG; q += (int)blockDim.x) {
    const int r = q / NWG, j = q - r * NWG;
    if (e0 + j < E) {
      const size_t ro = (size_t)(row0 + r) * (size_t)E;
      const uint32_t o = (uint32_t)(e0 + j);
      at(out.reward + ro, 4u * o) = srew[q];
      at(out.done + ro, o) = sdone[q];
    }
  }
  __syncthreads();
}

template <bool PER_ENV_BS, bool LEAN, int UC, int LDSM, int SCN = 0, bool TF = false>
__global__ __launch_bounds__(64 * lds_waves(LDSM)) void k_steps_packed(
    KParams kp, KState st, KOut out, KTables tb, int ngroups, int nsteps, int traj,
    int stage_rows) {
  extern __shared__ int lds_all[];
  constexpr bool LDSA = LDSM != 0;
  // waves per workgroup: up to lds_waves(LDSM) (the launch bounds); LDSA launches with few
  // groups take fewer, so that the workgroups spread over every CU
  const int NW = (int)(blockDim.x >> 6);
  int* lds_hist = lds_all;
  const char* lblob = nullptr;
  if (LDSA) {
    // LDS-DMA copy (no registers): wave w moves 1 KB pieces w, w + NW, ...
    const int n16 = blob_copy_n16<SCN>(kp, tb);
    const int ln = threadIdx.x & 63;
    for (int c = (int)(threadIdx.x >> 6); c * 64 < n16; c += NW)
      if (c * 64 + ln < n16) glds(tb.lds_blob + c * 64 + ln, reinterpret_cast<int4*>(lds_all) + c * 64);
    wait_vmem();
    __syncthreads();
    lblob = reinterpret_cast<const char*>(lds_all);
    lds_hist = lds_all + (KPS(lds_assoc) >> 2);
  }
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  constexpr int PC = UC ? pitch_of(UC) : 0;
  constexpr bool ROWS = PC == 16 || PC == 32;
  const int U = UC ? UC : kp.U;
  const int P = PC ? PC : kp.U;
  const int G = PC ? 64 / (PC ? PC : 1) : kp.envs_per_wave;
  const LaneMap m = lane_map<PC>(lane, P);
  // per wave: stream slots [G][2] u128 {state, inc}, the n_b histogram, the group's episode
  // draw tables (x, y pairs) in LDS for the whole launch (lds_per_wave)
  // (per-env station keys right after the stream slots: 16-byte aligned for ds_read_b128)
  const int LB = SCN ? 0 : kp.lbs;  // ints per env of the staged station keys
  u128* lpcg = reinterpret_cast<u128*>(lds_hist) + wv * G * 2;
  int* lbs = lds_hist + NW * G * 8 + wv * G * LB;
  int* hist = lds_hist + NW * G * (8 + LB) + wv * G * KPS(B) * KPS(hist_lds);
  int* ltab = lds_hist + NW * G * (8 + LB + KPS(B) * KPS(hist_lds)) + wv * G * KPS(tab_m);
  // STG (LDS-table trajectory launches, lean outputs): the per-env rows (reward float32, done
  // byte) of the workgroup's NW * G consecutive envs are staged in LDS for stage_rows steps and
  // then written by the whole workgroup as contiguous row pieces (128 B of reward per row for
  // mobile-large) -- instead of every wavefront writing 2 x 4 B and 2 x 1 B pieces of each row
  // (measured: those partial-line writes cost 1.5 of 13.5 us per step). The group loop is then
  // uniform over the workgroup (its barriers): waves past the last group only take part in them.
  constexpr bool STG = LDSM >= 2 && LEAN && UC != 0;
  const int NWG = NW * (PC ? 64 / (PC ? PC : 1) : 1);  // envs per workgroup tile (STG)
  float* srew = reinterpret_cast<float*>(lds_hist + NW * G * (8 + LB + KPS(B) * KPS(hist_lds) +
                                                              KPS(tab_m)));
  uint8_t* sdone = reinterpret_cast<uint8_t*>(srew + (STG ? stage_rows * NWG : 0));
  const int gstride = LDSA ? (int)gridDim.x * NW : ngroups;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  for (int gb = block_slot(kp.xcd_remap) * NW; gb < (STG ? ngroups : ngroups - wvu); gb += gstride) {
    const int g = gb + wvu;
    if (STG && g >= ngroups) {  // no group for this wave: its part of the flushes only
      for (int i0 = 0; i0 < nsteps; i0 += stage_rows)
        flush_staged(out, srew, sdone, kp.E, gb * G, traj ? i0 : 0, min(stage_rows, nsteps - i0),
                     NWG);
      continue;
    }
    const int e = g * G + m.seg;
    const bool env_ok = (m.seg < G) && (e < kp.E);
    // the group's inputs: the draw table (LDS-DMA, 256 B per instruction), the env state and
    // the stream state, all issued before one wait
    if (KPS(tab_m)) {
      const int n = G * KPS(tab_m);
      const int* src = tb.tab_xy + (size_t)g * n;
      const int lim = min(n, (kp.E - g * G) * KPS(tab_m));  // rows of envs that exist
      for (int c = 0; c * 64 < lim; ++c)
        if (c * 64 + lane < lim) glds(src + c * 64 + lane, ltab + c * 64);
    }
    GroupIn a = load_group<SCN>(kp, st, tb, e, min(m.u, U - 1), U, true);
    // per-env layouts: the env's station keys in the wave's LDS slots, 16 per env, as
    // {m = -16 q (int16x2), c = ((|q|^2 + 2^21) << 4) | j}, so that the key of station j for
    // a UE at p is ONE dot product: dot2(2 p, m) + c = ((|p - q|^2 - |p|^2 + 2^21) << 4) | j
    // (coordinates < 1024: |2 p|, |16 q| < 2^15, and the key < 2^32); slots past the env's
    // count hold {0, UINT_MAX}, a key that never wins
    int nb_f = 0;
    if (PER_ENV_BS && LB) {
      const int ec = min(e, kp.E - 1);
      nb_f = env_ok ? (st.bs_count ? st.bs_count[ec] : KPS(B)) : 0;
      if (m.seg < G)  // (lanes past the last segment hold no env)
        for (int k = m.u; k < 16; k += P) {
          int2 kv = make_int2(0, -1);
          if (k < nb_f) {
            const int2 q = st.bs_xy[(size_t)ec * KPS(B) + k];
            const s16x2 m2 = {(short)(-16 * q.x), (short)(-16 * q.y)};
            kv = make_int2(__builtin_bit_cast(int, m2),
                           (int)(((unsigned)(q.x * q.x + q.y * q.y + (1 << 21)) << 4) | (unsigned)k));
          }
          *reinterpret_cast<int2*>(lbs + m.seg * 32 + 2 * k) = kv;
        }
    }
    const bool leader = ROWS ? m.u == P - 1 : m.u == 0;
    ulonglong2 pa = make_ulonglong2(0, 0), pb = pa;
    if (env_ok && leader) {
      ulonglong2* pr = reinterpret_cast<ulonglong2*>(st.pcg);
      pa = at(pr, 48u * (uint32_t)e);
      pb = at(pr, 48u * (uint32_t)e + 16u);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (env_ok && leader) {
      lpcg[2 * m.seg] = mk128(pa.x, pa.y);
      lpcg[2 * m.seg + 1] = mk128(pb.x, pb.y);
    }
    bool moved = false;
    Pending pend;  // nothing to store before the first step
    pend.valid = pend.lead = pend.done = false;
    pend.srv = pend.ui = pend.e = 0;
    pend.obs = pend.met = make_float4(0.f, 0.f, 0.f, 0.f);
    pend.rate = pend.util = 0.0;
    pend.reward = 0.f;
    // the group's inputs have landed before the loop: otherwise the compiler's wait for them,
    // merged into the loop header, would also wait for the previous step's stores
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t envok_w = bal(env_ok), valid_w = bal(env_ok && m.u < U);
    for (int i = 0; i < nsteps; ++i) {
      const int sr = STG ? i % stage_rows : 0;
      moved |= packed_group<PER_ENV_BS, LEAN, UC, true, LDSM, SCN, STG, TF>(
          kp, st, out, tb, m, a, e, env_ok, hist, ltab, &pend, traj ? i : 0, lblob, lpcg,
          srew + sr * NWG + wvu * G, sdone + sr * NWG + wvu * G, envok_w, valid_w, lbs, nb_f);
      if (STG && (sr == stage_rows - 1 || i == nsteps - 1))
        flush_staged(out, srew, sdone, kp.E, gb * G, traj ? i - sr : 0, sr + 1, NWG);
    }
    if (!LDSA)  // the last step's deferred outputs
      flush_pending<LEAN>(out, pend, (uint32_t)kp.E, (uint32_t)(kp.E * U),
                          traj ? (uint32_t)(nsteps - 1) : 0u);
    // the state after the last step
    if (env_ok && m.u < U)
      store_ue_at(st.ue_state, (uint32_t)(e * U + m.u), make_int2(a.s.x, a.s.y),
                  make_int2(a.s.z, a.s.w), KST8);
    // the env's stream moved during the launch: some lane of it owned a new state
    const uint64_t mv = bal(moved);
    moved = ROWS ? seg_field<PC>(mv, m) != 0u : (mv & m.segmask) != 0;
    if (env_ok && leader) {
      at(st.t, 4u * (uint32_t)e) = a.t;
      if (KPS(tab_m)) at(tb.drawn, 4u * (uint32_t)e) = a.drawn;
      // the stream state after the last pair drawn, where the slot holds it (without a table:
      // always; with one: after draws past it -- otherwise the table's entry is the state and
      // the row is left as it is, mev_state.pcg; no global load, whose wait would drain every
      // store of the launch)
      if (moved && a.s_ok) {
        const u128 sl = lpcg[2 * m.seg];
        at(reinterpret_cast<ulonglong2*>(st.pcg), 48u * (uint32_t)e) =
            make_ulonglong2((uint64_t)sl, (uint64_t)(sl >> 64));
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Two env groups per wavefront: k_steps_lds2 (trajectory rollouts, mode-3 LDS tables)
// ------------------------------------------------------------------------------------
// The LDS tables (mode 3, 113 KB for 200 x 200) leave room for one 16-wave workgroup per CU,
// i.e. 4 waves per SIMD; a rollout step at that occupancy waits on its own dependency chains
// (LDS reads, ballots, the DPP sums) much of the time (measured: 2 waves per SIMD 16.6 vs 4
// waves 11.6 us per step). Here each wavefront advances TWO env groups (contexts r = 0, 1) in
// one instruction stream: the common path of a step is branch-free (movement, association,
// n_b, share, utility, sums and stores computed for every lane and selected), so the two
// contexts' instructions sit in the same basic blocks and the scheduler interleaves them. The
// rare paths (fallback draws past the draw table, the exact float64 movement, share ties, far
// cells, episode resets) are wave-uniform branches per context. Same results as packed_group
// bit for bit (tests). Shapes: U = 15 / 30 at compile time (aligned segments), lean outputs,
// a draw table (tab_m > 0), staged per-env rows.
// Per-env histogram stride of k_steps_lds2 (see lds2_per_wave): max(B + 1, P = 64 / G)
__host__ __device__ constexpr int lds2_hist_stride(int G, int B) {
  return B + 1 > 64 / G ? B + 1 : 64 / G;
}
// A group's context in k_steps_lds2. The per-env flags are bits of one int per lane (the env's
// value in each of its lanes), changed only inside the wave-uniform draw / reset branch: as
// per-lane bools the compiler kept them as SGPR lane masks and merged them across every
// divergent region of the step (three s_andn2 / s_and / s_or per flag and group, every step).
//   bit 0 (kSok): the env's stream slot holds its stream state (draws past the episode table);
//   bit 1 (kMov): the env drew past the table in this pair (its state row is stored at the end).
// (The pipelined loop, pipe_move, keeps no flags: there the slot is current exactly when
// drawn > M -- an env draws from the episode table while its pair index is below M, and only
// past it from the stream state, whose last drawing lane writes the slot; restored rows have
// drawn = M + 1. Measured: the flag-free form 101 vs 104 us per 200-step launch at 4,096 medium
// envs, but 1.55 vs 1.51 ms at 65,536 large envs in the two-group loop, interleaved on one box.)
constexpr int kSok = 1, kMov = 2;
struct Ctx2 {
  int t, drawn, fl;
  int2 pos, wp;
};

// FULL: every env of both groups exists (all pairs but the batch's last partial one): the
// env / valid lane masks are constants, no per-step mask arithmetic.
// HET: heterogeneous entities with a shared layout (KParams::lds_mode 6, build_het_lds): the
// lane's UE class hcu and movement parameters hmv (per UE, tb.mv); the association from the
// LDS cell map of the closest station within any pair's reach, s*, which serves the UE when the
// (class of s*, UE class) pair connects at that distance -- the closest station overall is then
// the closest connectable one, ties by index included -- else from the UE class's L2 map.
template <int UC, int SCN, int R, bool PE, bool TF = false, bool FULL = false, bool HET = false,
          bool RT1 = false>
__device__ __forceinline__ void lds2_step(const KParams& kp, const KState& st, const KOut& out,
                                          const KTables& tb, const LaneMap& m, Ctx2 (&c)[R],
                                          const int (&e)[R], const int (&nok)[R], int kval,
                                          int klead, int row,
                                          const char* __restrict__ lblob, u128* __restrict__ lpcg,
                                          int* __restrict__ hist, const int* __restrict__ ltab,
                                          int* __restrict__ srow, const int* __restrict__ lkeys,
                                          uint32_t hpk = 0, float hvf = 0.f, float hml = 0.f) {
  constexpr int PC = pitch_of(UC), U = ue_of(UC), G = 64 / PC;
  const int M = KPS(tab_m), B = KPS(B), HS = lds2_hist_stride(G, B);
  const int u = m.u;
  // lanes UE u of segment s hold valid = u < U; wave masks of the envs that exist (nok[r] of
  // the group's G) from the uniform count, in SALU each step (kept loop-variant: hoisted, the
  // masks would be spilled from SGPRs and restored by v_readlane every step)
  constexpr uint64_t kValidPat = [] {
    uint64_t v = 0;
    for (int q = 0; q < 64 / PC; ++q) v |= ((1ull << U) - 1ull) << (q * PC);
    return v;
  }();
  bool env_ok[R];
  uint64_t envok_w[R], valid_w[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (FULL) {
      envok_w[r] = ~0ull;
      valid_w[r] = kValidPat;
      env_ok[r] = true;
    } else {
      int nk = nok[r];
      asm volatile("" : "+s"(nk));
      envok_w[r] = nk >= G ? ~0ull : ((1ull << (uint32_t)(nk * PC)) - 1ull);
      valid_w[r] = envok_w[r] & kValidPat;
      env_ok[r] = m.seg < nk;
    }
  }
  bool valid[R], active[R], need[R], do_reset[R], reset_env[R];
  int tot[R], rank[R];
  uint64_t act_w[R], mneed_w[R], rs_w[R];
  // ---- A: lazy auto-reset, ballots (base.py:288-291) ----------------------------------------
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int er = r * G + m.seg;  // the env's slot among the wave's R * G
    valid[r] = FULL ? u < U : kval < nok[r];
    reset_env[r] = env_ok[r] && c[r].t >= KPS(t_end);
    do_reset[r] = reset_env[r] && valid[r];
    rs_w[r] = bal(c[r].t >= KPS(t_end)) & envok_w[r];
    if (rs_w[r]) {  // initial positions = the episode's first U
      if (reset_env[r]) {                          // pairs of the draw table
        c[r].t = 0;
        c[r].drawn = U;
      }
      if (do_reset[r]) {
        const int p = ltab[er * M + u];
        c[r].pos = make_int2((int)(short)p, p >> 16);
        c[r].wp = make_int2(-1, -1);
      }
    }
    const int t = c[r].t;
    const bool on = scn_all_active<SCN>() ||
                    (t >= KPS(arr_start) && t < KPS(arr_exit) && (KPS(first_step_active) || t != 0));
    active[r] = valid[r] && on;
    act_w[r] = scn_all_active<SCN>() ? valid_w[r] : bal(on) & valid_w[r];
    // (no waypoint: wp.x == -1 exactly; as `< 0` the compiler formed the predicate twice, as a
    // shift and as a mask test, each with its own compare)
    const bool nowp = c[r].wp.x == -1;
    need[r] = active[r] && nowp;
    mneed_w[r] = bal(nowp) & act_w[r];
    const uint32_t f = seg_field<PC>(mneed_w[r], m);
    tot[r] = __popc(f);
    rank[r] = __popc(__builtin_amdgcn_ubfe(f, 0u, (uint32_t)u));
  }
  // ---- B: waypoint draws in ue_id order (movement.py:44-47) -----------------------------------
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int er = r * G + m.seg;
    u128* const slot = lpcg + 2 * er;
    bool fell_back = false;
    u128 s_fin = 0;
    if (mneed_w[r]) {
      const int k = c[r].drawn + rank[r];
      if ((bal(k >= M) & mneed_w[r]) == 0) {  // every pair precomputed (the common case)
        if (need[r]) {
          const int p = ltab[er * M + k];
          c[r].wp = make_int2((int)(short)p, p >> 16);
        }
      } else {  // beyond the table: from the stream state (see packed_group)
        fell_back = true;
        const u128 inc = slot[1];
        u128 s;
        if (!(c[r].fl & kSok) && c[r].drawn > 0) {
          s = at(const_cast<u128*>(tb.tab_st),
                 16u * ((uint32_t)e[r] * (uint32_t)M + (uint32_t)(min(c[r].drawn, M) - 1)));
          wait_vmem();
        } else {
          s = slot[0];
        }
        if (reset_env[r]) {  // the state after this episode's U initial pairs
          s = at(const_cast<u128*>(tb.tab_st), 16u * ((uint32_t)e[r] * (uint32_t)M + (uint32_t)(U - 1)));
          wait_vmem();
        }
        if ((bal(rank[r] != 0) & mneed_w[r]) == 0) {
          if (need[r]) s_fin = pcg_draw_pair_next(s, inc, kp.Wd, kp.Hd, c[r].wp.x, c[r].wp.y);
        } else {
          if (need[r])
            s_fin = pcg_draw_pair(s, inc, 2 * rank[r], tb.jump, kp.Wd, kp.Hd, c[r].wp.x, c[r].wp.y);
        }
        wait_vmem();
      }
    }
    // the stream bookkeeping, only where a draw or a reset happened (uniform; without either
    // nothing changes, and the per-lane masks cost ~15 SALU per group)
    if (mneed_w[r] | rs_w[r]) {
      // the slot holds the state after draws past the table (fell_back, uniform); a draw from
      // the table or a reset leaves it to the table: per env, as lane masks (see Ctx2)
      const bool tw = tot[r] > 0;
      int f = c[r].fl;
      if (fell_back) {
        const bool own_fin = (need[r] && rank[r] == tot[r] - 1) ||
                             (do_reset[r] && tot[r] == 0 && u == U - 1);
        if (own_fin) slot[0] = s_fin;
        f = tw ? (f | kSok | kMov) : reset_env[r] ? (f & ~kSok) : f;
      } else {
        f = (tw || reset_env[r]) ? (f & ~kSok) : f;
      }
      c[r].fl = f;
      c[r].drawn += tot[r];
    }
  }
  // ---- C: movement (movement.py:49-62), branch-free fast path --------------------------------
  // (move_ue_p per lane: arrival snap; axis-parallel moves exactly in float32 when the velocity
  // is a float32 value (scenario constants); the float32 step clear of a tie; else float64)
  constexpr bool AXF = SCN != 0;  // scenario velocity 1.5: pos +- 1.5 exact in float32
  constexpr bool V15 = scn_v15<SCN>();  // velocity 1.5 in integers (step_v15)
  int2 npos[R];
  bool arrive[R];
  if constexpr (HET) {  // each UE with its own velocity: move_ue_p with the lane's parameters
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int2 p = c[r].pos, w = c[r].wp;
      if (active[r]) move_ue_pc(p, w, hvf, hml, hpk, tb.mv + min(m.u, U - 1));
      c[r].pos = p;
      c[r].wp = w;
    }
  }
#pragma unroll
  for (int r = 0; r < R && !HET; ++r) {
    const int2 pos = c[r].pos, wp = c[r].wp;
    const int dx = wp.x - pos.x, dy = wp.y - pos.y;
    const int ax2 = __mul24(dx, dx), ay2 = __mul24(dy, dy);
    const int d2 = ax2 + ay2;
    arrive[r] = d2 <= KPS(d2snap);
    if (V15 || KPS(axis_exact) == 2) {  // (generic instances: a uniform branch)
      // the step for every lane, then a select: as a branch on `arrive` (nearly every lane
      // moves) the compiler spent three SALU on exec masks per group and step
      int2 np = step_v15(pos, dx, dy, ax2, ay2);
      asm volatile("" : "+v"(np.x), "+v"(np.y));
      npos[r] = arrive[r] ? wp : np;
      continue;
    }
    const float sc = KPSF(vel_f) * __builtin_amdgcn_rsqf((float)d2);
    const float qx = (float)dx * sc, qy = (float)dy * sc;
    const float rx = rintf(qx), ry = rintf(qy);
    const bool axis = dx == 0 || dy == 0;
    bool ok = fmaxf(fabsf(qx - rx), fabsf(qy - ry)) < KPSF(move_lim);
    int2 np = make_int2(pos.x + (int)rx, pos.y + (int)ry);
    if (AXF) {
      const float vs = KPSF(vel_f);
      const int ax = (int)rintf((float)pos.x + (dx > 0 ? vs : -vs));
      const int ay = (int)rintf((float)pos.y + (dy > 0 ? vs : -vs));
      if (axis) np = dy == 0 ? make_int2(ax, pos.y) : make_int2(pos.x, ay);
      ok = ok || axis;
    }
    const bool xneed = active[r] && !arrive[r] && !ok;
    if (bal(xneed)) {  // rare: the exact float64 step (ties, non-float32 axis moves)
      if (xneed) np = move_exact(pos, dx, dy, kp.vel);
    }
    npos[r] = arrive[r] ? wp : np;
  }
#pragma unroll
  for (int r = 0; r < R && !HET; ++r) {  // selects (an `if` here became an exec-mask branch)
    const bool pop = active[r] && arrive[r];
    c[r].pos = active[r] ? npos[r] : c[r].pos;
    c[r].wp = pop ? make_int2(-1, -1) : c[r].wp;
  }
  // ---- D: association, n_b, share, utility ---------------------------------------------------
  int srv[R];
  double full[R];
  uint32_t cell[R], ent[R];
  if (PE) {
    // per-env layouts: the env's pre-scaled station keys (staged in LDS, see k_steps_packed),
    // one v_dot2 per station; the full rate at the rank of d2 in S (rank index + rates in LDS)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const s16x2 p2 = {(short)(c[r].pos.x << 1), (short)(c[r].pos.y << 1)};
      const v4u32* sv = reinterpret_cast<const v4u32*>(lkeys + (r * G + m.seg) * 32);
      unsigned best = UINT_MAX;
      auto scan = [&](auto npair) {
#pragma unroll
        for (int q = 0; q < decltype(npair)::value; ++q) {
          const v4u32 w = sv[q];
          const unsigned k0 = (unsigned)__builtin_amdgcn_sdot2(p2, as_s16x2(w.x), (int)w.y, false);
          const unsigned k1 = (unsigned)__builtin_amdgcn_sdot2(p2, as_s16x2(w.z), (int)w.w, false);
          best = min(best, min(k0, k1));
        }
      };
      // (scenario constants: ceil(B / 2) slot pairs -- the slots past the env's stations hold
      // the never-winning key)
      constexpr int NPS = SCN ? (scn_const(SCN).B + 1) / 2 : 0;
      if (NPS) scan(std::integral_constant<int, NPS ? NPS : 1>());
      else if (KPS(B) <= 8) scan(std::integral_constant<int, 4>());
      else scan(std::integral_constant<int, 8>());
      const int d2s = (int)(best >> 4) - (1 << 21) + __mul24(c[r].pos.x, c[r].pos.x) +
                      __mul24(c[r].pos.y, c[r].pos.y);
      srv[r] = active[r] && best != UINT_MAX && d2s <= kp.d2max ? (int)(best & 15u) : -1;
      const uint32_t dq = (uint32_t)min(max(d2s, 0), kp.d2max);
      const uint2 w = *reinterpret_cast<const uint2*>(lblob + 8u * (dq >> 5));  // (mode 4: at 0)
      const uint32_t k = w.y + (uint32_t)__popc(w.x & ((1u << (dq & 31u)) - 1u));
      full[r] = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * k);
      cell[r] = ent[r] = 0;
    }
  } else if (HET) {
    // mode 6: s* per cell (4 bits, 15: none within reach), its coordinates and class, d2 to it,
    // the rank k of d2 in D of its class (the class's rank index); per (UE class, station) the
    // pair's {rate offset, largest connectable rank} (read beside the coordinates)
    const int cells = KPS(W) * KPS(H);
    const uint32_t nwd = (uint32_t)kp.d2max / 32u + 1u, reach = (uint32_t)kp.d2max;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      cell[r] = min(__umul24((uint32_t)c[r].pos.y, (uint32_t)KPS(W)) + (uint32_t)c[r].pos.x,
                    (uint32_t)(cells - 1));
      const uint32_t nib =
          ((uint32_t)*reinterpret_cast<const uint8_t*>(lblob + (cell[r] >> 1)) >> ((cell[r] & 1u) << 2)) & 15u;
      const bool has = nib != 15u;
      const uint32_t s = has ? nib : 0u;
      const uint32_t sp = *reinterpret_cast<const uint32_t*>(lblob + kp.lds_st_off + 4u * s);
      const int2 pk = *reinterpret_cast<const int2*>(lblob + kp.lds_r16_off +
                                                     8u * ((hpk & 15u) * (uint32_t)B + s));
      const int dx = c[r].pos.x - (int)(sp & 4095u), dy = c[r].pos.y - (int)((sp >> 12) & 4095u);
      const uint32_t d2 = (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
      const uint32_t dq = min(d2, reach);
      const uint2 w = *reinterpret_cast<const uint2*>(lblob + kp.lds_rank_off +
                                                      8u * ((sp >> 24) * (nwd + 1u) + (dq >> 5)));
      const uint32_t k = w.y + (uint32_t)__popc(w.x & ((1u << (dq & 31u)) - 1u));
      const bool conn = has && d2 <= reach && (int)k <= pk.y && k < 4095u;  // (runs: <= 4,095, k_het_info)
      full[r] = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) +
                                                 8u * (conn ? (uint32_t)pk.x + k : 0u));
      srv[r] = active[r] && conn ? (int)s : -1;
      // s* out of this class's reach (another station may serve it): the class's L2 map
      const bool fb = active[r] && has && !conn;
      if (bal(fb) & act_w[r]) {
        if (fb) {
          const int4 q = at(const_cast<int4*>(tb.assoc),
                            16u * ((hpk & 15u) * (uint32_t)cells + cell[r]));
          srv[r] = q.x;
          full[r] = __hiloint2double(q.w, q.z);
        }
        wait_vmem();
      }
      ent[r] = 0;
    }
  } else {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    cell[r] = min(__umul24((uint32_t)c[r].pos.y, (uint32_t)KPS(W)) + (uint32_t)c[r].pos.x,
                  (uint32_t)(KPS(W) * KPS(H) - 1));
    ent[r] = *reinterpret_cast<const uint16_t*>(lblob + 2u * cell[r]);
    full[r] = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * (ent[r] & 4095u));
    srv[r] = active[r] && ent[r] < 0xF000u ? (int)(ent[r] >> 12) : -1;
  }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (!PE && !HET && (bal(ent[r] == 0xFFFFu) & act_w[r])) {  // cells beyond the table's ranks: L2 map
      if (active[r] && ent[r] == 0xFFFFu) {
        const int4 q = at(const_cast<int4*>(tb.assoc), 16u * cell[r]);
        srv[r] = q.x;
        full[r] = __hiloint2double(q.w, q.z);
      }
      wait_vmem();
    }
  }
  // per-env histograms in the wave's LDS (bin B: lanes without a station): zero, count, read
  // (16-lane segments of a registered scenario: packed DPP counts instead, row_count_same)
  constexpr bool PCNT = PC == 16 && SCN != 0 && packed_counts_ok(ue_of(UC), SCN ? scn_const(SCN).B : 0);
  int* h[R];
  int bin[R], n[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    h[r] = hist + (r * G + m.seg) * HS;
    bin[r] = srv[r] >= 0 ? srv[r] : B;
    if (!PCNT) h[r][HS >= PC ? u : min(u, B)] = 0;  // (u < PC: one word per lane)
  }
  if (PCNT) {
#pragma unroll
    for (int r = 0; r < R; ++r) n[r] = row_count_same(srv[r]);
  } else {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r)
      __hip_atomic_fetch_add(h[r] + bin[r], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) n[r] = min(h[r][bin[r]], 64);
  }
  float cf[R];
  bool tie[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double r100 = *reinterpret_cast<const double*>(lblob + KPS(lds_r100_off) + 8u * (uint32_t)n[r]);
    // share_cents_r (ResourceFair share + numpy round(., 2)), the tie test in float32
    const double cc = full[r] * r100;
    const double rr = rint(cc);
    const float d = (float)(cc - rr);
    const float rf = (float)rr;
    // (TF: the host showed the product rounds like the reference for every rate and count)
    tie[r] = !TF && srv[r] >= 0 && !(0.5f - fabsf(d) > __builtin_fmaf(rf, 0x1p-46f, 0x1p-25f));
    cf[r] = srv[r] >= 0 ? rf : 0.f;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (bal(tie[r])) {  // rare: within 2^-46 of a half cent -- the reference's two divisions
      if (tie[r]) cf[r] = (float)rint((full[r] / (double)n[r]) * 100.0);
    }
  }
  // ---- E: utility, reward sum, stores -------------------------------------------------------
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float rate_f = cf[r] * 0.01f;
    const float util = active[r] ? (float)utility_f32r<SCN>(cf[r], rate_f, kp) : 0.f;
    const int isum = seg_isum_rows<PC>((int)(util * 0x1p25f));  // (util = 0 where inactive)
    // (every UE active -- registered scenarios: the env's count is U in every lane that stores)
    const int nact = scn_all_active<SCN>() ? U : __popc(seg_field<PC>(act_w[r], m));
    Pending up;
    up.srv = srv[r];
    up.obs = make_float4((float)c[r].pos.x * KPSF(inv_w), (float)c[r].pos.y * KPSF(inv_h),
                         rate_f, util);
    up.ui = (uint32_t)(e[r] * U + u);
    up.valid = valid[r];
    up.lead = up.done = false;
    up.e = 0;
    up.reward = 0.f;
    flush_pending<true, false>(out, up, (uint32_t)kp.E, (uint32_t)(kp.E * U), (uint32_t)row);
    // the env's staged row entry {the 2^-25 fixed-point utility sum, nact | done << 7}, one
    // two-word LDS write; the workgroup's flush forms the float32 reward from them. Lanes other
    // than the env's last write into two words of their env's histogram instead (no branch;
    // re-zeroed next step; min(): never past the env's area)
    const bool lead = klead < nok[r];
    // (reward_risky, rare: the exact reward's float32 bits instead, flag 0x100; the constants
    // from the blob's RewardC)
    const char* rcp = lblob + KPS(lds_r100_off) + 8 * kRewardCSlot;
    const int er = r * G + m.seg;
    int* const hw = h[r] + min(u, PC - 2);
    int* sw = lead ? srow + 2 * er : hw;
    if constexpr (RT1 && scn_all_active<SCN>()) {
      // RT1 (short launches of the scenario instances): |isum| <= T = nact r_thr25 (every UE
      // active: nact = U > 0) as one unsigned compare, (uint)(isum + T) <= 2T (|isum| <= U 2^25
      // and T <= U 2^25: no wrap across the band), its ballot ANDed in SALU with the lanes that
      // store the env rows (u = PC - 1 of the envs that exist: the ballot of `lead` itself costs
      // two VALU), and the risky flag set in the rare branch only. Measured (interleaved, four
      // boxes): 20-step launches at 65,536 large envs 161.5-162.3 vs 165.1-166.3 us, 200-step
      // launches 1.52-1.53 vs 1.48-1.50 ms on three of the boxes (long launches are store-bound,
      // and the cheaper step did not make them faster) -- the host takes it for launches of
      // fewer than 64 steps only
      constexpr uint64_t kLeadPat = [] {
        uint64_t v = 0;
        for (int q = 0; q < 64 / PC; ++q) v |= 1ull << (q * PC + PC - 1);
        return v;
      }();
      int word0 = isum;
      int word1 = nact | ((c[r].t + 1 >= KPS(t_end)) ? 0x80 : 0);
      const uint32_t T = (uint32_t)U * (uint32_t)kp.r_thr25;
      const uint64_t risk_w = bal((uint32_t)isum + T <= 2u * T) & (envok_w[r] & kLeadPat);
      if (risk_w) {
        wait_vmem();  // (no prefetch in flight across the call: see below)
        const RewardC rc = reward_c(rcp);
        const float ex = packed_fix<true, PC>(active[r] ? (double)cf[r] : -1.0, U, u, rc.tab,
                                              rc.kmax, rc.sat, nact);
        if ((risk_w >> __lane_id()) & 1ull) {
          word0 = __float_as_int(ex);
          word1 |= 0x100;
        }
      }
      sw[0] = word0;
      sw[1] = word1;
    } else {
      const bool risky = lead && nact > 0 && (uint32_t)abs(isum) <= (uint32_t)nact * (uint32_t)kp.r_thr25;
      int word0 = isum, flag = 0;
      if (bal(risky)) {
        // (every load landed before the call: the next pair's prefetch registers are not
        // tracked by the compiler, and a callee's save / restore of one in flight would lose its
        // data; tools/check_prefetch_regs.py checks the wait)
        wait_vmem();
        const RewardC rc = reward_c(rcp);
        const float ex = packed_fix<true, PC>(active[r] ? (double)cf[r] : -1.0, U, u, rc.tab,
                                              rc.kmax, rc.sat, nact);
        if (risky) {
          word0 = __float_as_int(ex);
          flag = 0x100;
        }
      }
      sw[0] = word0;
      sw[1] = nact | ((c[r].t + 1 >= KPS(t_end)) ? 0x80 : 0) | flag;
    }
    c[r].t += 1;
  }
}

// ---- Software-pipelined steps (k_steps_lds2 with PIPE: one group per wavefront) ----------------
// A step's movement (lds2_step's phases A-C) depends only on the previous step's movement, its
// outputs (phases D-E) on nothing that comes later. With one wavefront per SIMD (a small batch:
// 4,096 medium envs are 1,024 groups on 1,024 SIMDs) a step is one dependency chain that the SIMD
// waits through instruction by instruction. Iteration i of the pipelined loop moves step i + 1
// and emits step i's outputs: two independent chains in one basic block (the rare paths --
// resets, draws past the episode table -- are uniform branches at the iteration's start, the
// cell entry of step i is read before them), which the scheduler interleaves. Same results as
// lds2_step bit for bit (the same operations per step, in another order across steps).
// What a step's outputs need from its movement (the step's t, before the increment).
struct Snap {
  int2 pos;
  int t;
  bool active, valid;
  uint64_t act_w;
};

// The draw-table word a lane takes in its group's next step if that step neither resets nor
// draws past the table: pair drawn + rank among the lanes without a waypoint (ue_id order),
// read one step ahead (pipe_move issues it after its movement, so the LDS latency passes while
// the previous step's outputs are emitted; the next pipe_move takes it from a register).
template <int UC, int SCN>
__device__ __forceinline__ int pipe_pre(const KParams& kp, const LaneMap& m, const Ctx2& c,
                                        uint64_t valid_w, const int* __restrict__ ltab) {
  constexpr int PC = pitch_of(UC);
  const int M = KPS(tab_m);
  const int t = c.t;
  const bool on = scn_all_active<SCN>() ||
                  (t >= KPS(arr_start) && t < KPS(arr_exit) && (KPS(first_step_active) || t != 0));
  const uint64_t act_w = scn_all_active<SCN>() ? valid_w : bal(on) & valid_w;
  const uint32_t f = seg_field<PC>(bal(c.wp.x == -1) & act_w, m);  // (no waypoint: see lds2_step)
  const int k = c.drawn + __popc(__builtin_amdgcn_ubfe(f, 0u, (uint32_t)m.u));
  return ltab[m.seg * M + min(k, M - 1)];
}

// lds2_step's phases A-C for one group (R = 1): lazy reset, waypoint draws, movement; returns
// the step's snapshot and advances c.t. pre: the lane's pipe_pre word for this step, replaced
// by the next step's.
struct PipeNoMid {
  __device__ void operator()() const {}
};
// mid(): run between the rare branches and the movement (the kernel issues the previous step's
// output reads there, pipe_emit_front; a scheduling barrier keeps them ahead of the movement,
// whose instructions then pass while those LDS reads are in flight).
template <int UC, int SCN, class Mid>
__device__ __forceinline__ Snap pipe_move(const KParams& kp, const KTables& tb, const LaneMap& m,
                                          Ctx2& c, int e, int nok, int kval,
                                          u128* __restrict__ lpcg, const int* __restrict__ ltab,
                                          int& pre, Mid&& mid) {
  constexpr int PC = pitch_of(UC), U = ue_of(UC), G = 64 / PC;
  const int M = KPS(tab_m);
  const int u = m.u;
  constexpr uint64_t kValidPat = [] {
    uint64_t v = 0;
    for (int q = 0; q < 64 / PC; ++q) v |= ((1ull << U) - 1ull) << (q * PC);
    return v;
  }();
  int nk = nok;
  asm volatile("" : "+s"(nk));
  const uint64_t envok_w = nk >= G ? ~0ull : ((1ull << (uint32_t)(nk * PC)) - 1ull);
  const uint64_t valid_w = envok_w & kValidPat;
  const bool env_ok = m.seg < nk;
  const int er = m.seg;
  const bool valid = kval < nok;
  // ---- A: lazy auto-reset (base.py:288-291) ----
  const bool reset_env = env_ok && c.t >= KPS(t_end);
  const bool do_reset = reset_env && valid;
  const uint64_t rs_w = bal(c.t >= KPS(t_end)) & envok_w;
  if (rs_w) {
    if (reset_env) {
      c.t = 0;
      c.drawn = U;
    }
    if (do_reset) {
      const int p = ltab[er * M + u];
      c.pos = make_int2((int)(short)p, p >> 16);
      c.wp = make_int2(-1, -1);
    }
    if (PC == 16) pre = pipe_pre<UC, SCN>(kp, m, c, valid_w, ltab);  // (the reset moved drawn and the waypoints)
  }
  const int t = c.t;
  const bool on = scn_all_active<SCN>() ||
                  (t >= KPS(arr_start) && t < KPS(arr_exit) && (KPS(first_step_active) || t != 0));
  const bool active = valid && on;
  const uint64_t act_w = scn_all_active<SCN>() ? valid_w : bal(on) & valid_w;
  const bool nowp = c.wp.x == -1;  // (no waypoint: see lds2_step)
  const bool need = active && nowp;
  const uint64_t mneed_w = bal(nowp) & act_w;
  const uint32_t f = seg_field<PC>(mneed_w, m);
  const int tot = __popc(f);
  const int rank = __popc(__builtin_amdgcn_ubfe(f, 0u, (uint32_t)u));
  const int k = c.drawn + rank;
  // ---- B: waypoint draws in ue_id order (movement.py:44-47) ----
  // every draw of the group inside the episode table: the common, branch-free path below;
  // else (rare) every drawing lane from the stream state, as lds2_step's fallback
  const uint64_t fb_w = bal(k >= M) & mneed_w;
  const bool past = need && k >= M;
  if (fb_w) {  // (rare) lanes drawing past the table: as lds2_step
    u128* const slot = lpcg + 2 * er;
    const u128 inc = slot[1];
    u128 s = slot[0];
    if (c.drawn > 0 && c.drawn <= M) {
      s = at(const_cast<u128*>(tb.tab_st),
             16u * ((uint32_t)e * (uint32_t)M + (uint32_t)(c.drawn - 1)));
      wait_vmem();
    }
    u128 s_fin = 0;
    if ((bal(rank != 0) & bal(past)) == 0) {
      if (past) s_fin = pcg_draw_pair_next(s, inc, kp.Wd, kp.Hd, c.wp.x, c.wp.y);
    } else {
      if (past) s_fin = pcg_draw_pair(s, inc, 2 * rank, tb.jump, kp.Wd, kp.Hd, c.wp.x, c.wp.y);
    }
    wait_vmem();
    if (past && rank == tot - 1) slot[0] = s_fin;
  }
  mid();
  if constexpr (!std::is_same_v<std::decay_t<Mid>, PipeNoMid>) __builtin_amdgcn_sched_barrier(0);
  {  // the table's pair (16-lane segments: read a step ahead, pipe_pre), taken where a table
     // draw is due
    const bool take = need && !past;
    const int p = PC == 16 ? pre : ltab[er * M + min(k, M - 1)];
    c.wp = take ? make_int2((int)(short)p, p >> 16) : c.wp;
  }
  c.drawn += tot;
  // ---- C: movement (movement.py:49-62) ----
  constexpr bool AXF = SCN != 0;
  constexpr bool V15 = scn_v15<SCN>();
  const int2 pos = c.pos, wp = c.wp;
  const int dx = wp.x - pos.x, dy = wp.y - pos.y;
  const int ax2 = __mul24(dx, dx), ay2 = __mul24(dy, dy);
  const int d2 = ax2 + ay2;
  const bool arrive = d2 <= KPS(d2snap);
  int2 npos;
  if (V15 || KPS(axis_exact) == 2) {
    int2 np = step_v15_mad(pos, dx, dy, ax2, ay2);
    asm volatile("" : "+v"(np.x), "+v"(np.y));  // (a select, not a branch on `arrive`)
    npos = arrive ? wp : np;
  } else {
    const float sc = KPSF(vel_f) * __builtin_amdgcn_rsqf((float)d2);
    const float qx = (float)dx * sc, qy = (float)dy * sc;
    const float rx = rintf(qx), ry = rintf(qy);
    const bool axis = dx == 0 || dy == 0;
    bool ok = fmaxf(fabsf(qx - rx), fabsf(qy - ry)) < KPSF(move_lim);
    int2 np = make_int2(pos.x + (int)rx, pos.y + (int)ry);
    if (AXF) {
      const float vs = KPSF(vel_f);
      const int ax = (int)rintf((float)pos.x + (dx > 0 ? vs : -vs));
      const int ay = (int)rintf((float)pos.y + (dy > 0 ? vs : -vs));
      if (axis) np = dy == 0 ? make_int2(ax, pos.y) : make_int2(pos.x, ay);
      ok = ok || axis;
    }
    const bool xneed = active && !arrive && !ok;
    if (bal(xneed)) {
      if (xneed) np = move_exact(pos, dx, dy, kp.vel);
    }
    npos = arrive ? wp : np;
  }
  const bool pop = active && arrive;
  c.pos = active ? npos : c.pos;
  c.wp = pop ? make_int2(-1, -1) : c.wp;
  Snap sn;
  sn.pos = c.pos;
  sn.t = t;
  sn.active = active;
  sn.valid = valid;
  sn.act_w = act_w;
  c.t = t + 1;
  // the next step's draw word, in flight from here (32-lane segments read it in the step: 212
  // vs 207 us per 200-step launch at 8,192 large envs with it read ahead)
  if (PC == 16) pre = pipe_pre<UC, SCN>(kp, m, c, valid_w, ltab);
  return sn;
}

// The cell entry of a snapshot's position (mode-3 LDS table), read ahead of the next move.
template <int UC, int SCN>
__device__ __forceinline__ uint32_t pipe_cell(const KParams& kp, const Snap& sn,
                                              const char* __restrict__ lblob) {
  const uint32_t cell = min(__umul24((uint32_t)sn.pos.y, (uint32_t)KPS(W)) + (uint32_t)sn.pos.x,
                            (uint32_t)(KPS(W) * KPS(H) - 1));
  return *reinterpret_cast<const uint16_t*>(lblob + 2u * cell);
}

// lds2_step's phases D-E for one group from its snapshot and cell entry. The layout has no
// cell beyond the table's ranks (0xFFFF; the host selects PIPE only when |D| <= 4,094).
// Split in two around the next step's movement: the front issues the LDS reads (the full rate
// at the cell's rank, 100 / n after the station counts), the back waits for them and finishes.
struct EmitF {
  double full, r100;
  int srv, n;
};
template <int UC, int SCN>
__device__ __forceinline__ EmitF pipe_emit_front(const KParams& kp, const LaneMap& m,
                                                 const Snap& sn, uint32_t ent,
                                                 const char* __restrict__ lblob,
                                                 int* __restrict__ hist) {
  constexpr int PC = pitch_of(UC), G = 64 / PC;
  const int B = KPS(B), HS = lds2_hist_stride(G, B);
  const int u = m.u;
  EmitF f;
  f.full = *reinterpret_cast<const double*>(lblob + KPS(lds_rate_off) + 8u * (ent & 4095u));
  f.srv = sn.active && ent < 0xF000u ? (int)(ent >> 12) : -1;
  constexpr bool PCNT = PC == 16 && SCN != 0 && packed_counts_ok(ue_of(UC), SCN ? scn_const(SCN).B : 0);
  int* const h = hist + m.seg * HS;
  if (PCNT) {
    f.n = row_count_same(f.srv);
  } else {
    const int bin = f.srv >= 0 ? f.srv : B;
    h[HS >= PC ? u : min(u, B)] = 0;
    __builtin_amdgcn_wave_barrier();
    __hip_atomic_fetch_add(h + bin, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __builtin_amdgcn_wave_barrier();
    f.n = min(h[bin], 64);
  }
  f.r100 = *reinterpret_cast<const double*>(lblob + KPS(lds_r100_off) + 8u * (uint32_t)f.n);
  return f;
}

template <int UC, int SCN, bool TF>
__device__ __forceinline__ void pipe_emit_back(const KParams& kp, const KOut& out,
                                               const LaneMap& m, const Snap& sn, const EmitF& f,
                                               int e, int nok, int klead, int row,
                                               int* __restrict__ hist, int* __restrict__ srow) {
  constexpr int PC = pitch_of(UC), U = ue_of(UC), G = 64 / PC;
  const int B = KPS(B), HS = lds2_hist_stride(G, B);
  const int u = m.u;
  int* const h = hist + m.seg * HS;
  const double full = f.full, r100 = f.r100;
  const int srv = f.srv, n = f.n;
  (void)n;
  (void)B;
  const double cc = full * r100;
  const double rr = rint(cc);
  const float d = (float)(cc - rr);
  const float rf = (float)rr;
  const bool tie = !TF && srv >= 0 && !(0.5f - fabsf(d) > __builtin_fmaf(rf, 0x1p-46f, 0x1p-25f));
  float cf = srv >= 0 ? rf : 0.f;
  if (!TF && bal(tie)) {
    if (tie) cf = (float)rint((full / (double)n) * 100.0);
  }
  const float rate_f = cf * 0.01f;
  const float util = sn.active ? (float)utility_f32r<SCN>(cf, rate_f, kp) : 0.f;
  const int isum = seg_isum_rows<PC>((int)(util * 0x1p25f));
  const int nact = scn_all_active<SCN>() ? U : __popc(seg_field<PC>(sn.act_w, m));
  Pending up;
  up.srv = srv;
  up.obs = make_float4((float)sn.pos.x * KPSF(inv_w), (float)sn.pos.y * KPSF(inv_h), rate_f, util);
  up.ui = (uint32_t)(e * U + u);
  up.valid = sn.valid;
  up.lead = up.done = false;
  up.e = 0;
  up.reward = 0.f;
  flush_pending<true, false>(out, up, (uint32_t)kp.E, (uint32_t)(kp.E * U), (uint32_t)row);
  const bool lead = klead < nok;
  // (reward_risky: tested by the flush, flush_staged2<true> -- a branch here, on the pipelined
  // loop's path, cost 9 % at 4,096 medium envs)
  int* const hw = h + min(u, PC - 2);  // (see lds2_step)
  int* sw = lead ? srow + 2 * m.seg : hw;
  sw[0] = isum;
  sw[1] = nact | ((sn.t + 1 >= KPS(t_end)) ? 0x80 : 0);
}

// The staged rows of k_steps_lds2: reward = (float)isum 2^-25 / nact (float32, as packed_group's
// lean path), or the utility's lower bound without active UEs; done = bit 7.
// Workgroup barrier for LDS data: this wave's LDS operations complete (lgkmcnt(0)), then
// s_barrier; compiler-only fences keep the LDS accesses on their side. Unlike __syncthreads no
// memory-model fence: its release could also wait for the wave's global stores in flight
// (vmcnt(0), seen in the generated code), a drain of the trajectory stores at every flush.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only (vmcnt 63, expcnt 7: no wait)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// `trailing`: a second barrier after the reads, before the window's slots are written again
// (not needed when consecutive pairs alternate between two windows: the next write of this
// window follows the next flush's first barrier, which every reader here has passed).
// The flush's rare fix-up (see flush_staged2).
MEV_GUARD_FN void flush_fix(const int* srow, const float* obs_f, float* rew, const char* rc, int E,
                            int e0, int row0, int nr, int NWG, int U) {
  const float inv_nwg = 1.0f / (float)NWG;
  const RewardC c = reward_c(rc);
#pragma unroll 1
  for (int q = threadIdx.x; q < nr * NWG; q += (int)blockDim.x) {
    const int r = (int)(((float)q + 0.5f) * inv_nwg), j = q - r * NWG;
    if (e0 + j >= E) continue;
    const int2 v = *reinterpret_cast<const int2*>(srow + 2 * q);
    const uint32_t b = (uint32_t)v.y;
    const int nact = (int)(b & 0x7fu);
    if ((b & 0x100u) || !(nact > 0 && (uint32_t)abs(v.x) <= (uint32_t)nact * (uint32_t)c.thr25))
      continue;
    const float* rates = obs_f + 4 * ((size_t)(row0 + r) * (size_t)E + (size_t)(e0 + j)) * (size_t)U + 2;
    long long su = 0;
#pragma unroll 1
    for (int u = 0; u < U; ++u) su += util_fix50c(rint((double)rates[4 * u] * 100.0), c);
    rew[(size_t)(row0 + r) * (size_t)E + (size_t)(e0 + j)] = exact_mean50(su, nact);
  }
}

// DETECT (the pipelined loop, whose steps do not test reward_risky): the flush tests every row's
// fixed-point sum, and if any row of the workgroup's window is risky (block-uniform, one
// __syncthreads_or per flush) re-forms those rows' rewards from the exact utilities of the
// window's obs rates (every wave's stores made visible by a fenced barrier first; cents =
// rint(100 rate) exactly below 6e6, every table index is below 2^22; the env's UEs are all
// active or none, nact = U or 0). U: UEs per env.
template <bool DETECT = false>
__device__ __forceinline__ void flush_staged2(const KOut& out, const int* srow, int E, int e0,
                                              int row0, int nr, float lower, int NWG,
                                              bool trailing = true, const char* rc = nullptr,
                                              int U = 0) {
  lds_barrier();
  const float inv_nwg = 1.0f / (float)NWG;
  bool any = false;
  // (the same test as the two-group and packed steps' in-step one -- the integer compare of the
  // 2^-25 sum against nact r_thr25 -- so every kernel shape sends the same rows to the exact path)
  const uint32_t thr25 = DETECT ? *reinterpret_cast<const uint32_t*>(rc + 28) : 0u;
  for (int q = threadIdx.x; q < nr * NWG; q += (int)blockDim.x) {
    // q / NWG through float (q + 1/2 is >= 1/2 away from a multiple of NWG; exact for q < 2^22)
    const int r = (int)(((float)q + 0.5f) * inv_nwg), j = q - r * NWG;
    if (e0 + j < E) {
      const size_t ro = (size_t)(row0 + r) * (size_t)E;
      const uint32_t o = (uint32_t)(e0 + j);
      // {isum, nact | done << 7}, or {the exact reward's bits, ... | 0x100} (reward_risky)
      const int2 v = *reinterpret_cast<const int2*>(srow + 2 * q);
      const uint32_t b = (uint32_t)v.y;
      const int nact = (int)(b & 0x7fu);
      at(out.reward + ro, 4u * o) =
          (b & 0x100u) ? __int_as_float(v.x)
                       : nact > 0 ? (float)v.x * 0x1p-25f * __builtin_amdgcn_rcpf((float)nact) : lower;
      at(out.done + ro, o) = (uint8_t)((b >> 7) & 1u);
      if (DETECT)
        any = any || (!(b & 0x100u) && nact > 0 && (uint32_t)abs(v.x) <= (uint32_t)nact * thr25);
    }
  }
  if (DETECT && __syncthreads_or(any)) {  // rare
    __syncthreads();  // (fenced: the window's obs stores of every wave visible)
    const float* obs_f = reinterpret_cast<const float*>(out.obs);
    float* rew = out.reward;
    asm volatile("" : "+s"(obs_f), "+s"(rew));
    wait_vmem();  // (see lds2_step: no prefetch in flight across the call)
    flush_fix(srow, obs_f, rew, rc, E, e0, row0, nr, NWG, U);
  }
  if (trailing) lds_barrier();
}

// Dev builds only (-DMEV_TIMING, tools/ts_probe.py): per-wave timestamps of k_steps_lds2's
// phases (s_memrealtime, 100 MHz) into a buffer set by mev_debug_timestamps.
#ifdef MEV_TIMING
__device__ uint64_t* g_mev_ts;
#define MEV_TS(k)                                                                         \
  do {                                                                                    \
    if (g_mev_ts && lane == 0)                                                            \
      g_mev_ts[(size_t)(blockIdx.x * NW + wv) * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define MEV_CLK(k)                                                                        \
  do {                                                                                    \
    if (g_mev_ts && lane == 0)                                                            \
      g_mev_ts[(size_t)(blockIdx.x * NW + wv) * 32 + (k)] = __builtin_amdgcn_s_memtime();  \
  } while (0)
// the wave's HW_ID (CU / SIMD / shader engine) and XCC_ID registers
#define MEV_HWID(k)                                                                       \
  do {                                                                                    \
    if (g_mev_ts && lane == 0) {                                                          \
      g_mev_ts[(size_t)(blockIdx.x * NW + wv) * 32 + (k)] = __builtin_amdgcn_s_getreg(0xF804); \
      g_mev_ts[(size_t)(blockIdx.x * NW + wv) * 32 + (k) + 1] = __builtin_amdgcn_s_getreg(0xF814); \
    }                                                                                     \
  } while (0)
#else
#define MEV_TS(k) \
  do {            \
  } while (0)
#define MEV_CLK(k) \
  do {             \
  } while (0)
#define MEV_HWID(k) \
  do {              \
  } while (0)
#endif

// A pair's inputs (k_steps_lds2), loaded into registers one pair ahead: issued when the wave
// starts a pair, consumed when it starts the next, so their HBM latency hides behind the
// current pair's steps. (Loaded at the pair's start instead, every wave of the chip waited for
// them at the same moment -- the pairs of all waves start together, the workgroup flush being
// a barrier -- four times per launch, ~3 us each.) Registers, not LDS-DMA: an LDS-DMA in
// flight makes the compiler wait for it (vmcnt) before every later LDS access of the wave.
template <int R, int NT, int NK>
struct Pre2 {
  v2u32 s[R];   // the lane's UE row {x, y, wx, wy} (int16x4) in each group
  int s8[R];    // the same in the compact form (uint8x4, KParams::st8)
  int t, d, c;  // lanes [0, R G): t, drawn and (per-env layouts) the station count of env slot
                // `lane` (each from a wave-uniform base: no per-lane pointer kept live)
  v2u32 pc;     // lanes [0, 4 R G): word lane & 3 of {state, inc} of env slot lane >> 2
  int tab[NT];  // words q * 64 + lane of the pair's episode draw tables [R G][M]
  v2u32 bq[NK]; // (per-env layouts) station (slot, k) = (i >> 4, i & 15), i = q * 64 + lane
};

// Words of the pair's draw tables per lane: R G M / 64 (scenario instances), else at most 8
// (the host selects k_steps_lds2 only when R G M <= 512).
template <int UC, int SCN, int R>
__host__ __device__ constexpr int lds2_pre_words() {
  return SCN ? (R * (64 / pitch_of(UC)) * scn_const(SCN).tab_m + 63) / 64 : 8;
}

// The prefetch loads are inline assembly, i.e. invisible to the compiler's wait-count
// bookkeeping: tracked, their use one pair later got a compiler wait counted from the shortest
// path (one step), vmcnt(~18) -- and since vmcnt retires loads and stores in issue order, that
// waited for every trajectory store more than ~18 instructions back, ~5 us at each pair
// boundary of a write-bound launch (tools/ts_probe.py). lds2_consume waits for them explicitly
// (lds2_pf_wait): after >= 63 younger VMEM instructions (nsteps >= 14: four unconditional
// trajectory stores per step, eight state stores per pair) vmcnt(63) -- which only waits for
// instructions at least 63 back, and the counter never exceeds 63 -- else vmcnt(0). The
// registers stay untouched in between (tied to the wait by "+v"; checked on the generated
// assembly by tools/check_prefetch_regs.py: no copy, no spill).
__device__ __forceinline__ int pf_b32(const void* p) {
  int v;
  asm volatile("global_load_dword %0, %1, off ; mev-prefetch" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ v2u32 pf_b64(const void* p) {
  v2u32 v;
  asm volatile("global_load_dwordx2 %0, %1, off ; mev-prefetch" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
template <class T>
__device__ __forceinline__ void pf_tie(T& x) {
  asm volatile("; mev-prefetch-wait %0" : "+v"(x));
}
template <int R, int NT, int NK, bool PE>
__device__ __forceinline__ void lds2_pf_wait(Pre2<R, NT, NK>& f, bool saturated, bool st8) {
  if (saturated) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (st8) pf_tie(f.s8[r]);
    else pf_tie(f.s[r]);
  }
  pf_tie(f.t);
  pf_tie(f.d);
  if (PE) pf_tie(f.c);
  pf_tie(f.pc);
#pragma unroll
  for (int q = 0; q < NT; ++q) pf_tie(f.tab[q]);
  if (PE) {
#pragma unroll
    for (int q = 0; q < NK; ++q) pf_tie(f.bq[q]);
  }
}

template <int UC, int SCN, int R, bool PE, int NT, int NK, bool C8>
__device__ __forceinline__ void lds2_prefetch(const KParams& kp, const KState& st,
                                              const KTables& tb, const LaneMap& m, int lane,
                                              int p, Pre2<R, NT, NK>& f) {
  constexpr int PC = pitch_of(UC), G = 64 / PC, U = ue_of(UC), RG = R * G;
  const int M = KPS(tab_m);
  const int e0 = p * RG, elast = kp.E - 1;  // the pair's envs [e0, e0 + R G), clamped
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int ec = min(e0 + r * G + m.seg, elast);
    const uint32_t ui = (uint32_t)(ec * U + min(m.u, U - 1));
    if (C8) f.s8[r] = pf_b32(reinterpret_cast<const unsigned*>(st.ue_state) + ui);
    else f.s[r] = pf_b64(st.ue_state + ui);
  }
  const int ej = min(e0 + min(lane, RG - 1), elast);
  f.t = pf_b32(st.t + ej);
  f.d = pf_b32(tb.drawn + ej);
  if (PE) f.c = pf_b32((st.bs_count ? st.bs_count : st.t) + ej);  // (no count array: B, below)
  const int ep = min(e0 + min(lane >> 2, RG - 1), elast);
  f.pc = pf_b64(reinterpret_cast<const char*>(st.pcg) + 48u * (uint32_t)ep + 8u * (uint32_t)(lane & 3));
  const int lim = max(1, min(RG * M, (kp.E - e0) * M));
  const int* src = tb.tab_xy + (size_t)e0 * M;
#pragma unroll
  for (int q = 0; q < NT; ++q) f.tab[q] = pf_b32(src + min(q * 64 + lane, lim - 1));
  if (PE) {
#pragma unroll
    for (int q = 0; q < NK; ++q) {
      const int i = q * 64 + lane;
      const int es = min(e0 + (i >> 4), elast), k = min(i & 15, KPS(B) - 1);
      f.bq[q] = pf_b64(st.bs_xy + ((size_t)es * KPS(B) + k));
    }
  }
}

// The prefetched inputs into the pair's contexts and the wave's LDS (draw tables, stream
// slots, per-env station keys; t / drawn / counts through `scratch`, a free histogram area).
template <int UC, int SCN, int R, bool PE, int NT, int NK, bool C8>
__device__ __forceinline__ void lds2_consume(const KParams& kp, const KState& st, const LaneMap& m,
                                             int lane, int p, Pre2<R, NT, NK>& f, bool saturated,
                                             Ctx2 (&c)[R], int* __restrict__ ltab,
                                             u128* __restrict__ lpcg, int* __restrict__ scratch,
                                             int* __restrict__ lkeys) {
  constexpr int PC = pitch_of(UC), G = 64 / PC, RG = R * G;
  const int M = KPS(tab_m);
  lds2_pf_wait<R, NT, NK, PE>(f, saturated, C8);
  const int lim = max(1, min(RG * M, (kp.E - p * RG) * M));
  // Unconditional stores (no branch: the compiler laid guarded ones out of line, past the code
  // tools/check_prefetch_regs.py scans): a lane past the end writes the slot whose value it
  // loaded (lds2_prefetch clamps the same way), a duplicate of the same value.
#pragma unroll
  for (int q = 0; q < NT; ++q) ltab[min(q * 64 + lane, lim - 1)] = f.tab[q];
  reinterpret_cast<v2u32*>(lpcg)[min(lane >> 2, RG - 1) * 4 + (lane & 3)] = f.pc;
  {
    const int j = min(lane, RG - 1);
    scratch[j] = f.t;
    scratch[RG + j] = f.d;
    // (the station count: 0 for slots past the batch's last env)
    if (PE) scratch[2 * RG + j] = p * RG + j < kp.E ? (st.bs_count ? f.c : KPS(B)) : 0;
  }
  __builtin_amdgcn_wave_barrier();
  if (PE) {
    // the env's station keys, 16 slots per env, {m = -16 q (int16x2), c = ((|q|^2 + 2^21) << 4)
    // | k}: the key of station k for a UE at p is dot2(2 p, m) + c (see k_steps_packed); slots
    // past the env's count hold {0, UINT_MAX}, a key that never wins
#pragma unroll
    for (int q = 0; q < NK; ++q) {
      const int i = q * 64 + lane, slot = i >> 4, k = i & 15;
      int2 kv = make_int2(0, -1);
      if (k < scratch[2 * RG + slot]) {
        const int2 bq = make_int2((int)f.bq[q].x, (int)f.bq[q].y);
        const s16x2 m2 = {(short)(-16 * bq.x), (short)(-16 * bq.y)};
        kv = make_int2(__builtin_bit_cast(int, m2),
                       (int)(((unsigned)(bq.x * bq.x + bq.y * bq.y + (1 << 21)) << 4) | (unsigned)k));
      }
      *reinterpret_cast<int2*>(lkeys + slot * 32 + 2 * k) = kv;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int slot = r * G + m.seg;
    c[r].t = scratch[slot];
    c[r].drawn = scratch[RG + slot];
    // the stream slot holds the env's state only after draws past the table (mev_state.pcg)
    c[r].fl = c[r].drawn > M ? kSok : 0;
    if (C8) {
      const int4 q = unpack8((unsigned)f.s8[r]);
      c[r].pos = make_int2(q.x, q.y);
      c[r].wp = make_int2(q.z, q.w);
    } else {
      const int2 v = make_int2((int)f.s[r].x, (int)f.s[r].y);
      c[r].pos = make_int2((int)(short)v.x, v.x >> 16);
      c[r].wp = make_int2((int)(short)v.y, v.y >> 16);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// LDS of k_steps_lds2 per wave: stream slots [R G][2] u128, (PE) station keys [R G][16][2] int,
// histograms [R G][HS] int, draw tables [R G][M] int. HS = max(B + 1, P): with a bin per lane
// of the segment, the per-step zeroing and the non-leader lanes' dummy row writes go to
// distinct words (at HS = B + 1 the lanes past B all hit bin B: same-word LDS writes)
__host__ __device__ inline size_t lds2_per_wave(int G, int B, int M, int R, bool PE = false) {
  return sizeof(int) * (size_t)(R * G) *
         (8 + (PE ? 32 : 0) + (size_t)lds2_hist_stride(G, B) + (size_t)M);
}

// PE: per-env station layouts (KParams::lds_mode 4: the blob holds the rank index of S, 100/n
// and rate_full over S; the env's station keys are staged per launch like k_steps_packed's)
// R = 2 env groups per wavefront; R = 1 (batches too small to fill the resident workgroups
// with pairs: one group per wavefront, the same step code).
// C8: the compact UE state form (KParams::st8) as a compile-time property of the instance (the
// prefetch registers of one form only: a runtime choice kept both sets live, and spilled them)
// PIPE: the software-pipelined step loop (pipe_move / pipe_emit; R = 1, shared layout, a layout
// without cells beyond the mode-3 table's ranks)
// HET: heterogeneous entities, shared layout (lds2_step's HET; the generic instance only)
template <int UC, int SCN, bool PE = false, bool TF = false, int R = 2, bool C8 = scn_st8(SCN),
          bool PIPE = false, bool HET = false, bool RT1 = false>
__global__ __launch_bounds__(64 * kLds2Waves) void k_steps_lds2(
    KParams kp, KState st, KOut out, KTables tb, int ngroups, int nsteps, int traj,
    int stage_rows) {
  const int NW = (int)(blockDim.x >> 6);  // <= kLds2Waves
  constexpr int PC = pitch_of(UC), G = 64 / PC, U = ue_of(UC);
  const int NWG = NW * G * R;  // envs per workgroup tile
  extern __shared__ int lds_all[];
  const char* lblob = reinterpret_cast<const char*>(lds_all);
  const int M = KPS(tab_m), B = KPS(B);
  const int wv = threadIdx.x >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int lane = threadIdx.x & 63;
  const LaneMap m = lane_map<PC>(lane, PC);
  int* lw = lds_all + (KPS(lds_assoc) >> 2);
  constexpr int KB = PE ? 32 : 0;  // ints per env of staged station keys
  u128* lpcg = reinterpret_cast<u128*>(lw) + wv * R * G * 2;
  int* lkeys = lw + NW * R * G * 8 + wv * R * G * KB;
  const int HS = lds2_hist_stride(G, B);
  int* hist = lw + NW * R * G * (8 + KB) + wv * R * G * HS;
  int* ltab = lw + NW * R * G * (8 + KB + HS) + wv * R * G * M;
  int* srow = lw + NW * R * G * (8 + KB + HS + M);  // staged rows [stage_rows][NWG] int2
  const int npairs = (ngroups + R - 1) / R;  // ("pairs": the wave's R groups)
  const int gstride = (int)gridDim.x * NW;
  const float lower = (float)kp.lower;
  const int pb0 = block_slot(kp.xcd_remap) * NW;
  static_assert(!HET || (SCN == 0 && !PE && !PIPE), "HET: the generic shared-layout instance");
  // (HET) this lane's UE class and movement parameters, for the launch
  // (the class and movement parameters packed: three registers, move_ue_pc)
  uint32_t hpk = 0;
  float hvf = 0.f, hml = 0.f;
  if (HET) {
    const MoveP mv = tb.mv[min(m.u, U - 1)];
    hpk = ((uint32_t)mv.d2snap << 8) | ((uint32_t)mv.axis_exact << 4) | (uint32_t)tb.ue_cls[min(m.u, U - 1)];
    hvf = mv.vel_f;
    hml = mv.move_lim;
  }
  constexpr int NT = lds2_pre_words<UC, SCN, R>();
  constexpr int NK = PE ? (R * G * 16 + 63) / 64 : 1;
  Pre2<R, NT, NK> f;  // the inputs of the wave's next pair
  Ctx2 c[R];
  MEV_TS(0);
  MEV_CLK(25);
  MEV_HWID(23);
  {  // the tables (LDS-DMA, wave w moves 1 KB pieces w, w + NW, ...) and the first pair's
     // inputs, issued together before one wait (before the pair loop: a wait inside it would
     // leave the compiler unsure the copy is done, and it would wait before LDS accesses)
    const int n16 = blob_copy_n16<SCN>(kp, tb);
    for (int q = wv; q * 64 < n16; q += NW)
      if (q * 64 + lane < n16) glds(tb.lds_blob + q * 64 + lane, reinterpret_cast<int4*>(lds_all) + q * 64);
    if (pb0 + wvu < npairs) lds2_prefetch<UC, SCN, R, PE, NT, NK, C8>(kp, st, tb, m, lane, pb0 + wvu, f);
    wait_vmem();
    __syncthreads();
    MEV_TS(1);
    if (pb0 + wvu < npairs)
      lds2_consume<UC, SCN, R, PE, NT, NK, C8>(kp, st, m, lane, pb0 + wvu, f, false, c, ltab, lpcg,
                                           hist, lkeys);
    MEV_TS(2);
  }
  // Software pipeline over the workgroup's pair tiles: iteration k issues the loads of the wave's
  // pair of tile k + 1, runs its pair of tile k (steps, state stores), then moves the next
  // pair's inputs into the contexts / LDS (lds2_consume) and flushes tile k's staged rows. The
  // prefetched registers are never carried around a loop edge (a copy there would read them
  // before the loads land, tools/check_prefetch_regs.py). Every store between a prefetch and
  // its wait is unconditional -- the trajectory rows of every step, the state's buffer stores
  // below -- so that 2R nsteps + 4R >= 64 of them make the wait free (vmcnt(63)).
  // Staged per-env rows: a pair whose steps fit twice in the window alternates between its two
  // halves (one barrier per flush), else the window cycles: stage_rows < 0 (the two-group
  // launches) -- two windows of -stage_rows rows, filled in turn, so that a flush needs only its
  // leading barrier (the other window is written meanwhile; a window is written again only
  // after the next flush's barrier, which every reader of its last flush has passed), and a pair
  // starts in the window after the one its predecessor flushed last; else one window and two
  // barriers per flush (the trailing one before the window is written again).
  const bool dbl = stage_rows < 0;
  if (dbl) stage_rows = -stage_rows;
  const bool alt = 2 * nsteps <= stage_rows;
  int hcur = 0;  // (dbl) the window being filled
  const bool saturated = 2 * R * nsteps + 4 * R >= 64;  // (2R trajectory stores per step, 4R state)
  int hb = 0;  // the pair's first row slot (alt)
  const bool leader = m.u == PC - 1;
  const int kval = m.u < U ? m.seg : 99, klead = m.u == PC - 1 ? m.seg : 99;
  const uint32_t bst = (C8 ? 4u : 8u) * (uint32_t)(kp.E * U), bt = 4u * (uint32_t)kp.E;
  int it = 0;  // (MEV_TIMING)
  (void)it;
  for (int pb = pb0; pb < npairs; pb += gstride) {
    const int p = pb + wvu, pn = p + gstride;  // this wave's current / next pair
    const bool cur_ok = p < npairs, nxt_ok = pn < npairs;
    if (nxt_ok) lds2_prefetch<UC, SCN, R, PE, NT, NK, C8>(kp, st, tb, m, lane, pn, f);
    int* const sw = srow + 2 * hb * NWG;
    const int e0 = pb * G * R;  // the current tile's first env
    const int wrows = stage_rows * NWG;  // (dbl) ints / 2 per window
    if (cur_ok) {
      int e[R], nok[R];
      bool env_ok[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int g = R * p + r;
        e[r] = g * G + m.seg;
        env_ok[r] = (m.seg < G) && (e[r] < kp.E);
        nok[r] = __builtin_amdgcn_readfirstlane(min(max(kp.E - g * G, 0), G));  // envs that exist
      }
      // the pair's steps; a pair whose envs all exist (every pair but the batch's last partial
      // one) runs the FULL step: constant env masks
      auto steps = [&](auto full) {
        int i = 0, sr = 0;
        do {  // (nsteps >= 1: the loop body runs at least once)
          int* const win = sw + (dbl ? 2 * hcur * wrows : 0);
          lds2_step<UC, SCN, R, PE, TF, decltype(full)::value, HET, RT1>(
              kp, st, out, tb, m, c, e, nok, kval, klead, traj ? i : 0, lblob, lpcg, hist, ltab,
              win + 2 * (sr * NWG + wvu * G * R), lkeys, hpk, hvf, hml);
          if (!alt && (sr + 1 == stage_rows || i + 1 == nsteps)) {
            flush_staged2(out, win, kp.E, e0, traj ? i - sr : 0, sr + 1, lower, NWG, !dbl);
            if (dbl) hcur ^= 1;
          }
          ++i;
          sr = sr + 1 == stage_rows ? 0 : sr + 1;
        } while (i < nsteps);
      };
      if constexpr (PIPE) {
        static_assert(R == 1 && !PE, "PIPE: one group per wavefront, a shared layout");
        // iteration i: the cell entry of step i, the move of step i + 1, the outputs of step i
        constexpr uint64_t kVP = [] {
          uint64_t v = 0;
          for (int q = 0; q < G; ++q) v |= ((1ull << U) - 1ull) << (q * PC);
          return v;
        }();
        int nk0 = nok[0];
        asm volatile("" : "+s"(nk0));
        int pre = PC != 16 ? 0 : pipe_pre<UC, SCN>(
            kp, m, c[0], (nk0 >= G ? ~0ull : ((1ull << (uint32_t)(nk0 * PC)) - 1ull)) & kVP, ltab);
        Snap sn = pipe_move<UC, SCN>(kp, tb, m, c[0], e[0], nok[0], kval, lpcg, ltab, pre, PipeNoMid{});
        // 16-lane segments (medium: packed DPP counts) issue the outputs' LDS reads before the
        // next movement and wait for them after it (108.5 vs 116 us per 200-step launch at 4,096
        // medium envs); 32-lane segments (the LDS histogram's atomics) emit after the movement
        constexpr bool SPLIT = PC == 16;
        int i = 0, sr = 0;
        auto emit = [&](const Snap& q, const EmitF& ef) {
          pipe_emit_back<UC, SCN, TF>(kp, out, m, q, ef, e[0], nok[0], klead, traj ? i : 0,
                                      hist, sw + 2 * (sr * NWG + wvu * G));
          if (!alt && (sr + 1 == stage_rows || i + 1 == nsteps))
            flush_staged2<true>(out, sw, kp.E, e0, traj ? i - sr : 0, sr + 1, lower, NWG, true,
                                lblob + KPS(lds_r100_off) + 8 * kRewardCSlot, U);
          ++i;
          sr = sr + 1 == stage_rows ? 0 : sr + 1;
        };
        while (i + 1 < nsteps) {  // (emit advances i)
          const uint32_t ent = pipe_cell<UC, SCN>(kp, sn, lblob);
          if constexpr (SPLIT) {
            EmitF ef;
            const Snap nx = pipe_move<UC, SCN>(
                kp, tb, m, c[0], e[0], nok[0], kval, lpcg, ltab, pre,
                [&] { ef = pipe_emit_front<UC, SCN>(kp, m, sn, ent, lblob, hist); });
            __builtin_amdgcn_sched_barrier(0);  // (the movement ahead of the front's waits)
            emit(sn, ef);
            sn = nx;
          } else {
            const Snap nx = pipe_move<UC, SCN>(kp, tb, m, c[0], e[0], nok[0], kval, lpcg, ltab,
                                               pre, PipeNoMid{});
            emit(sn, pipe_emit_front<UC, SCN>(kp, m, sn, ent, lblob, hist));
            sn = nx;
          }
        }
        emit(sn, pipe_emit_front<UC, SCN>(kp, m, sn, pipe_cell<UC, SCN>(kp, sn, lblob), lblob, hist));
      } else {
        steps(std::false_type{});
      }
      MEV_TS(min(3 + 3 * it, 27));
      // the state after the last step (see k_steps_packed), as unconditional buffer stores; the
      // stream state only where the slot holds it (draws past the table, mev_state.pcg): no
      // global load here, whose wait would drain every store of the pair
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool sv_ok = env_ok[r] && m.u < U;
        if (C8) {
          __builtin_amdgcn_raw_buffer_store_b32(pack8(c[r].pos, c[r].wp), out_rsrc(st.ue_state, bst),
                                                sv_ok ? 4u * (uint32_t)(e[r] * U + m.u) : bst, 0, 0);
        } else {
          const int2 pw = make_int2((int)(((unsigned)c[r].pos.x & 0xffffu) | ((unsigned)c[r].pos.y << 16)),
                                    (int)(((unsigned)c[r].wp.x & 0xffffu) | ((unsigned)c[r].wp.y << 16)));
          const v2u32 pv = {(unsigned)pw.x, (unsigned)pw.y};
          __builtin_amdgcn_raw_buffer_store_b64(pv, out_rsrc(st.ue_state, bst),
                                                sv_ok ? 8u * (uint32_t)(e[r] * U + m.u) : bst, 0, 0);
        }
        // (the slot is current: flags in the two-group loop, drawn > M in the pipelined one)
        const bool cur_st = PIPE ? c[r].drawn > M : ((c[r].fl & kMov) != 0 && (c[r].fl & kSok) != 0);
        const bool ld = env_ok[r] && leader;
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)c[r].t, out_rsrc(st.t, bt),
                                              ld ? 4u * (uint32_t)e[r] : bt, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)c[r].drawn, out_rsrc(tb.drawn, bt),
                                              ld ? 4u * (uint32_t)e[r] : bt, 0, 0);
        const u128 sl = lpcg[2 * (r * G + m.seg)];
        const v4u32 sv = {(unsigned)(uint64_t)sl, (unsigned)((uint64_t)sl >> 32),
                          (unsigned)(uint64_t)(sl >> 64), (unsigned)((uint64_t)(sl >> 64) >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(sv, out_rsrc(st.pcg, 12u * bt),
                                               ld && cur_st ? 48u * (uint32_t)e[r] : 12u * bt, 0, 0);
      }
    }
    if (nxt_ok) {  // the next pair's inputs (waited for: free after a whole pair's stores)
      lds2_consume<UC, SCN, R, PE, NT, NK, C8>(kp, st, m, lane, pn, f, saturated, c, ltab, lpcg, hist,
                                           lkeys);
      MEV_TS(min(4 + 3 * it, 28));
    }
    if (alt) {
      flush_staged2<PIPE>(out, sw, kp.E, e0, 0, nsteps, lower, NWG, false,
                          lblob + KPS(lds_r100_off) + 8 * kRewardCSlot, U);
    } else if (!cur_ok) {  // no pair for this wave: its part of the flushes only (the same
                           // barriers as the waves with pairs: DETECT as theirs)
      for (int i0 = 0; i0 < nsteps; i0 += stage_rows) {
        flush_staged2<PIPE>(out, sw + (dbl ? 2 * hcur * wrows : 0), kp.E, e0, traj ? i0 : 0,
                            min(stage_rows, nsteps - i0), lower, NWG, !dbl,
                            lblob + KPS(lds_r100_off) + 8 * kRewardCSlot, U);
        if (dbl) hcur ^= 1;
      }
    }
    MEV_TS(min(5 + 3 * it, 29));
    hb = alt ? nsteps - hb : 0;
    ++it;
  }
  MEV_TS(31);
  MEV_CLK(26);
}

// ------------------------------------------------------------------------------------
// Block shape: 64 < U <= 1024, one workgroup per env, lane u = threadIdx.x.
// ------------------------------------------------------------------------------------
// Reset (mev_reset): MComCore.reset for the envs with mask[e] (all if NULL), as k_reset_packed.
__global__ __launch_bounds__(1024) void k_reset_block(KParams kp, KState st, KOut out,
                                                      KTables tb,
                                                      const uint8_t* __restrict__ mask) {
  const int e = blockIdx.x;
  const int u = threadIdx.x;
  const int U = kp.U;
  if (mask != nullptr && !mask[e]) return;  // uniform over the workgroup
  const bool valid = u < U;
  const size_t idx = (size_t)e * U + u;
  const uint64_t* pr = st.pcg + (size_t)6 * e;
  const ulonglong2 b2 = *reinterpret_cast<const ulonglong2*>(pr + 2);
  const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(pr);
  const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(pr + 4);
  const u128 s0 = kp.movement_reseed ? mk128(c.x, c.y) : mk128(a.x, a.y);
  int x = 0, y = 0;
  u128 s_fin = s0;
  if (valid) s_fin = pcg_draw_pair(s0, mk128(b2.x, b2.y), 2 * u, tb.jump, kp.Wd, kp.Hd, x, y);
  if (valid) {
    store_ue_at(st.ue_state, (uint32_t)idx, make_int2(x, y), make_int2(-1, -1), kp.st8 != 0);
    out.serving[idx] = -1;
    out.obs[idx] = make_float4((float)x * kp.inv_w, (float)y * kp.inv_h, 0.f, 0.f);
    if (out.rate64) out.rate64[idx] = 0.0;
    if (out.util64) out.util64[idx] = 0.0;
  }
  if (u == U - 1)  // the state after the 2U initial draws
    *reinterpret_cast<ulonglong2*>(st.pcg + (size_t)6 * e) =
        make_ulonglong2((uint64_t)s_fin, (uint64_t)(s_fin >> 64));
  if (u == 0) {
    if (kp.tab_m) tb.drawn[e] = U;
    st.t[e] = 0;
    out.reward[e] = 0.f;
    out.done[e] = 0;
    if (out.metrics) out.metrics[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Sum over the 64 lanes of a wavefront (all active), valid in lane 63: row prefix sums by
// row_shr 1/2/4/8, then the row totals carried by row_bcast:15 (into rows 1, 3) and
// row_bcast:31 (into rows 2, 3).

// Smallest association key over the station pairs [j0, j1) of the LDS key array (two
// stations per broadcast ds_read_b128): scaled keys dot2(32 p, m) + c, else (dot2(p, m) << 10) + c
// (see k_steps_block's prologue).
// (wide maps, W or H > 1024: the keys hold the station itself, {q as int16x2, j}; a UE's key is
// (min(|p - q|^2, 2^22 - 1) << 10) | j -- the clamp only merges distances far beyond any
// connectable one, kD2Top < 2^21, whose order does not matter: such a minimum serves nobody)
__device__ __forceinline__ unsigned wide_key(int2 pos, unsigned qw, unsigned j) {
  const s16x2 d = s16x2{(short)pos.x, (short)pos.y} - as_s16x2(qw);
  const unsigned d2 = (unsigned)__builtin_amdgcn_sdot2(d, d, 0, false);
  return (min(d2, (1u << 22) - 1u) << kKeyBits) | j;
}

__device__ __forceinline__ unsigned scan_key_pairs(const v4u32* __restrict__ kk2, int j0, int j1,
                                                   bool scaled, int2 pos, bool wide = false) {
  unsigned best = UINT_MAX;
  if (wide) {
#pragma unroll 4
    for (int j = j0; j < j1; ++j) {
      const v4u32 kv = kk2[j];
      best = min(best, min(wide_key(pos, kv.x, kv.y), wide_key(pos, kv.z, kv.w)));
    }
  } else if (scaled) {
    const s16x2 p32 = {(short)(pos.x << 5), (short)(pos.y << 5)};
#pragma unroll 4
    for (int j = j0; j < j1; ++j) {
      const v4u32 kv = kk2[j];
      const unsigned k0 = (unsigned)__builtin_amdgcn_sdot2(p32, as_s16x2(kv.x), (int)kv.y, false);
      const unsigned k1 = (unsigned)__builtin_amdgcn_sdot2(p32, as_s16x2(kv.z), (int)kv.w, false);
      best = min(best, min(k0, k1));
    }
  } else {
    const s16x2 pu = {(short)pos.x, (short)pos.y};
#pragma unroll 4
    for (int j = j0; j < j1; ++j) {
      const v4u32 kv = kk2[j];
      const int d0 = __builtin_amdgcn_sdot2(pu, as_s16x2(kv.x), 0, true);
      const int d1 = __builtin_amdgcn_sdot2(pu, as_s16x2(kv.z), 0, true);
      best = min(best, min(((unsigned)d0 << kKeyBits) + kv.y, ((unsigned)d1 << kKeyBits) + kv.w));
    }
  }
  return best;
}

// squared distance encoded in an association key of the UE at pos: key - 2^21 + |p|^2 (wide
// maps: the key's (clamped) squared distance itself)
__device__ __forceinline__ int key_d2(unsigned key, int2 pos, bool wide = false) {
  if (wide) return (int)(key >> kKeyBits);
  return (int)(key >> kKeyBits) - (1 << 21) + (pos.x * pos.x + pos.y * pos.y);
}

__device__ __forceinline__ double wave_sum_f64(double x) {
  x += dpp_f64<0x111>(x);
  x += dpp_f64<0x112>(x);
  x += dpp_f64<0x114>(x);
  x += dpp_f64<0x118>(x);
  x += dpp_f64<0x142, 0xa>(x);
  x += dpp_f64<0x143, 0xc>(x);
  return x;
}

// LDS of k_steps_block (dynamic; sized by the host, block_lds_bytes): int2 keys[B + 2] (the
// env's station keys), int cnt[3][B] (per-station connected-UE counts, three steps in flight),
// int wt[2][4][16] (per-wave counts by step parity: need | active << 16, -, connected, low QoE), double
// ps[2][4][16] (per-wave partial sums by step parity: utility, rate, QoE, QoE^2), u128 slot[2]
// (stream state after the env's last draw, increment), int tab[M] (the env's episode draw
// table), double r100[kMaxU + 1] (100 / n correctly rounded: the ResourceFair share without a
// division, filled once per workgroup). The per-step buffers rotate so that ONE barrier per
// step orders every producer before its consumers (k_steps_block).
struct BlockLds {
  int2* key;
  int* cnt;
  int* wt;
  double* ps;
  u128* slot;
  int* tab;
  double* r100;
};

// (the keys live in a static array: its 16-byte alignment is known to the compiler, which
// then reads two stations per broadcast ds_read_b128 -- from the dynamic area it issued four
// ds_read2_b32, twice the LDS cycles)
__host__ __device__ inline size_t block_tab_off(int B) {
  return ((12 * (size_t)B + 15) & ~(size_t)15) + 4 * 128 + 8 * 128 + 32;
}
__host__ __device__ inline size_t block_r100_off(int B, int M) {
  return (block_tab_off(B) + 4 * (size_t)M + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t block_lds_bytes(int B, int M) {
  return block_r100_off(B, M) + 8 * (size_t)(kMaxU + 1);
}
// Station culling (k_steps_block): the map in square cells of 2^cull_log, per cell a 16-byte
// LDS record {count, up to 15 candidate station indices} after the other areas. Chosen on the
// host for homogeneous layouts of 32..255 stations on maps up to 512 x 512: the cell side about
// a third of the mean station spacing sqrt(W H / B), doubled until the records fit 40 KB (the
// block kernel's two workgroups per CU); 128 stations on 200 x 200: 4 x 4 cells, 2,500 records,
// 1.8 candidates per cell on average.
struct CullP {
  int log, nx, nc;
};
inline CullP block_cull_params(int B, int W, int H, bool het) {
  CullP r{0, 0, 0};
  if (het || B < 32 || B > 255 || W > 512 || H > 512) return r;
  const double spacing = sqrt((double)W * (double)H / (double)B);
  int k = 1;
  while ((double)(2 << k) <= spacing / 3.0) ++k;
  for (;; ++k) {
    const int nx = (W + (1 << k) - 1) >> k, ny = (H + (1 << k) - 1) >> k;
    if (16 * nx * ny <= 40960) {
      r = CullP{k, nx, nx * ny};
      return r;
    }
  }
}

// The records kept in HBM for short launches (mev_update_layouts) use cells twice as wide (a
// quarter of the records: 9.8 KB per env for 128 stations on 200 x 200, 3.2 candidates per cell
// on average), since a one-step launch reads about one 64-byte line per UE of them.
__host__ __device__ inline CullP pers_cull(int log, int W, int H) {
  const int k = log + 1;
  const int nx = (W + (1 << k) - 1) >> k, ny = (H + (1 << k) - 1) >> k;
  return CullP{k, nx, nx * ny};
}

// LDS bytes of k_steps_block's culling records: only launches of >= 32 steps build them in LDS
// (shorter ones read the HBM records, or scan every station); with two UEs per lane in cells
// twice as wide (pers_cull), so that four workgroups fit beside each other on a CU.
inline size_t block_rec_bytes(const CullP& cp, int W, int H, int nsteps, int upl) {
  if (cp.log <= 0 || nsteps < 32) return 0;
  return 16 * (size_t)(upl == 2 ? pers_cull(cp.log, W, H).nc : cp.nc);
}

__device__ __forceinline__ BlockLds block_lds(char* base, int2* keys, int B) {
  BlockLds l;
  l.key = keys;
  char* p = base;
  l.cnt = reinterpret_cast<int*>(p);
  p += (12 * (size_t)B + 15) & ~(size_t)15;
  l.wt = reinterpret_cast<int*>(p);
  l.ps = reinterpret_cast<double*>(p + 4 * 128);
  l.slot = reinterpret_cast<u128*>(p + 4 * 128 + 8 * 128);
  l.tab = reinterpret_cast<int*>(p + 4 * 128 + 8 * 128 + 32);
  return l;
}

__device__ __forceinline__ BlockLds block_lds(char* base, int2* keys, int B, int M) {
  BlockLds l = block_lds(base, keys, B);
  l.r100 = reinterpret_cast<double*>(base + block_r100_off(B, M));
  return l;
}

// int32 sum over the 64 lanes of a wavefront (all active), valid in lane 63
__device__ __forceinline__ int wave_isum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, true);
  return x;
}

// Station culling records (k_steps_block, k_cull_build): for every cell c of the map in squares
// of 2^clog, rec[16 c] = {count, up to 15 candidate station indices}: s* = the station closest
// to a point of the cell, D2 = its squared distance to the cell's farthest corner (every point
// of the cell has a station within D2), and every station s whose squared distance to the cell
// is <= D2. A station outside the list is farther than D2 from every point of the cell, so
// strictly farther than s*: the minimum key over the list (ties by index included) is the
// minimum over all stations. More than 15 candidates: count 255, the lane scans every station.
// keys: the env's scaled station keys in LDS (k_steps_block's form); threads tid, tid + nt, ...
__device__ __forceinline__ void cull_cells(const int2* keys, int nb, int clog, int cnx, int cnc, int W, int H,
                           int tid, int nt, unsigned char* rec_out) {
  const v4u32* kk2 = reinterpret_cast<const v4u32*>(keys);
  for (int c = tid; c < cnc; c += nt) {
    const int cy = c / cnx, cx = c - cy * cnx;
    const int x0 = cx << clog, y0 = cy << clog;
    const int x1 = min(x0 + (1 << clog) - 1, W - 1);
    const int y1 = min(y0 + (1 << clog) - 1, H - 1);
    const int xm = (x0 + x1) >> 1, ym = (y0 + y1) >> 1;  // a point of the cell
    const unsigned bk = scan_key_pairs(kk2, 0, nb >> 1, true, make_int2(xm, ym));
    unsigned best = bk;
    if (nb & 1) {
      const int2 kv = keys[nb - 1];
      const s16x2 p32 = {(short)(xm << 5), (short)(ym << 5)};
      best = min(best, (unsigned)__builtin_amdgcn_sdot2(p32, as_s16x2((unsigned)kv.x), kv.y, false));
    }
    const int2 ks = keys[best & ((1u << kKeyBits) - 1)];
    const int sx = -(int)(short)(ks.x & 0xffff) >> 6, sy = -(int)(short)(ks.x >> 16) >> 6;
    const int fx = max(sx - x0, x1 - sx), fy = max(sy - y0, y1 - sy);
    const int D2 = fx * fx + fy * fy;
    unsigned char* const r = rec_out + 16 * c;  // (byte stores: LDS in k_steps_block)
    int n = 0;
    for (int j = 0; j < nb; ++j) {
      const int2 kv = keys[j];
      const int qx = -(int)(short)(kv.x & 0xffff) >> 6, qy = -(int)(short)(kv.x >> 16) >> 6;
      const int dx = max(max(x0 - qx, qx - x1), 0), dy = max(max(y0 - qy, qy - y1), 0);
      if (dx * dx + dy * dy <= D2) {
        if (n < 15) r[1 + n] = (unsigned char)j;
        ++n;
      }
    }
    for (int j = n; j < 15; ++j) r[1 + j] = (unsigned char)nb;
    r[0] = (unsigned char)(n > 15 ? 255 : n);
  }
}

// The env's steps i0 .. nsteps-1 for one workgroup (block shape); see k_steps_block.
// Per-env values of a step whose row the leader writes after the next step's first barrier.
struct BlockRow {
  int t_after, nact, ncon;
};

// The block row's exact mean (block_finish_row_lean's rare path; wave-wide, lane 63 holds it)
MEV_GUARD_FN float block_fix_row(const float* rates, int U, int lane, const char* rc, int nact) {
  const RewardC c = reward_c(rc);
  long long v = 0;
#pragma unroll 1
  for (int u = lane; u < U; u += 64) v += util_fix50c(rint((double)rates[4 * u] * 100.0), c);
  return exact_mean50(seg_lsum_rows<64>(v), nact);
}

template <bool LEAN>
__device__ __forceinline__ void block_finish_row(const KParams& kp, const KOut& out,
                                                 const double* ps, const int* wt, int nw, int e,
                                                 int row, const BlockRow& r) {
  // the step's per-wave partials (its parity's buffers), summed in wave order (float64)
  double su = 0.0, sr = 0.0, sq = 0.0, sq2 = 0.0;
  int nlow = 0;
  for (int i = 0; i < nw; ++i) {
    su += ps[i];
    if (!LEAN) {
      sr += ps[16 + i];
      sq += ps[32 + i];
      sq2 += ps[48 + i];
      nlow += wt[48 + i];
    }
  }
  const double mean_u = r.nact > 0 ? su / (double)r.nact : kp.lower;
  const size_t re = (size_t)row * kp.E + e;
  out.reward[re] = (float)mean_u;
  out.done[re] = (uint8_t)(r.t_after >= kp.t_end);
  if (!LEAN) {
    if (out.metrics) {
      const double mean_r = r.ncon > 0 ? sr / (double)r.ncon : 0.0;
      out.metrics[re] = make_float4((float)r.ncon, (float)r.ncon, (float)mean_u, (float)mean_r);
    }
    if (out.qoe_stats) {
      double4 a = r.t_after == 1 ? make_double4(0.0, 0.0, 0.0, 0.0) : out.qoe_stats[e];
      a.x += (double)r.nact;
      a.y += sq;
      a.z += sq2;
      a.w += (double)nlow;
      out.qoe_stats[e] = a;
    }
  }
}

// The lean path's row: the per-wave utility sums are 2^-24 fixed-point integers (stored as
// doubles, exact), summed by the 64 lanes of wave 0 in one DPP tree (exact: integers below
// 2^53, any order) instead of one lane's chain of dependent LDS reads; lane 63 writes.
__device__ __forceinline__ void block_finish_row_lean(const KParams& kp, const KOut& out,
                                                      const double* ps, int nw, int e, int row,
                                                      const BlockRow& r, int lane, bool fix,
                                                      const char* rc) {
  const double su = wave_sum_f64(lane < nw ? ps[lane] : 0.0);
  // reward_risky (rare, wave-uniform): the exact mean from the row's obs rates, which every wave
  // stored before the barrier this one follows (fenced: __syncthreads); `fix`: the row is still
  // there (trajectory rows, or the launch's last row). cents = rint(100 rate) exactly below 6e6,
  // every table index is below 2^22; the env's UEs are all active or none (nact = U or 0).
  float exact = 0.f;
  const float sum_f = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                    __builtin_bit_cast(int, (float)su), 63));
  const bool risky = fix && r.nact > 0 && fabsf(sum_f * 0x1p-24f) <= (float)r.nact * kp.r_thr;
  if (risky) {  // (the pointer laundered inside the branch: see flush_staged2)
    const float* obs_f = reinterpret_cast<const float*>(out.obs);
    asm volatile("" : "+s"(obs_f));
    wait_vmem();  // (no load in flight across the call)
    exact = block_fix_row(obs_f + 4 * ((size_t)row * kp.E + (size_t)e) * (size_t)kp.U + 2, kp.U,
                          lane, rc, r.nact);
  }
  if (lane == 63) {
    // the float32 reward as the packed kernels' lean path forms it (a float32 product with the
    // reciprocal; ~1e-7 relative of np.mean), not a float64 division on wave 0's path every step
    const float mean_u = risky ? exact
                       : r.nact > 0 ? (float)su * 0x1p-24f * __builtin_amdgcn_rcpf((float)r.nact)
                                    : (float)kp.lower;
    const size_t re = (size_t)row * kp.E + e;
    out.reward[re] = mean_u;
    out.done[re] = (uint8_t)(r.t_after >= kp.t_end);
  }
}

// nsteps steps of MComCore.step (base.py:230-296) for U > 64: one workgroup of ceil(U/64)
// waves per env (lane u = UE u), env e = blockIdx.x (grid = E); each env's
// state stays in registers / LDS for the launch (loaded once, stored once) and every step's
// outputs go to row i of the trajectory (traj) or over the previous step's. Per step, ONE
// workgroup barrier:
//   A  lazy auto-reset (initial positions from the LDS draw table), need / active; the
//      workgroup scan of the waypoint draws (ue_id order) from the per-wave counts the
//      previous step wrote before its barrier
//   B  waypoint draws (LDS draw table; beyond it, the stream state), move, association (the
//      env's station keys in LDS, broadcast reads), per-station counts by LDS atomics; the
//      NEXT step's per-wave need / active counts (its reset applied ahead: both follow from
//      t + 1 and the waypoint after this move)
//   -- barrier --
//   C  ResourceFair share, rounded rate, utility, per-UE stores, per-wave partial sums; the
//      previous step's per-env row (reward, done, metrics) from its partial sums
// Ordering without a second barrier: the per-wave counts and partial sums alternate between
// two buffers by step parity and the per-station counts rotate over three arrays (the array
// zeroed in step i's B phase was last read in step i-2's C phase, before step i-1's
// barrier); the rare stream-state path (draws past the table, resets without one) takes an
// extra barrier, block-uniform, before it writes the slot the other waves read at the step's
// start.
// UPL UEs per lane (1, or 2 for U > 512: half the waves per env, so that a batch whose
// one-UE-per-lane workgroups would take two rounds of the chip's resident waves fits in one):
// the lane's UEs are tid + h * blockDim.x, h < UPL, and UE u belongs to the "virtual wave"
// u >> 6 = w + h * nw -- the same partition of the env's UEs into 64-UE groups as with one UE
// per lane, so that every per-wave count, scan and partial sum (and its summation order) is
// the same.
template <bool PER_ENV_BS, bool LEAN, bool HET, int SCN = 0, bool TF = false, int UPL = 1>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void k_steps_block(
    KParams kp, KState st, KOut out, KTables tb, int nsteps, int traj) {
  static_assert(UPL == 1 || (UPL == 2 && !HET), "two UEs per lane: homogeneous entities only");
  extern __shared__ __align__(16) char lds_raw[];
  // (a scenario instance: its station count; LDS for four workgroups per CU with two UEs per lane)
  __shared__ __align__(16) int2 lds_keys[SCN ? scn_const(SCN).B + 2 : kMaxB + 2 + kMaxClasses];
  __shared__ __align__(8) double lds_rc[4];  // (lean) RewardC, written in the prologue
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  const int U = KPS(U);
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int nw = (nt + 63) >> 6;  // waves of the workgroup
  const int nv = UPL * nw;        // virtual waves (<= 16: U <= 1024)
  int uh[UPL];
  bool valid[UPL];
#pragma unroll
  for (int h = 0; h < UPL; ++h) {
    uh[h] = tid + h * nt;
    valid[h] = uh[h] < U;
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  const int M = KPS(tab_m);
  const BlockLds L = block_lds(lds_raw, lds_keys, KPS(B), KPS(tab_m));
  // 100 / n for n <= rlim: every count for a multi-step launch; a one-step launch fills n <= 64
  // (one division per lane of the first wave instead of ~two per lane of every wave) and divides
  // where a station has more (the same correctly rounded value)
  const int rlim = nsteps == 1 ? min(U, 64) : U;
  for (int n = tid; n <= rlim; n += nt) L.r100[n] = n ? 100.0 / (double)n : 0.0;
  // station culling: per cell of the map, the stations that can be the closest to some point
  // of the cell (see the prologue)
  const bool CULL = !HET && KPS(cull_log) > 0;
  const int CLOG = KPS(cull_log), CNX = KPS(cull_nx), CNC = KPS(cull_nc);
  unsigned char* const crec =
      reinterpret_cast<unsigned char*>(lds_raw + block_lds_bytes(KPS(B), KPS(tab_m)));
  // heterogeneous entities (UPL 1): this UE's class and movement parameters
  const int cu = HET ? (valid[0] ? (int)tb.ue_cls[tid] : 0) : 0;
  const MoveP mp = HET ? tb.mv[valid[0] ? tid : 0]
                       : MoveP{kp.vel, KPSF(vel_f), KPSF(move_lim), KPS(d2snap), KPS(axis_exact)};
  // one workgroup per env (grid = E): no loop over envs, whose loop-invariant values the
  // compiler would hoist and spill under the 64-VGPR budget (76 B of scratch per lane, written
  // by every wave at its start: 80 MB per launch at 1,024 envs of 1,024 UEs)
  {
    const int e = blockIdx.x;
    if (e >= kp.E) return;
    // ---- prologue: state, stream, station keys, draw table -------------------------------
    const size_t ebase = (size_t)e * U;
    int2 pos[UPL], wp[UPL];
#pragma unroll
    for (int h = 0; h < UPL; ++h) {
      pos[h] = make_int2(0, 0);
      wp[h] = make_int2(-1, -1);
      if (valid[h]) {
        const int4 sv = load_ue_at(st.ue_state, (uint32_t)(ebase + uh[h]), KST8);
        pos[h] = make_int2(sv.x, sv.y);
        wp[h] = make_int2(sv.z, sv.w);
      }
    }
    int t = st.t[e];
    int drawn = M ? tb.drawn[e] : 0;
    if (tid == 0) {
      const ulonglong2* pr = reinterpret_cast<const ulonglong2*>(st.pcg + (size_t)6 * e);
      L.slot[0] = mk128(pr[0].x, pr[0].y);
      L.slot[1] = mk128(pr[1].x, pr[1].y);
    }
    const int nb = PER_ENV_BS ? (st.bs_count ? st.bs_count[e] : KPS(B)) : KPS(B);
    // station keys {m as int16x2, c = ((|q|^2 + 2^21) << 10) | j}: with the map <= 512 x 512 and
    // every station in [0, 512)^2, m = -64 q and key = dot2(32 p, m) + c =
    // ((|p - q|^2 - |p|^2 + 2^21) << 10) | j; otherwise m = -2 q, key = (dot2(p, m) << 10) + c
    const int2* bsx = PER_ENV_BS ? st.bs_xy + (size_t)e * KPS(B) : st.bs_xy;
    bool in512 = true;
    int2 q_own = make_int2(0, 0);  // station tid (kept for its key below: no second load)
    for (int i = tid; i < nb; i += nt) {
      const int2 qq = bsx[i];
      if (i == tid) q_own = qq;
      in512 = in512 && qq.x >= 0 && qq.y >= 0 && qq.x < 512 && qq.y < 512;
    }
    // the episode draw table in LDS: all M pairs for launches of several steps; a one-step
    // launch copies only the window it can use, 2U pairs from `tb` = 0 (a reset this step: the
    // U initial positions, then the draws) or from `drawn` (the draws: at most U)
    // (a one-step launch reads its few pairs straight from HBM instead: the copy loop waits for
    // each of a lane's loads before its store, a chain of global round trips in the prologue)
    const bool tab_g = nsteps == 1;
    const int* const tab_src = tb.tab_xy + (size_t)e * M;
    const int tb0 = 0;
    const int tlim = M;
    if (M && !tab_g)
      for (int k = tb0 + tid; k < tlim; k += nt) L.tab[k - tb0] = tab_src[k];
    auto tab_at = [&](int k) { return tab_g ? tab_src[k] : L.tab[k - tb0]; };  // (k < M)
    const bool scaled = __syncthreads_and(in512) && KPS(W) <= 512 && KPS(H) <= 512;
    const bool wide = KPS(W) > 1024 || KPS(H) > 1024;  // (uniform; a scenario: constant false)
    // key slots: station k (homogeneous), or station perm[k] grouped by class (HET; padding
    // and stations beyond the env's count get the key that never wins, m = 0, c = UINT_MAX)
    const int nslot = HET ? kp.bperm : nb;
    for (int k = tid; k < nslot; k += nt) {
      const int i = HET ? (int)tb.perm[k] : k;
      if (HET && (i < 0 || i >= nb)) {
        lds_keys[k] = make_int2(0, -1);
        continue;
      }
      const int2 qq = !HET && k == tid ? q_own : bsx[i];
      if (wide) {  // the station itself (scan_key_pairs' wide form)
        lds_keys[k] = make_int2((int)(((unsigned)qq.x & 0xffffu) | ((unsigned)qq.y << 16)), i);
        continue;
      }
      const int f = scaled ? -64 : -2;
      const s16x2 m2 = {(short)(f * qq.x), (short)(f * qq.y)};
      lds_keys[k] = make_int2(__builtin_bit_cast(int, m2),
                              (int)(((unsigned)(qq.x * qq.x + qq.y * qq.y + (1 << 21)) << kKeyBits) |
                                    (unsigned)i));
    }
    for (int i = tid; i < KPS(B); i += nt) L.cnt[i] = 0;  // step 0's counts
    if (LEAN && tid == 0) {
      *reinterpret_cast<const double**>(&lds_rc[0]) = tb.util;
      lds_rc[1] = kp.util_sat;
      lds_rc[2] = (double)kp.util_kmax;
      *reinterpret_cast<float*>(&lds_rc[3]) = kp.u_err;
    }
    if (CULL && tid == 0) lds_keys[nb] = make_int2(0, -1);  // the candidate lists' padding slot
    // the slot holds the state after the env's last draw: the state row without a table, or
    // after draws past it (mev_state.pcg)
    bool s_ok = !M || drawn > M;
    BlockRow prev{0, 0, 0};
    // step 0's per-virtual-wave need / active counts (its lazy reset applied ahead)
    auto ahead_counts = [&](int tn, const int2 (&wpn)[UPL], int* wt) {
      const bool rs = tn >= KPS(t_end);
      const int t0 = rs ? 0 : tn;
      const bool on = t0 >= KPS(arr_start) && t0 < KPS(arr_exit) &&
                      (KPS(first_step_active) || t0 != 0);
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        const bool act = valid[h] && on;
        const uint64_t mn = bal(act && (rs || wpn[h].x < 0)), ma = bal(act);
        // {need, active} packed in one int (each <= 64 per wave, <= 1024 per env): one read
        // and one scan per step
        if (lane == 0) wt[w + h * nw] = __popcll(mn) | (__popcll(ma) << 16);
      }
    };
    ahead_counts(t, wp, L.wt);
    __syncthreads();
    // (uniform) launches of >= 32 steps build the records in LDS (they cost about as much as
    // 18 steps' full scans); shorter ones read the env's records kept in HBM by
    // mev_update_layouts, where they are valid for its layout
    const bool pers = CULL && tb.crec_g != nullptr && nsteps < 32;
    const int erec = PER_ENV_BS ? e : 0;  // (a shared layout: one record set)
    const bool cull = CULL && scaled && nb > 0 && (pers ? tb.crec_ok[erec] != 0 : nsteps >= 32);
    // the records' cells: the HBM records' (twice as wide) for pers, and in LDS with two UEs per
    // lane (a quarter of the LDS: four workgroups per CU, see block_rec_bytes)
    const CullP pc = pers_cull(CLOG, KPS(W), KPS(H));
    const bool wcell = pers || UPL == 2;
    const int RLOG = wcell ? pc.log : CLOG, RNX = wcell ? pc.nx : CNX, RNC = wcell ? pc.nc : CNC;
    const unsigned char* const grec = pers ? tb.crec_g + (size_t)erec * pc.nc * 16 : nullptr;
    if (cull && !pers) {
      cull_cells(lds_keys, nb, RLOG, RNX, RNC, KPS(W), KPS(H), tid, nt, crec);
      __syncthreads();
    }

    for (int i = 0, par = 0, c3 = 0; i < nsteps; ++i) {
      const int row = traj ? i : 0;
      int* cnt = L.cnt + c3 * KPS(B);  // (B = count array stride; three arrays, rotating)
      int* const wt = L.wt + 64 * par;       // this step's per-wave counts
      double* const ps = L.ps + 64 * par;    // this step's per-wave partial sums
      // ---- A: lazy auto-reset, ballots ------------------------------------------------
      const bool reset = t >= KPS(t_end);  // uniform
      int koff = 0;
      // the stream slot {state, increment}: read only on the rare paths that draw from it, and
      // there before the branch's barrier (the slot's write follows that barrier)
      u128 base = 0, inc = 0;
      if (reset) {
        t = 0;
#pragma unroll
        for (int h = 0; h < UPL; ++h) wp[h] = make_int2(-1, -1);
        if (M) {
#pragma unroll
          for (int h = 0; h < UPL; ++h)
            if (valid[h]) {
              const int p = tab_at(uh[h]);
              pos[h] = make_int2((int)(short)p, p >> 16);
            }
          drawn = U;
          s_ok = false;
        } else {
          base = L.slot[0];
          inc = L.slot[1];
          const ulonglong2 c = reinterpret_cast<const ulonglong2*>(st.pcg + (size_t)6 * e)[2];
          if (kp.movement_reseed) base = mk128(c.x, c.y);
#pragma unroll
          for (int h = 0; h < UPL; ++h)
            if (valid[h])
              (void)pcg_draw_pair(base, inc, 2 * uh[h], tb.jump, kp.Wd, kp.Hd, pos[h].x, pos[h].y);
          koff = 2 * U;
          wait_vmem();
        }
      }
      const bool on = t >= KPS(arr_start) && t < KPS(arr_exit) && (KPS(first_step_active) || t != 0);
      bool active[UPL], need[UPL];
      uint64_t mneed[UPL];
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        active[h] = valid[h] && on;
        need[h] = active[h] && wp[h].x < 0;
        mneed[h] = bal(need[h]);
      }

      const int scan_na = row_scan_i32(lane < nv ? wt[lane & 15] : 0);
      const int tot_na = __builtin_amdgcn_readlane(scan_na, nv - 1);
      const int tot = tot_na & 0xffff;
      const int nact = tot_na >> 16;
      const int c3n = c3 == 2 ? 0 : c3 + 1;
      int* cnt_next = L.cnt + c3n * KPS(B);  // (last read in step i - 2)
      if (SCN) {  // (a scenario instance: one store per lane)
        static_assert(!SCN || scn_const(SCN).U / UPL >= scn_const(SCN).B, "block scenario: U >= UPL B");
        if (tid < KPS(B)) cnt_next[tid] = 0;
      } else {
        for (int k = tid; k < KPS(B); k += nt) cnt_next[k] = 0;
      }

      // ---- B: waypoint draws in ue_id order (movement.py:44-47), move ------------------
      int rank[UPL];
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        const int vw = w + h * nw;
        const int pre_need = vw ? (__builtin_amdgcn_readlane(scan_na, vw - 1) & 0xffff) : 0;
        rank[h] = pre_need + (int)__popcll(mneed[h] & lt);
      }
      if (tot > 0) {
        if (M && drawn + tot <= M) {  // every pair precomputed (the common case)
#pragma unroll
          for (int h = 0; h < UPL; ++h)
            if (need[h]) {
              const int p = tab_at(drawn + rank[h]);  // pair index in the episode
              wp[h] = make_int2((int)(short)p, p >> 16);
            }
          s_ok = false;
        } else {
          // beyond the table (or none): from the stream state after pair bidx - 1 (the slot,
          // or the table's last entry), pair k at offset 2 (k - bidx); every wave has read
          // the slot before it is written (block-uniform branch)
          if (!(reset && !M)) {  // (a reset without a table read it above)
            base = L.slot[0];
            inc = L.slot[1];
          }
          __syncthreads();
          int bidx = drawn;
          if (M && !s_ok) {
            base = tb.tab_st[(size_t)e * M + (M - 1)];
            bidx = M;
            // (waited for here: a load left pending into the common path's merge makes the
            // compiler's vmcnt(0) there wait for the previous step's stores as well)
            wait_vmem();
          }
#pragma unroll
          for (int h = 0; h < UPL; ++h)
            if (need[h]) {
              const int k = drawn + rank[h];
              u128 s_fin;
              if (M && k < M) {
                const int p = tab_at(k);
                wp[h] = make_int2((int)(short)p, p >> 16);
                s_fin = base;
              } else {
                s_fin = pcg_draw_pair(base, inc, koff + 2 * (k - bidx), tb.jump, kp.Wd, kp.Hd,
                                      wp[h].x, wp[h].y);
              }
              if (rank[h] == tot - 1) L.slot[0] = s_fin;  // the env's new stream state
            }
          s_ok = true;
        }
        drawn += tot;
      } else if (reset && !M) {  // reset without draws: after the initial pairs (uniform)
        __syncthreads();
#pragma unroll
        for (int h = 0; h < UPL; ++h)
          if (uh[h] == U - 1)
            L.slot[0] = pcg_draw_pair(base, inc, 2 * (U - 1), tb.jump, kp.Wd, kp.Hd, pos[h].x,
                                      pos[h].y);
      }
#pragma unroll
      for (int h = 0; h < UPL; ++h)
        if (active[h]) move_ue_p(pos[h], wp[h], mp);
      // the next step's, after this move (none after a launch's last step: the next launch's
      // prologue counts from the stored state)
      if (i + 1 < nsteps) ahead_counts(t + 1, wp, L.wt + 64 * (par ^ 1));

      // ---- association: min over the env's station keys (LDS broadcast reads) ----------
      // (ext_vector_type loads: one broadcast ds_read_b128 per two stations; HIP's int4 struct is
      // loaded member-wise, which became four ds_read2_b32 -- twice the LDS cycles)
      const v4u32* kk2 = reinterpret_cast<const v4u32*>(lds_keys);
      int srv[UPL];
      double full[UPL];
      unsigned best[UPL];
      // the cell's candidate list (CULL): its count and up to 15 station indices, one key per
      // candidate (a per-lane ds_read_b64), until no lane of the wave has more; with two UEs
      // per lane both records are read, and both lists walked, together (one chain of reads,
      // not two)
      bool full_scan[UPL];
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        best[h] = UINT_MAX;
        full_scan[h] = true;
      }
      if (cull) {
        v4u32 rec[UPL];
        int cn[UPL];
        s16x2 p32[UPL];
#pragma unroll
        for (int h = 0; h < UPL; ++h) {
          const int cell = min(__mul24(max(pos[h].y, 0) >> RLOG, RNX) + (max(pos[h].x, 0) >> RLOG),
                               RNC - 1);
          rec[h] = pers ? *reinterpret_cast<const v4u32*>(grec + 16 * cell)
                        : *reinterpret_cast<const v4u32*>(crec + 16 * cell);
        }
#pragma unroll
        for (int h = 0; h < UPL; ++h) {
          cn[h] = active[h] ? (int)(rec[h].x & 255u) : 0;
          full_scan[h] = bal(cn[h] > 15) != 0;
          p32[h] = s16x2{(short)(pos[h].x << 5), (short)(pos[h].y << 5)};
        }
        // the first four candidates unconditionally (four reads in flight; past a lane's
        // count the record holds the padding index, whose key never wins), then one at a
        // time while a lane of the wave has more (two at a time: timing-neutral)
        auto key_of = [&](int h, int j) {
          const unsigned wd = j < 3 ? rec[h].x : j < 7 ? rec[h].y : j < 11 ? rec[h].z : rec[h].w;
          const int2 kv = lds_keys[__builtin_amdgcn_ubfe(wd, (unsigned)(((j + 1) & 3) * 8), 8u)];
          return (unsigned)__builtin_amdgcn_sdot2(p32[h], as_s16x2((unsigned)kv.x), kv.y, false);
        };
#pragma unroll
        for (int h = 0; h < UPL; ++h)
          if (!full_scan[h])
            best[h] = min(min(key_of(h, 0), key_of(h, 1)), min(key_of(h, 2), key_of(h, 3)));
#pragma unroll
        for (int j = 4; j < 15; ++j) {
          bool more = false;
#pragma unroll
          for (int h = 0; h < UPL; ++h) more = more || (!full_scan[h] && bal(cn[h] > j) != 0);
          if (!more) break;
#pragma unroll
          for (int h = 0; h < UPL; ++h)
            if (!full_scan[h]) best[h] = min(best[h], key_of(h, j));
        }
#pragma unroll
        for (int h = 0; h < UPL; ++h)
          if (!full_scan[h] && !active[h]) best[h] = UINT_MAX;
      }
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        srv[h] = -1;
        full[h] = 0.0;
        int d2s = 0;
        if (!HET) {
          if (active[h] && full_scan[h]) {
            best[h] = scan_key_pairs(kk2, 0, nb >> 1, scaled, pos[h], wide);
            if (nb & 1) {  // the odd last station
              const int2 kv = lds_keys[nb - 1];
              const s16x2 p32 = {(short)(pos[h].x << 5), (short)(pos[h].y << 5)};
              const s16x2 pu = {(short)pos[h].x, (short)pos[h].y};
              best[h] = min(best[h], wide ? wide_key(pos[h], (unsigned)kv.x, (unsigned)kv.y)
                                     : scaled ? (unsigned)__builtin_amdgcn_sdot2(p32, as_s16x2((unsigned)kv.x), kv.y, false)
                                            : ((unsigned)__builtin_amdgcn_sdot2(pu, as_s16x2((unsigned)kv.x), 0, true) << kKeyBits) +
                                                  (unsigned)kv.y);
            }
          }
          d2s = key_d2(best[h], pos[h], wide);
          if (best[h] != UINT_MAX && d2s <= KPS(d2max)) srv[h] = (int)(best[h] & ((1u << kKeyBits) - 1));
          full[h] = tb.rate_full[max(0, min(d2s, KPS(d2max)))];
        } else {
          // per station class: the class's closest station, connectable iff d2 <= d2max of the
          // (station class, this UE's class) pair -- the closest connectable station overall is
          // the smallest key among the connectable class minima (base.py:236-241)
          if (active[h]) {
            for (int c = 0; c < kp.nb_cls; ++c) {
              const unsigned bc = scan_key_pairs(kk2, tb.seg[c] >> 1, tb.seg[c + 1] >> 1, scaled, pos[h], wide);
              if (bc != UINT_MAX && key_d2(bc, pos[h], wide) <= tb.pair[c * kp.nu_cls + cu].y)
                best[h] = min(best[h], bc);
            }
          }
          d2s = key_d2(best[h], pos[h], wide);
          if (best[h] != UINT_MAX) {
            srv[h] = (int)(best[h] & ((1u << kKeyBits) - 1));
            full[h] = tb.rate_full[tb.pair[(int)tb.bs_cls[srv[h]] * kp.nu_cls + cu].x + d2s];
          }
        }
      }
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        if (srv[h] >= 0) atomicAdd(&cnt[srv[h]], 1);
        if (!LEAN) {
          const int nc = __popcll(bal(srv[h] >= 0));  // (the ballot over the whole wavefront)
          if (lane == 0) wt[32 + w + h * nw] = nc;
        }
      }
      __syncthreads();  // ---- the step's barrier
      // the rate gather is waited for here (after the barrier: its latency overlaps the wait for
      // the other waves), on every path, before this step's stores: a lane or wave that never
      // reads `full` would carry the load as pending to a later merge, whose vmcnt(0) (before
      // the register is reused) would then also wait for the stores
#pragma unroll
      for (int h = 0; h < UPL; ++h) asm volatile("" ::"v"(full[h]));

      // ---- C: ResourceFair share + rounding, utility, stores, partial sums -------------
      // this env's rows in the output rows: a wave-uniform base and a 32-bit lane offset
      const size_t rb = (size_t)row * kp.E * U + ebase;
#pragma unroll
      for (int h = 0; h < UPL; ++h) {
        const int vw = w + h * nw;
        double cents = 0.0;
        float cents_f = 0.f;
        if (srv[h] >= 0) {
          const int n = cnt[srv[h]];
          const double r100 = n <= rlim ? L.r100[n] : 100.0 / (double)n;
          if (TF) {  // tie-free table (share_tie_free): the product rounds like the reference
            cents = rint(full[h] * r100);
            cents_f = (float)cents;
          } else {
            cents = share_cents_r(full[h], r100, n, cents_f);
          }
        }
        const bool exact_util = !LEAN;
        const double rate = cents / 100.0;
        double util = 0.0;
        if (active[h])
          util = exact_util ? utility_of(rate, cents, kp, tb.util)
                            : utility_f32r<SCN>(cents_f, cents_f * 0.01f, kp);
        if (valid[h]) {
          at(out.serving + rb, 4u * (uint32_t)uh[h]) = srv[h];
          at(out.obs + rb, 16u * (uint32_t)uh[h]) =
              make_float4((float)pos[h].x * KPSF(inv_w), (float)pos[h].y * KPSF(inv_h),
                          cents_f * 0.01f, (float)util);
          if (!LEAN) {
            if (out.rate64) out.rate64[rb + uh[h]] = rate;
            if (out.util64) out.util64[rb + uh[h]] = active[h] ? util : __builtin_nan("");
          }
        }
        if (LEAN) {  // 2^-24 fixed point: |sum| <= 64 * 2^24 (block_finish_row_lean)
          const int isu = wave_isum((int)((float)util * 0x1p24f));  // (util = 0 where inactive)
          if (lane == 63) ps[vw] = (double)isu;
        } else {
          const double su = wave_sum_f64(active[h] ? util : 0.0);
          const double q = rint(util * 100.0) / 100.0;  // numpy round(u, 2)
          const double sr = wave_sum_f64(srv[h] >= 0 ? rate : 0.0);
          const double sq = wave_sum_f64(active[h] ? q : 0.0);
          const double sq2 = wave_sum_f64(active[h] ? q * q : 0.0);
          const int nlow = __popcll(bal(active[h] && q < kp.qoe_low));
          if (lane == 63) {
            ps[vw] = su;
            ps[16 + vw] = sr;
            ps[32 + vw] = sq;
            ps[48 + vw] = sq2;
            wt[48 + vw] = nlow;
          }
        }
      }
      int ncon = 0;
      if (!LEAN) {
        const int sc = row_scan_i32(lane < nv ? wt[32 + (lane & 15)] : 0);
        ncon = __builtin_amdgcn_readlane(sc, nv - 1);
      }
      // the previous step's per-env row (its partial sums are complete: written before this
      // step's barrier)
      if (LEAN ? (w == 0 && i > 0) : (tid == 0 && i > 0)) {
        const double* pps = L.ps + 64 * (par ^ 1);
        if (LEAN) block_finish_row_lean(kp, out, pps, nv, e, traj ? i - 1 : 0, prev, lane, traj != 0,
                                        reinterpret_cast<const char*>(lds_rc));
        else block_finish_row<LEAN>(kp, out, pps, L.wt + 64 * (par ^ 1), nv, e, traj ? i - 1 : 0, prev);
      }
      prev = BlockRow{t + 1, nact, ncon};
      t += 1;
      par ^= 1;
      c3 = c3n;
    }
    __syncthreads();  // the last step's partial sums
    if (LEAN ? (w == 0 && nsteps > 0) : (tid == 0 && nsteps > 0)) {
      const int lp = (nsteps - 1) & 1;  // the last step's parity
      if (LEAN) block_finish_row_lean(kp, out, L.ps + 64 * lp, nv, e, traj ? nsteps - 1 : 0, prev, lane, true,
                                      reinterpret_cast<const char*>(lds_rc));
      else block_finish_row<LEAN>(kp, out, L.ps + 64 * lp, L.wt + 64 * lp, nv, e, traj ? nsteps - 1 : 0, prev);
    }
    // ---- epilogue: the state after the last step ----------------------------------------
#pragma unroll
    for (int h = 0; h < UPL; ++h)
      if (valid[h]) store_ue_at(st.ue_state, (uint32_t)(ebase + uh[h]), pos[h], wp[h], KST8);
    if (tid == 0) {
      st.t[e] = t;
      if (M) tb.drawn[e] = drawn;
      if (s_ok || !M) {  // (with a table and drawn <= M its entry is the state: row unchanged)
        const u128 sf = L.slot[0];
        *reinterpret_cast<ulonglong2*>(st.pcg + (size_t)6 * e) =
            make_ulonglong2((uint64_t)sf, (uint64_t)(sf >> 64));
      }
    }
  }
}

// Station culling records of per-env layouts (mev_update_layouts): one workgroup per env with
// mask[e] (all if NULL), the env's scaled station keys in LDS as k_steps_block forms them, then
// its records (cull_cells) to crec_g[e]; crec_ok[e] = 1 where k_steps_block would cull (every
// station and the map inside 512 x 512, at least one station).
// (A shared layout: one workgroup, one record set for every env.)
__global__ __launch_bounds__(256) void k_cull_build(KParams kp, KState st,
                                                    const uint8_t* __restrict__ mask,
                                                    int per_env, unsigned char* __restrict__ crec_g,
                                                    uint8_t* __restrict__ crec_ok) {
  __shared__ __align__(16) int2 keys[kMaxB + 2];
  const int e = blockIdx.x;
  if (e >= kp.E || (mask != nullptr && !mask[e])) return;
  const int t = threadIdx.x;
  const int nb = per_env && st.bs_count ? st.bs_count[e] : kp.B;
  const int2* bsx = st.bs_xy + (per_env ? (size_t)e * kp.B : 0);
  bool in512 = true;
  for (int i = t; i < nb; i += blockDim.x) {
    const int2 q = bsx[i];
    in512 = in512 && q.x >= 0 && q.y >= 0 && q.x < 512 && q.y < 512;
    const s16x2 m2 = {(short)(-64 * q.x), (short)(-64 * q.y)};
    keys[i] = make_int2(__builtin_bit_cast(int, m2),
                        (int)(((unsigned)(q.x * q.x + q.y * q.y + (1 << 21)) << kKeyBits) | (unsigned)i));
  }
  if (t == 0) keys[nb] = make_int2(0, -1);
  const bool ok = __syncthreads_and(in512) && kp.W <= 512 && kp.H <= 512 && nb > 0;
  if (t == 0) crec_ok[e] = ok ? 1 : 0;
  if (!ok) return;
  const CullP pc = pers_cull(kp.cull_log, kp.W, kp.H);
  cull_cells(keys, nb, pc.log, pc.nx, pc.nc, kp.W, kp.H, t, blockDim.x,
             crec_g + (size_t)e * pc.nc * 16);
}

// ------------------------------------------------------------------------------------
// Table builders (run once per context, on the device)
// ------------------------------------------------------------------------------------
// Rounded ResourceFair shares as the step kernels form them (mev_share_cents, tests):
// cents[n - 1][d2] for n in [1, nmax]; path 1 uses the 100/n table form of the LDS rollouts.
__global__ void k_share_cents(const double* __restrict__ rate_full, int d2n, int nmax, int path,
                              double* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)d2n * nmax) return;
  const int n = (int)(i / d2n) + 1, d2 = (int)(i - (int64_t)(n - 1) * d2n);
  float cf;
  dst[i] = path ? share_cents_r(rate_full[d2], 100.0 / (double)n, n, cf)
                : share_cents(rate_full[d2], n, cf);
}

// Scaled-utility table over rounded rates: tab[k] = scaled_utility(k / 100), evaluated by
// the same device function the step kernel would use (utilities.py:44-55).
__global__ void k_util_table(KParams kp, int kmax, double* __restrict__ tab,
                             int* __restrict__ bad) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > kmax) return;
  const double rate = (double)k / 100.0;
  const double v = scaled_utility(rate, kp);
  tab[k] = v;
  if (k == kmax && v != kp.util_sat) *bad = 1;  // saturation point must lie inside the table
}

// Association map of a shared station layout: for every grid position (x, y) of the map,
// {serving station (or -1), d2 to it, full rate rate_full[d2] as float64}. The serving station
// is the closest one (ties: lower index, python's min() over the station dict) and only if
// d2 <= d2max (snr > snr_tr, base.py:212-214,236-241). d2 in 64-bit: any int32 coordinates.
__global__ void k_assoc_map(const int2* __restrict__ bs, int B, int W, int H, int d2max,
                            const double* __restrict__ rate_full, int4* __restrict__ map) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  const int x = i % W, y = i / W;
  long long best = LLONG_MAX;
  int jb = -1;
  for (int j = 0; j < B; ++j) {
    const int2 q = bs[j];
    const long long dx = (long long)x - q.x, dy = (long long)y - q.y;
    const long long d2 = dx * dx + dy * dy;
    if (d2 < best) {
      best = d2;
      jb = j;
    }
  }
  int4 r = make_int4(-1, 0, 0, 0);
  if (jb >= 0 && best <= d2max) {
    const double f = rate_full[best];
    r = make_int4(jb, (int)best, __double2loint(f), __double2hiint(f));
  }
  map[i] = r;
}

// Heterogeneous entities, shared layout: one association map per UE class cu, [NU][H][W]. The
// serving station of a UE of class cu at (x, y) is the closest station j (ties: lower index)
// among those it can connect to, d2 <= d2max of the pair (class of j, cu) (base.py:236-241
// with the pair's SNR, channels.py:133-146); the full rate is that pair's table at d2.
__global__ void k_assoc_map_het(const int2* __restrict__ bs, int B, int W, int H,
                                const uint8_t* __restrict__ bs_cls, const int2* __restrict__ pair,
                                int NU, const double* __restrict__ rate_full,
                                int4* __restrict__ map) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int cells = W * H;
  if (i >= cells * NU) return;
  const int cu = i / cells, cell = i - cu * cells;
  const int x = cell % W, y = cell / W;
  long long best = LLONG_MAX;
  int jb = -1;
  for (int j = 0; j < B; ++j) {
    const int2 q = bs[j];
    const long long dx = (long long)x - q.x, dy = (long long)y - q.y;
    const long long d2 = dx * dx + dy * dy;
    if (d2 < best && d2 <= (long long)pair[(int)bs_cls[j] * NU + cu].y) {
      best = d2;
      jb = j;
    }
  }
  int4 r = make_int4(-1, 0, 0, 0);
  if (jb >= 0) {
    const double f = rate_full[pair[(int)bs_cls[jb] * NU + cu].x + best];
    r = make_int4(jb, (int)best, __double2loint(f), __double2hiint(f));
  }
  map[i] = r;
}

// Compact association tables (KTables::lds_blob), layout part: the serving station of every
// cell from the association map as 4 bits (15 = none), and the station coordinates. One thread
// per byte of the cell map (two cells).
__global__ void k_lds_map(const int2* __restrict__ bs, int B, int cells,
                          const int4* __restrict__ map, uint8_t* __restrict__ blob, int mode,
                          int st_off, int r16_off, const uint2* __restrict__ rankw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == 1 && i < 16) {
    const int2 q = i < B ? bs[i] : make_int2(0, 0);
    reinterpret_cast<int*>(blob + st_off)[i] = (int)(((unsigned)q.x & 0xffffu) | ((unsigned)q.y << 16));
  }
  if (2 * i >= cells) return;
  int sv[2];
  for (int h = 0; h < 2; ++h) {
    const int cl = 2 * i + h;
    const int4 r = cl < cells ? map[cl] : make_int4(-1, 0, 0, 0);
    sv[h] = r.x;
    if (mode == 2 && cl < cells) {  // rank of the cell's d2 (to its station) in S
      uint32_t k = 0;
      if (r.x >= 0) {
        const uint32_t d2 = (uint32_t)r.y;
        const uint2 w = rankw[d2 >> 5];
        k = w.y + (uint32_t)__popc(w.x & ((1u << (d2 & 31u)) - 1u));
      }
      reinterpret_cast<uint16_t*>(blob + r16_off)[cl] = (uint16_t)k;
    }
  }
  blob[i] = (uint8_t)((sv[0] < 0 ? 15 : sv[0]) | ((sv[1] < 0 ? 15 : sv[1]) << 4));
}

// Mode-3 tables (KTables::lds_blob), built from the association map on the device in three
// launches: the set D of squared distances between a cell and its serving station (a flag
// byte per d2: plain stores of the same value, no atomics), its rank index {bits, prefix} over
// words of 32, then the u16 cell entries and rate_full over D.
__global__ void k_d2_mark(const int4* __restrict__ map, int cells, uint8_t* __restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cells) return;
  const int4 r = map[i];
  if (r.x >= 0) flag[r.y] = 1;
}

// The words' bits from the flags and their exclusive prefix counts (one workgroup of 1024
// threads, each a contiguous run of words).
__global__ __launch_bounds__(1024) void k_d2_prefix(const uint8_t* __restrict__ flag, int nflag,
                                                    uint2* __restrict__ words, int nwords) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int per = (nwords + 1023) / 1024;
  const int w0 = min(t * per, nwords), w1 = min(w0 + per, nwords);
  uint32_t c = 0;
  for (int w = w0; w < w1; ++w) {
    uint32_t b = 0;
    for (int k = 0; k < 32 && 32 * w + k < nflag; ++k) b |= (uint32_t)(flag[32 * w + k] != 0) << k;
    words[w].x = b;
    c += (uint32_t)__popc(b);
  }
  part[t] = c;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - c;
  for (int w = w0; w < w1; ++w) {
    words[w].y = run;
    run += (uint32_t)__popc(words[w].x);
  }
  if (t == 1023) words[nwords] = make_uint2(part[t], 0u);  // |D|: the rates a copy needs
}

constexpr uint32_t kLds3Rates = 4096;  // rate slots of a mode-3 blob (ranks 0..4094 used)

__global__ void k_lds_map3(const int4* __restrict__ map, int cells, const uint2* __restrict__ words,
                           int d2max, const double* __restrict__ rate_full,
                           uint8_t* __restrict__ blob, int rate_off) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  auto rank = [&](uint32_t d2) {
    const uint2 w = words[d2 >> 5];
    return w.y + (uint32_t)__popc(w.x & ((1u << (d2 & 31u)) - 1u));
  };
  if (i < cells) {
    const int4 r = map[i];
    uint32_t ent = 0xF000u;  // no station in reach
    if (r.x >= 0) {
      const uint32_t k = rank((uint32_t)r.y);
      ent = k < kLds3Rates - 1 ? ((uint32_t)r.x << 12) | k : 0xFFFFu;
    }
    reinterpret_cast<uint16_t*>(blob)[i] = (uint16_t)ent;
  }
  if (i <= d2max && ((words[(uint32_t)i >> 5].x >> (i & 31)) & 1u)) {
    const uint32_t k = rank((uint32_t)i);
    if (k < kLds3Rates - 1) reinterpret_cast<double*>(blob + rate_off)[k] = rate_full[i];
  }
}

// Heterogeneous entities with a shared layout, LDS form (KParams::lds_mode 6, the two-group
// rollout's HET instances), built per layout on the device:
//   k_het_cells: per cell the closest station s* within `reach` (the largest pair d2max; ties to
//     the lower index) and its squared distance, flagged in the set D_cb of its station class cb;
//   k_d2_prefix (per class): the rank index of each D_cb;
//   k_het_info: T = sum |D_cb|, the class bases, and per (UE class cu, station j) the pair's
//     rate offset cu T + base_cb(j) and its largest connectable rank (d2 <= the pair's d2max);
//   k_het_map: the 4-bit s* per cell (15: nothing in reach) and the rates [cu][cb][k] of every
//     pair over D_cb.
__global__ void k_het_cells(const int2* __restrict__ bs, int B, int W, int H, int reach,
                            const uint8_t* __restrict__ bs_cls, int2* __restrict__ cellv,
                            uint8_t* __restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  const int x = i % W, y = i / W;
  long long best = LLONG_MAX;
  int jb = -1;
  for (int j = 0; j < B; ++j) {
    const int2 q = bs[j];
    const long long dx = (long long)x - q.x, dy = (long long)y - q.y;
    const long long d2 = dx * dx + dy * dy;
    if (d2 < best) {
      best = d2;
      jb = j;
    }
  }
  if (jb >= 0 && best <= reach) {
    cellv[i] = make_int2(jb, (int)best);
    flag[(size_t)bs_cls[jb] * (size_t)(reach + 1) + (size_t)best] = 1;
  } else {
    cellv[i] = make_int2(-1, 0);
  }
}

// rank of d2 in D_cb (d2 <= reach) from its rank index; d2 = reach + 1: |D_cb|
__device__ __forceinline__ uint32_t het_rank(const uint2* __restrict__ words, int nwords, uint32_t d2,
                                             uint32_t reach) {
  if (d2 > reach) return words[nwords].x;
  const uint2 w = words[d2 >> 5];
  return w.y + (uint32_t)__popc(w.x & ((1u << (d2 & 31u)) - 1u));
}

// info: [0] the rates a copy needs (the sum of the pairs' runs), [2 + cb NU + cu] the offset of
// pair (cb, cu)'s run of rates, [2 + NB NU + cb NU + cu] its largest connectable rank (-1: none);
// and per (UE class cu, station j) the pair's {offset, largest rank} into the blob at pk
__global__ void k_het_info(const uint2* __restrict__ words, int nwords, int NB, int NU, int B,
                           const uint8_t* __restrict__ bs_cls, const int2* __restrict__ pair,
                           int reach, int2* __restrict__ pk, int* __restrict__ info,
                           const int2* __restrict__ bs, uint32_t* __restrict__ st) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  if (st)  // (mode 6) station j: x | y << 12 | class << 24
    for (int j = 0; j < B; ++j)
      st[j] = ((uint32_t)bs[j].x & 4095u) | (((uint32_t)bs[j].y & 4095u) << 12) | ((uint32_t)bs_cls[j] << 24);
  int off = 0;
  for (int cu = 0; cu < NU; ++cu)
    for (int cb = 0; cb < NB; ++cb) {
      const int dmx = pair[cb * NU + cu].y;  // (-1: the pair never connects)
      const uint2* w = words + (size_t)cb * (nwords + 1);
      const int kmax = dmx < 0 ? -1
                                : (int)het_rank(w, nwords, (uint32_t)min(dmx, reach) + 1u, (uint32_t)reach) - 1;
      info[2 + cb * NU + cu] = off;
      info[2 + NB * NU + cb * NU + cu] = kmax;
      off += min(kmax + 1, (int)kLds3Rates - 1);
    }
  info[0] = off;
  for (int cu = 0; cu < NU; ++cu)
    for (int j = 0; j < B; ++j) {
      const int q = (int)bs_cls[j] * NU + cu;
      pk[cu * B + j] = make_int2(info[2 + q], info[2 + NB * NU + q]);
    }
}

__global__ void k_het_map(const int2* __restrict__ cellv, int cells, const uint2* __restrict__ words,
                          int nwords, int reach, int NB, int NU, const uint8_t* __restrict__ bs_cls,
                          const int2* __restrict__ pair, const double* __restrict__ rate_full,
                          const int* __restrict__ info, uint8_t* __restrict__ blob, int rate_off,
                          int rate_cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i < cells) {  // s* per cell, 4 bits, two cells a byte
    uint32_t v = 0;
    for (int h = 0; h < 2; ++h) {
      const int cl = 2 * i + h;
      const int sx = cl < cells ? cellv[cl].x : -1;
      v |= (uint32_t)(sx < 0 ? 15 : sx) << (4 * h);
    }
    blob[i] = (uint8_t)v;
  }
  const int nd = reach + 1;
  if (i < NB * nd) {
    const int cb = i / nd, d = i - cb * nd;
    const uint2* w = words + (size_t)cb * (nwords + 1);
    if ((w[(uint32_t)d >> 5].x >> (d & 31)) & 1u) {
      const int k = (int)het_rank(w, nwords, (uint32_t)d, (uint32_t)reach);
      for (int cu = 0; cu < NU; ++cu) {
        const int q = cb * NU + cu, at_k = info[2 + q] + k;
        if (k <= info[2 + NB * NU + q] && k < (int)kLds3Rates - 1 && at_k < rate_cap)
          reinterpret_cast<double*>(blob + rate_off)[at_k] = rate_full[pair[q].x + d];
      }
    }
  }
}

// Episode draw table of the envs with mask[e] (all if NULL): pair k of env e = draws 2k and
// 2k + 1 of the stream re-seeded to state0 (what every episode of the env draws, in order),
// and the stream state after them. One thread per (env, pair).
__global__ void k_draw_table(KParams kp, const uint64_t* __restrict__ pcg,
                             const uint8_t* __restrict__ mask, const u128* __restrict__ jump,
                             int* __restrict__ tab_xy, u128* __restrict__ tab_st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int M = kp.tab_m;
  if (i >= (int64_t)kp.E * M) return;
  const int e = (int)(i / M), k = (int)(i - (int64_t)e * M);
  if (mask != nullptr && !mask[e]) return;
  const ulonglong2* pr = reinterpret_cast<const ulonglong2*>(pcg + (size_t)6 * e);
  const ulonglong2 pb = pr[1], pc = pr[2];
  int x, y;
  const u128 s2 = pcg_draw_pair(mk128(pc.x, pc.y), mk128(pb.x, pb.y), 2 * k, jump, kp.Wd, kp.Hd,
                                x, y);
  tab_xy[i] = (int)(((unsigned)x & 0xffffu) | ((unsigned)y << 16));
  tab_st[i] = s2;
}

// The stream state after the env's draws so far into its pcg row, where the kernels left it
// to the draw table (drawn in [1, M]: the state is the table's entry of pair drawn - 1).
__global__ void k_sync_stream_state(int E, int M, const int* __restrict__ drawn,
                                    const u128* __restrict__ tab_st, uint64_t* __restrict__ pcg) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int d = drawn[e];
  if (d < 1 || d > M) return;
  const u128 s = tab_st[(size_t)e * M + (d - 1)];
  *reinterpret_cast<ulonglong2*>(pcg + (size_t)6 * e) = make_ulonglong2((uint64_t)s, (uint64_t)(s >> 64));
}

// A checkpoint restored into this context (mev_restore_stream_state): the pcg rows of the envs
// with mask[e] hold their current stream states, so their draws come from the row, not from
// the episode draw table, until their next reset (drawn > M: the kernels' stream-state path).
__global__ void k_restore_stream_state(int E, int M, const uint8_t* __restrict__ mask,
                                       int* __restrict__ drawn) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E || (mask && !mask[e])) return;
  drawn[e] = M + 1;
}

// Jump table for k in [0, kmax]: a^k and G(k) = 1 + a + ... + a^(k-1) (mod 2^128).
__global__ void k_jump_table(int kmax, u128* __restrict__ jump) {
  const int k0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (k0 > kmax) return;
  u128 acc_mult = 1, acc_plus = 0;
  u128 cur_mult = mk128(PCG_MULT_LO, PCG_MULT_HI), cur_plus = 1;
  unsigned k = (unsigned)k0;
  while (k) {
    if (k & 1u) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    k >>= 1;
  }
  jump[2 * k0] = acc_mult;
  jump[2 * k0 + 1] = acc_plus;
}

}  // namespace

// ======================================================================================
// C ABI
// ======================================================================================
struct mev_ctx {
  mev_params p;
  KParams kp;
  int device;
  int d2max;
  int jmax;
  double* rate_full;
  u128* jump;
  double* util;
  int4* assoc;    // [H][W] association map of the shared layout (mev_update_stations)
  int4* blob;     // its compact LDS form (KTables::lds_blob; null when it does not fit)
  uint2* rankw;   // {bits, prefix} rank index of the sums of two squares <= d2max (global)
  uint2* dwords;  // mode 3: {bits, prefix} of the layout's serving-d2 set D (mev_update_stations)
  uint8_t* dflag; // mode 3: a flag byte per d2 in [0, d2max] (D before its rank index)
  int nwords;     // words of rankw / dwords (d2max / 32 + 1)
  int lds_wgs;    // resident workgroups of the LDSA fused kernel (CUs x per CU)
  int lds2_wgs;   // ... of k_steps_lds2 (0: not used for this context)
  int stage_rows2;
  int stage_cap;  // MEV_STAGE_ROWS (test switch; 0: none)
  int stage_rows; // mode 2: rows of per-env outputs the lean fused kernel stages in LDS (STG)
  int parts;          // mev_step: 1 or 2 env halves (params.stream_split)
  int fuse_steps;     // mev_step(n > 1): one fused launch (params.fuse_steps)
  int* tab_xy;        // episode draw table (params.draw_table), see KTables
  u128* tab_st;
  int* drawn;
  hipStream_t aux;    // second stream of the two-half shape
  hipEvent_t ev_fork, ev_join;
  int scn_allowed;    // MEV_SCN at mev_create (0: the generic rollout instance only)
  int tie_free;       // share_tie_free: the rounded share needs no tie test for this table
  mutable int dcount_h;  // mode 3: |D| of the current layout (INT_MAX: unknown); the
                         // pipelined rollout needs |D| <= 4,094
  int* dcount_pin;       // pinned host word mev_update_stations copies |D| into, stream-ordered
  hipEvent_t ev_dcount;  // recorded after that copy; the first launch that needs |D| waits on it
  mutable int dcount_pending;
  mutable int last_kind;  // mev_last_launch_kind: the kernel the last step / rollout call ran
  int upl;            // k_steps_block: UEs per lane (params.ues_per_lane)
  unsigned char* crec_g;  // per-env layouts, block shape: culling records kept in HBM
  uint8_t* crec_ok;       // (mev_update_layouts; KTables::crec_g)
  int het_packed;     // heterogeneous entities on the packed kernels (U <= 64, shared layout;
                      // one association map per UE class), else the block kernel
  int block_small;    // U <= 64 on the block kernel: per-env layouts on a map beyond 1024 (the
                      // packed kernels' per-env station keys need coordinates < 1024)
  // heterogeneous entities (build_het)
  uint8_t* h_bcl;
  uint8_t* h_ucl;
  int2* h_pair;
  MoveP* h_mv;
  int het_snap_wide;  // some UE's d2snap needs more than 24 bits (velocity >= 4,096): no mode-6
                      // LDS tables (their per-lane word packs d2snap << 8)
  int16_t* h_perm;
  int* h_seg;
  // heterogeneous entities on the two-group rollout: KParams::lds_mode 6 tables of the shared
  // layout (mev_update_stations: k_het_cells / k_d2_prefix / k_het_info / k_het_map; their
  // rate count read back like mode 3's |D|, through dcount_pin); het_lds 0: packed kernels only
  int het_lds;
  int het_reach, het_nwords, het_r100_off, het_st_off, het_rate_off, het_rate_cap, het_cus;
  int het_nib_st, het_words_off;  // (mode 6) station words, rank indices
  int2* het_cell;
  uint8_t* het_flag;
  uint2* het_words;
  int* het_info;
  uint8_t* het_blob;
  mutable size_t het_occ_key;  // (the launch shape het_occ_n was computed for)
  mutable int het_occ_n;
};

static thread_local char g_hip_err[256] = "";

#define MEV_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess) {                                                            \
      snprintf(g_hip_err, sizeof(g_hip_err), "%s:%d %s: %s", __FILE__, __LINE__, #call, \
               hipGetErrorString(_e));                                                 \
      return MEV_EHIP;                                                                 \
    }                                                                                  \
  } while (0)

// Exported functions get C linkage from their declarations in mev.h.

int mev_abi_version(void) { return MEV_ABI_VERSION; }

#ifndef MEV_SRC_HASH
#define MEV_SRC_HASH "unknown"
#endif
const char* mev_source_hash(void) { return MEV_SRC_HASH; }

const char* mev_last_hip_error(void) { return g_hip_err; }

const char* mev_strerror(int code) {
  switch (code) {
    case MEV_OK: return "ok";
    case MEV_EINVAL: return "invalid parameters";
    case MEV_ENOMEM: return "device allocation failed";
    case MEV_EHIP: return g_hip_err[0] ? g_hip_err : "HIP runtime error";
    case MEV_ECHANNEL: return "channel connectivity is not a prefix of the squared distance";
    default: return "unknown error";
  }
}

static int validate(const mev_params* p) {
  if (!p) return MEV_EINVAL;
  if (p->num_envs < 1 || p->num_ues < 1 || p->num_ues > kMaxU) return MEV_EINVAL;
  if (p->compact_state < 0 || p->compact_state > 1 ||
      (p->compact_state && (p->width > 255 || p->height > 255)))
    return MEV_EINVAL;
  if (p->num_bs < 1 || p->num_bs > kMaxB) return MEV_EINVAL;
  if (p->width < 1 || p->height < 1 || p->width > kMaxMap || p->height > kMaxMap) return MEV_EINVAL;
  if (p->ep_max_time < 1 || p->arrival_exit < 1) return MEV_EINVAL;
  if (p->stream_split < 0 || p->stream_split > 2) return MEV_EINVAL;
  // every per-UE buffer below 4 GiB (32-bit byte offsets in the step kernel): E U < 2^28
  if ((int64_t)p->num_envs * p->num_ues >= ((int64_t)1 << 28)) return MEV_EINVAL;
  if (!(p->velocity >= 0.0) || !(p->ue_noise > 0.0) || !(p->util_upper > p->util_lower))
    return MEV_EINVAL;
  if (p->rate_table && (p->rate_table_len < 0 || p->rate_table_len > kD2Top + 1))
    return MEV_EINVAL;
  for (int u = 0; p->ue_velocity && u < p->num_ues; ++u)
    if (!(p->ue_velocity[u] >= 0.0) || !std::isfinite(p->ue_velocity[u])) return MEV_EINVAL;
  if (p->num_bs_classes < 0 || p->num_ue_classes < 0 || p->num_bs_classes > kMaxClasses ||
      p->num_ue_classes > kMaxClasses)
    return MEV_EINVAL;
  if (p->num_bs_classes > 1 || p->num_ue_classes > 1) {
    const int NB = p->num_bs_classes > 1 ? p->num_bs_classes : 1;
    const int NU = p->num_ue_classes > 1 ? p->num_ue_classes : 1;
    if ((NB > 1 && (!p->bs_class || !p->bs_class_params)) ||
        (NU > 1 && (!p->ue_class || !p->ue_class_params)))
      return MEV_EINVAL;
    for (int j = 0; NB > 1 && j < p->num_bs; ++j)
      if (p->bs_class[j] < 0 || p->bs_class[j] >= NB) return MEV_EINVAL;
    for (int u = 0; NU > 1 && u < p->num_ues; ++u)
      if (p->ue_class[u] < 0 || p->ue_class[u] >= NU) return MEV_EINVAL;
    for (int c = 0; NU > 1 && c < NU; ++c)
      if (!(p->ue_class_params[4 * c] >= 0.0) || !(p->ue_class_params[4 * c + 2] > 0.0))
        return MEV_EINVAL;
    if (p->rate_table) {
      if (!p->rate_table_offsets) return MEV_EINVAL;
      for (int i = 0; i < NB * NU; ++i)
        if (p->rate_table_offsets[i] < 0 || p->rate_table_offsets[i + 1] < p->rate_table_offsets[i] ||
            p->rate_table_offsets[i + 1] > p->rate_table_len ||
            p->rate_table_offsets[i + 1] - p->rate_table_offsets[i] > kD2Top + 1)
          return MEV_EINVAL;
    }
  }
  return MEV_OK;
}

typedef void (*StepsKernel)(KParams, KState, KOut, KTables, int, int, int, int);
static StepsKernel steps_kernel_for(bool per_env, bool lean, int ldsm, int U);

// The registered scenario whose constants (scn_const) equal every corresponding value of the
// context, or 0.
static unsigned fbits(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return u;
}
// True when, for every full rate of the table and every share count n <= nmax, the fast
// product of the LDS kernels rounds like the reference: rint(full * fl(100 / n)) ==
// rint(fl(full / n) * 100) (base.py:435, numpy round(., 2)). The rollout kernels then skip the
// tie test and its exact fallback (k_steps_lds2 TF). Exhaustive over the table (~20k entries x
// n), IEEE double on the host like the device's; a table that fails anywhere keeps the test.
static bool share_tie_free(const double* full, int64_t n_d2, int nmax) {
  if (!full || n_d2 <= 0 || nmax < 1 || nmax > kMaxU) return false;
  // (bounded host cost at mev_create: tables x counts beyond 10^8 pairs -- e.g. a 1024 x 1024
  // map where every distance connects, with 1,024 UEs -- keep the tie test instead)
  if ((double)n_d2 * (double)nmax > 1e8) return false;
  for (int n = 1; n <= nmax; ++n) {
    const double r100 = 100.0 / (double)n;
    for (int64_t d = 0; d < n_d2; ++d) {
      const double f = full[d];
      if (rint(f * r100) != rint((f / (double)n) * 100.0)) return false;
    }
  }
  return true;
}

static int match_scn(const mev_ctx* ctx) {
  if (!ctx->scn_allowed) return 0;
  const KParams& kp = ctx->kp;
  for (int s = 1; s <= 4; ++s) {
    const ScnConst c = scn_const(s);
    if ((s >= 3) != (ctx->p.bs_per_env != 0)) continue;
    if ((s == 4) != (kp.U > 64) || kp.het || (kp.st8 != 0) != scn_st8(s)) continue;
    if (kp.U == c.U && kp.B == c.B && kp.W == c.W && kp.H == c.H && kp.tab_m == c.tab_m &&
        kp.hist_lds == c.hist_lds && kp.t_end == c.t_end && kp.arr_start == c.arr_start &&
        kp.arr_exit == c.arr_exit && kp.first_step_active == c.first_step_active &&
        kp.lds_mode == (s == 4 ? 0 : s == 3 ? 4 : 3) && kp.d2max == c.d2max &&
        kp.lds_r100_off == c.lds_r100_off && kp.lds_rate_off == c.lds_rate_off &&
        kp.lds_assoc == c.lds_assoc && kp.d2snap == c.d2snap && kp.axis_exact == c.axis_exact &&
        fbits(kp.vel_f) == c.vel_f && fbits(kp.move_lim) == c.move_lim &&
        fbits(kp.inv_w) == c.inv_w && fbits(kp.inv_h) == c.inv_h &&
        fbits(kp.u_log2_coef) == c.u_log2_coef && fbits(kp.u_w2f) == c.u_w2f &&
        fbits(kp.u_lowerf) == c.u_lowerf && fbits(kp.u_upperf) == c.u_upperf &&
        fbits(kp.u_scale) == c.u_scale && fbits(kp.u_offset) == c.u_offset &&
        kp.cull_log == c.cull_log && kp.cull_nx == c.cull_nx && kp.cull_nc == c.cull_nc)
      return s;
  }
  return 0;
}

// LDS per workgroup of the fused LDSA kernel beyond the tables: each wave's n_b histogram and
// episode draw table.
static size_t lds_per_wave(const KParams& kp) {
  return sizeof(int) * (size_t)kp.envs_per_wave *
         (8 + (size_t)kp.B * kp.hist_lds + kp.tab_m + kp.lbs);
}
// STG staging per wave and row (reward float32 + done byte per env), and for `rows` rows of
// a workgroup of nw waves (only the compile-time-U kernels stage: U = 5, 15, 30)
static size_t stage_bytes_per_row(const KParams& kp) { return 5 * (size_t)kp.envs_per_wave; }
static bool stages(const KParams& kp) { return kp.U == 5 || kp.U == 15 || kp.U == 30; }
static size_t stage_lds_bytes(const KParams& kp, int rows, int nw) {
  return stages(kp) ? ((size_t)rows * nw * stage_bytes_per_row(kp) + 3) & ~(size_t)3 : 0;
}

// The layout-independent parts of the compact association tables (KTables::lds_blob): the
// set S of sums of two squares <= d2max as a rank index, and rate_full over S. Every d2 of a
// UE to a station is a sum of two squares, so rank(d2) indexes the compact rate array for every
// connectable pair. The layout part (cell map, stations) is written by mev_update_stations.
// Leaves c->blob null (the kernel then gathers from `assoc`) when the shape does not qualify:
// more than 15 stations (shared) / 16 (per-env), U > 64, or tables larger than one workgroup's
// share. Per-env layouts get mode 4 (rank index, 100/n, rates over S) for k_steps_lds2.
static int build_lds_tables(mev_ctx* c) {
  KParams& kp = c->kp;
  kp.lds_assoc = 0;
  kp.lds_mode = 0;
  // mev_params.lds_tables: 0 auto (mode 3 where it applies), -1 none, 1..3 force a mode
  const int lt = c->p.lds_tables;
  const bool forced = lt > 0;
  const int want = lt < 0 ? 0 : lt > 0 ? std::min(lt, 3) : 3;
  if (want == 0 || kp.U > 64 || c->d2max < 0) return MEV_OK;
  // per-env layouts (mode 4): the layout-independent rank index of S, 100/n and the rates over
  // S for the two-group kernel (k_steps_lds2<U, 0, true>); the station keys are staged per launch
  const bool lds2_off = c->p.two_groups < 0;  // mev_params.two_groups
  if (c->p.bs_per_env &&
      !(kp.B <= 16 && (kp.U == 15 || kp.U == 30) && kp.tab_m > 0 && !lds2_off))
    return MEV_OK;
  if (!c->p.bs_per_env && kp.B > 15) return MEV_OK;
  const int cells = kp.W * kp.H;
  const int d2max = c->d2max;
  const size_t nwords = (size_t)d2max / 32 + 1;
  std::vector<uint32_t> bits(nwords, 0u);
  for (int a = 0; (int64_t)a * a <= d2max; ++a)
    for (int b = a; (int64_t)a * a + (int64_t)b * b <= d2max; ++b) {
      const int d = a * a + b * b;
      bits[(size_t)d >> 5] |= 1u << (d & 31);
    }
  std::vector<uint32_t> rank(2 * nwords);
  uint32_t count = 0;
  for (size_t w = 0; w < nwords; ++w) {
    rank[2 * w] = bits[w];
    rank[2 * w + 1] = count;
    count += (uint32_t)__builtin_popcount(bits[w]);
  }
  // the rank index in global memory too: k_lds_map derives the per-cell ranks (mode 2)
  if (hipMalloc(&c->rankw, 8 * nwords) != hipSuccess) return MEV_ENOMEM;
  MEV_HIP(hipMemcpy(c->rankw, rank.data(), 8 * nwords, hipMemcpyHostToDevice));
  c->nwords = (int)nwords;
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t nib_bytes = up16(((size_t)cells + 1) / 2);
  // mode 2: [cell nibbles][cell ranks u16][100/n][rates]; mode 1: [cell nibbles][stations]
  // [rank index][100/n][rates]
  size_t st_off = 0, rank_off = 0, r16_off = 0, r100_off, rate_off, total;
  int mode = 0;
  if (c->p.bs_per_env) {
    r100_off = up16(8 * nwords);
    rate_off = r100_off + 8 * 72;
    total = up16(rate_off + 8 * (size_t)count);
    const int G = kp.envs_per_wave;
    const size_t sh2 = total + kLds2Waves * lds2_per_wave(G, kp.B, kp.tab_m, 2, true);
    const size_t row2 = (size_t)kLds2Waves * G * 2 * kStage2Bytes;
    if (sh2 + row2 + 4 > (size_t)kLds2BytesPerWG) return MEV_OK;
    std::vector<double> fullp((size_t)d2max + 1);
    MEV_HIP(hipMemcpy(fullp.data(), c->rate_full, sizeof(double) * fullp.size(),
                      hipMemcpyDeviceToHost));
    std::vector<char> host(total, 0);
    memcpy(host.data(), rank.data(), 8 * nwords);
    double* r100p = reinterpret_cast<double*>(host.data() + r100_off);
    for (int n = 1; n <= 64; ++n) r100p[n] = 100.0 / (double)n;
    double* ratesp = reinterpret_cast<double*>(host.data() + rate_off);
    for (int d = 0, k = 0; d <= d2max; ++d)
      if ((bits[(size_t)d >> 5] >> (d & 31)) & 1u) ratesp[k++] = fullp[(size_t)d];
    if (hipMalloc(&c->blob, total) != hipSuccess) return MEV_ENOMEM;
    MEV_HIP(hipMemcpy(c->blob, host.data(), total, hipMemcpyHostToDevice));
    kp.lds_assoc = (int)total;
    kp.lds_mode = 4;
    kp.lds_rank_off = 0;
    kp.lds_r100_off = (int)r100_off;
    kp.lds_rate_off = (int)rate_off;
    c->stage_cap = c->p.stage_rows > 0 ? c->p.stage_rows : 0;
    c->stage_rows2 = (int)(((size_t)kLds2BytesPerWG - sh2 - 4) / row2);
    if (c->stage_cap > 0) c->stage_rows2 = std::min(c->stage_rows2, c->stage_cap);
    int cus = 0, n2 = 0;
    MEV_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    MEV_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &n2, reinterpret_cast<const void*>(kp.U == 15 ? k_steps_lds2<15, 0, true>
                                                      : k_steps_lds2<30, 0, true>),
        64 * kLds2Waves, sh2 + (((size_t)c->stage_rows2 * row2 + 3) & ~(size_t)3)));
    c->lds2_wgs = cus * n2;
    return MEV_OK;
  }
  // mode 3 for aligned env segments (U -> 16 / 32 lanes); measured slower than mode 1 for
  // mobile-small (U = 5: 162 vs 142 us per 40-step launch at 65,536 envs)
  const bool aligned = pitch_of(kp.U) == 16 || pitch_of(kp.U) == 32;
  if (want >= 3 && cells <= 65536 && (aligned || forced)) {  // [cell entries u16][100/n][rates over D]
    r100_off = up16(2 * (size_t)cells);
    rate_off = r100_off + 8 * 72;
    total = up16(rate_off + 8 * (size_t)kLds3Rates);
    if (total + kLds2Waves * (lds_per_wave(kp) + stage_bytes_per_row(kp)) + 4 <=
        (size_t)kLds2BytesPerWG) {
      if (hipMalloc(&c->dwords, 8 * (nwords + 1)) != hipSuccess) return MEV_ENOMEM;
      if (hipMalloc(&c->dflag, (size_t)d2max + 1) != hipSuccess) return MEV_ENOMEM;
      mode = 3;
    }
  }
  if (!mode && want >= 2 && count < 65536) {
    r16_off = nib_bytes;
    r100_off = up16(r16_off + 2 * (size_t)cells);
    rate_off = r100_off + 8 * 72;
    total = up16(rate_off + 8 * (size_t)count);
    // (+ at least one staged row of per-env outputs, k_steps_packed STG)
    if (total + kLds2Waves * (lds_per_wave(kp) + stage_bytes_per_row(kp)) + 4 <=
        (size_t)kLds2BytesPerWG)
      mode = 2;
  }
  if (!mode) {
    st_off = nib_bytes;
    rank_off = st_off + 64;
    r100_off = up16(rank_off + 8 * nwords);  // 100 / n for n in [0, 64]
    rate_off = r100_off + 8 * 72;
    total = up16(rate_off + 8 * (size_t)count);
    if (total + kLdsWaves * lds_per_wave(kp) > (size_t)kLdsBytesPerWG) return MEV_OK;
    mode = 1;
  }
  std::vector<double> full((size_t)d2max + 1);
  MEV_HIP(hipMemcpy(full.data(), c->rate_full, sizeof(double) * full.size(),
                    hipMemcpyDeviceToHost));
  const size_t host_off = mode >= 2 ? r100_off : st_off;  // the layout-independent part
  std::vector<char> host(total - host_off, 0);
  if (mode == 1) memcpy(host.data() + (rank_off - host_off), rank.data(), 8 * nwords);
  double* r100 = reinterpret_cast<double*>(host.data() + (r100_off - host_off));
  for (int n = 1; n <= 64; ++n) r100[n] = 100.0 / (double)n;  // correctly rounded (IEEE host)
  double* rates = reinterpret_cast<double*>(host.data() + (rate_off - host_off));
  if (mode <= 2)
    for (int d = 0, k = 0; d <= d2max; ++d)
      if ((bits[(size_t)d >> 5] >> (d & 31)) & 1u) rates[k++] = full[(size_t)d];
  if (hipMalloc(&c->blob, total) != hipSuccess) return MEV_ENOMEM;
  if (mode == 3) {  // no station anywhere until a layout is set (0xF000), rates zero
    MEV_HIP(hipMemset(c->blob, 0, total));
    MEV_HIP(hipMemsetD16(reinterpret_cast<hipDeviceptr_t>(c->blob), 0xF000, (size_t)cells));
  }
  if (mode <= 2) MEV_HIP(hipMemset(c->blob, 0xff, nib_bytes));  // no station anywhere until a layout is set
  if (mode == 2) MEV_HIP(hipMemset(reinterpret_cast<char*>(c->blob) + r16_off, 0, r100_off - r16_off));
  MEV_HIP(hipMemcpy(reinterpret_cast<char*>(c->blob) + host_off, host.data(), host.size(),
                    hipMemcpyHostToDevice));
  kp.lds_assoc = (int)total;
  kp.lds_mode = mode;
  kp.lds_st_off = (int)st_off;
  kp.lds_rank_off = (int)rank_off;
  kp.lds_r16_off = (int)r16_off;
  kp.lds_rate_off = (int)rate_off;
  kp.lds_r100_off = (int)r100_off;
  // persistent grid: every resident workgroup (the fewer of the two output variants)
  int cus = 0;
  MEV_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  const int nw = lds_waves(mode);
  const size_t shmem = total + nw * lds_per_wave(kp);
  c->stage_rows = mode >= 2 ? (int)(((size_t)kLds2BytesPerWG - shmem - 4) /
                                    (nw * stage_bytes_per_row(kp)))
                            : 0;
  c->stage_cap = c->p.stage_rows > 0 ? c->p.stage_rows : 0;  // shorter staging windows
  if (c->stage_cap > 0) c->stage_rows = std::min(c->stage_rows, c->stage_cap);
  int per = 1 << 30;
  for (int lean = 0; lean < 2; ++lean) {
    int n = 0;
    MEV_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &n, reinterpret_cast<const void*>(steps_kernel_for(false, lean != 0, mode, kp.U)),
        64 * nw, shmem + (lean ? stage_lds_bytes(kp, c->stage_rows, nw) : 0)));
    per = std::min(per, n);
  }
  c->lds_wgs = cus * per;
  // two env groups per wavefront (k_steps_lds2): mode 3, U = 15 / 30, a draw table
  c->lds2_wgs = 0;
  if (mode == 3 && (kp.U == 15 || kp.U == 30) && kp.tab_m > 0 && !lds2_off) {
    const int G = kp.envs_per_wave;
    const size_t sh2 = total + kLds2Waves * lds2_per_wave(G, kp.B, kp.tab_m, 2);
    const size_t row2 = (size_t)kLds2Waves * G * 2 * kStage2Bytes;
    if (sh2 + row2 + 4 <= (size_t)kLds2BytesPerWG) {
      c->stage_rows2 = (int)(((size_t)kLds2BytesPerWG - sh2 - 4) / row2);
      if (c->stage_cap > 0) c->stage_rows2 = std::min(c->stage_rows2, c->stage_cap);
      int n2 = 0;
      MEV_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &n2, reinterpret_cast<const void*>(kp.U == 15 ? k_steps_lds2<15, 0> : k_steps_lds2<30, 0>),
          64 * kLds2Waves, sh2 + (((size_t)c->stage_rows2 * row2 + 3) & ~(size_t)3)));
      c->lds2_wgs = cus * n2;
    }
  }
  if (c->lds_wgs <= 0) {  // cannot be resident: the L2 gather path
    (void)hipFree(c->blob);
    c->blob = nullptr;
    kp.lds_assoc = 0;
    kp.lds_mode = 0;
  }
  return MEV_OK;
}

// Channel.calculateSNR + Channel.datarate at integer squared distance d2 on the host, float64,
// the reference's operation order (OkumuraHata.power_loss channels.py:133-146: shapely's
// distance = sqrt(d2); calculateSNR channels.py:24-27; datarate channels.py:78-83).
static double host_snr(const mev_params* p, int64_t d2) {
  const double distance = sqrt((double)d2);
  const double f = p->bs_freq, hb = p->bs_height, hu = p->ue_height;
  const double ch = 0.8 + (1.1 * log10(f) - 0.7) * hu - 1.56 * log10(f);
  const double tmp_1 = 69.55 - ch + 26.16 * log10(f) - 13.82 * log10(hb);
  const double tmp_2 = 44.9 - 6.55 * log10(hb);
  const double loss = tmp_1 + tmp_2 * log10(distance + 1e-16);
  const double power = pow(10.0, (p->bs_tx - loss) / 10.0);
  return power / p->ue_noise;
}

int64_t mev_build_rate_table(const mev_params* p, double* dst, int64_t cap) {
  if (!p || cap < 0 || (cap > 0 && !dst)) return MEV_EINVAL;
  if (p->width < 1 || p->height < 1 || p->width > kMaxMap || p->height > kMaxMap) return MEV_EINVAL;
  // connectable d2 = a prefix [0, n): scanned over the map's squared distances, and over every
  // station distance (coordinates < 1024) when the whole map range connects; on maps beyond
  // 1024 the scan stops at kD2Top, and a channel that still connects there is refused (its
  // keys would not hold the distance)
  const int64_t map_hi = (int64_t)(p->width - 1) * (p->width - 1) +
                         (int64_t)(p->height - 1) * (p->height - 1);
  int64_t n = 0;
  bool prefix = true;
  for (int64_t d2 = 0; d2 <= kD2Top; ++d2) {
    if (d2 > map_hi && n <= map_hi) break;  // the map's range decided it
    const double snr = host_snr(p, d2);
    if (snr > p->ue_snr_tr) {
      if (n != d2) prefix = false;
      if (d2 < cap) dst[d2] = p->bs_bw * log2(1.0 + snr);
      n = d2 + 1;
    }
  }
  if (map_hi > kD2Top && n == kD2Top + 1) return MEV_EINVAL;
  return prefix ? n : MEV_ECHANNEL;
}

// Movement parameters of a velocity (host IEEE float64 == device): the arrival threshold
// d2snap = largest integer d2 with sqrt(d2) <= velocity, axis-parallel exactness, the float32
// fast path's velocity and tie band (move_ue_p).
static MoveP host_move_params(double velocity, int W, int H, bool v15 = true) {
  MoveP mp;
  mp.vel = velocity;
  mp.vel_f = (float)velocity;
  const float band = 0x1p-16f * (velocity > 1.0 ? (float)velocity : 1.0f);
  mp.move_lim = 0.5f - band;
  const int d2_top = (W - 1) * (W - 1) + (H - 1) * (H - 1);
  int d2 = 0;
  while (d2 <= d2_top && sqrt((double)d2) <= velocity) ++d2;
  mp.d2snap = d2 - 1;
  mp.axis_exact = 1;
  const int amax = W > H ? W : H;
  for (int a = 1; a <= amax; ++a)
    if ((velocity * (double)a) / (double)a != velocity) mp.axis_exact = 0;
  // an integer velocity: an axis move is pos +- velocity, no tie, and the float32 fast path
  // (q = +-velocity within 5e-7 relative, far from a half-integer) gives it -- no axis branch
  if (velocity == floor(velocity) && velocity <= 0x1p20) mp.axis_exact = 0;
  // velocity 1.5 on maps up to 1024: the exact integer step (step_v15)
  if (v15 && velocity == 1.5 && W <= 1024 && H <= 1024) mp.axis_exact = 2;
  return mp;
}

static bool is_het(const mev_params* p) {
  return p->num_bs_classes > 1 || p->num_ue_classes > 1 || p->ue_velocity != nullptr;
}

// Heterogeneous entities: class arrays, per-pair channel tables (the caller's, else libm per
// pair), per-UE-class movement parameters, stations grouped by class. Fills c->rate_full and
// the KTables het pointers; kp.d2max = the largest pair d2max.
static int build_het(mev_ctx* c) {
  const mev_params* p = &c->p;
  KParams& kp = c->kp;
  const int NB = std::max(1, p->num_bs_classes), NU = std::max(1, p->num_ue_classes);
  const int B = p->num_bs, U = p->num_ues;
  std::vector<uint8_t> bcl(B, 0), ucl(U, 0);
  for (int j = 0; j < B; ++j) bcl[j] = (uint8_t)(p->bs_class ? p->bs_class[j] : 0);
  for (int u = 0; u < U; ++u) ucl[u] = (uint8_t)(p->ue_class ? p->ue_class[u] : 0);
  // per-pair tables, concatenated
  std::vector<double> all;
  std::vector<int2> pair((size_t)NB * NU);
  for (int cb = 0; cb < NB; ++cb)
    for (int cu = 0; cu < NU; ++cu) {
      const int pi = cb * NU + cu;
      mev_params q = *p;
      if (p->bs_class_params) {
        q.bs_bw = p->bs_class_params[4 * cb];
        q.bs_freq = p->bs_class_params[4 * cb + 1];
        q.bs_tx = p->bs_class_params[4 * cb + 2];
        q.bs_height = p->bs_class_params[4 * cb + 3];
      }
      if (p->ue_class_params) {
        q.ue_snr_tr = p->ue_class_params[4 * cu + 1];
        q.ue_noise = p->ue_class_params[4 * cu + 2];
        q.ue_height = p->ue_class_params[4 * cu + 3];
      }
      int64_t n;
      const size_t off = all.size();
      if (p->rate_table) {
        // one class pair (per-UE velocities only): validate() requires no offsets, the whole
        // table is that pair's
        const bool whole = !p->rate_table_offsets && NB * NU == 1;
        const int64_t a = whole ? 0 : p->rate_table_offsets[pi];
        const int64_t b = whole ? p->rate_table_len : p->rate_table_offsets[pi + 1];
        n = b - a;
        all.insert(all.end(), p->rate_table + a, p->rate_table + b);
      } else {
        n = mev_build_rate_table(&q, nullptr, 0);
        if (n < 0) return (int)n;
        all.resize(off + (size_t)n);
        if (n) (void)mev_build_rate_table(&q, all.data() + off, n);
      }
      pair[pi] = make_int2((int)off, (int)n - 1);
      kp.d2max = std::max(kp.d2max, (int)n - 1);
    }
  all.push_back(0.0);  // (never indexed; keeps the buffer non-empty)
  // movement parameters per UE: its own velocity (ue_velocity), else its class's; distinct
  // velocities need no class (velocity only drives movement, movement.py:42-62)
  // (the integer step of velocity 1.5, step_v15, only when every UE moves at 1.5: a wave of
  // mixed velocities issues both movement paths, and the float32 path with its tie fallback is
  // exact for 1.5 as for any velocity)
  std::vector<double> vel(U);
  bool all15 = true;
  for (int u = 0; u < U; ++u) {
    vel[u] = p->ue_velocity ? p->ue_velocity[u]
             : p->ue_class_params ? p->ue_class_params[4 * ucl[u]] : p->velocity;
    all15 = all15 && vel[u] == 1.5;
  }
  std::vector<MoveP> mv(U);
  for (int u = 0; u < U; ++u) mv[u] = host_move_params(vel[u], p->width, p->height, all15);
  c->het_snap_wide = 0;
  for (int u = 0; u < U; ++u) c->het_snap_wide |= mv[u].d2snap >= (1 << 24) ? 1 : 0;
  // stations grouped by class, each segment padded to an even length (pairs of keys)
  std::vector<int16_t> perm;
  std::vector<int> seg(NB + 1, 0);
  for (int cb = 0; cb < NB; ++cb) {
    seg[cb] = (int)perm.size();
    for (int j = 0; j < B; ++j)
      if (bcl[j] == cb) perm.push_back((int16_t)j);
    if (perm.size() & 1) perm.push_back(-1);
  }
  seg[NB] = (int)perm.size();
  kp.het = 1;
  kp.cull_log = kp.cull_nx = kp.cull_nc = 0;  // (class segments: no culling)
  kp.nb_cls = NB;
  kp.nu_cls = NU;
  kp.bperm = (int)perm.size();
  if (hipMalloc(&c->rate_full, sizeof(double) * all.size()) != hipSuccess ||
      hipMalloc(&c->h_bcl, (size_t)B) != hipSuccess || hipMalloc(&c->h_ucl, (size_t)U) != hipSuccess ||
      hipMalloc(&c->h_pair, sizeof(int2) * pair.size()) != hipSuccess ||
      hipMalloc(&c->h_mv, sizeof(MoveP) * mv.size()) != hipSuccess ||
      hipMalloc(&c->h_perm, sizeof(int16_t) * std::max<size_t>(perm.size(), 1)) != hipSuccess ||
      hipMalloc(&c->h_seg, sizeof(int) * seg.size()) != hipSuccess)
    return MEV_ENOMEM;
  MEV_HIP(hipMemcpy(c->rate_full, all.data(), sizeof(double) * all.size(), hipMemcpyHostToDevice));
  MEV_HIP(hipMemcpy(c->h_bcl, bcl.data(), (size_t)B, hipMemcpyHostToDevice));
  MEV_HIP(hipMemcpy(c->h_ucl, ucl.data(), (size_t)U, hipMemcpyHostToDevice));
  MEV_HIP(hipMemcpy(c->h_pair, pair.data(), sizeof(int2) * pair.size(), hipMemcpyHostToDevice));
  MEV_HIP(hipMemcpy(c->h_mv, mv.data(), sizeof(MoveP) * mv.size(), hipMemcpyHostToDevice));
  if (!perm.empty())
    MEV_HIP(hipMemcpy(c->h_perm, perm.data(), sizeof(int16_t) * perm.size(), hipMemcpyHostToDevice));
  MEV_HIP(hipMemcpy(c->h_seg, seg.data(), sizeof(int) * seg.size(), hipMemcpyHostToDevice));
  c->d2max = kp.d2max;
  return MEV_OK;
}

// The two-group rollout's tables for heterogeneous entities with a shared layout (lds_mode 6),
// allocated here and filled per layout by mev_update_stations (blob layout below). Eligible:
// U = 15 / 30, at most 15 stations (4-bit station field), a draw table, cells < 65,536 rounded
// into LDS beside at least one wavefront, every UE's d2snap within 24 bits; two_groups >= 0 and
// lds_tables >= 0.
static int build_het_lds(mev_ctx* c) {
  const KParams& kp = c->kp;
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  c->het_lds = 0;
  const size_t cells = (size_t)c->p.width * c->p.height;
  if (!c->het_packed || c->p.two_groups < 0 || c->p.lds_tables < 0 || !(kp.U == 15 || kp.U == 30) ||
      kp.B > 15 || kp.tab_m <= 0 || cells >= 65536 || c->d2max < 0 || c->het_snap_wide ||
      c->p.width > 4096 || c->p.height > 4096)
    return MEV_OK;
  const int NB = kp.nb_cls, NU = kp.nu_cls;
  const size_t nwords = (size_t)c->d2max / 32 + 1;
  // mode 6: [0, nib) 4-bit s* per cell; [st, +64) station x | y << 12 | class << 24; [pk,
  // +8 NU B) pairs; [words, +8 NB (nwords + 1)) the classes' rank indices; [r100, +576); rates.
  const size_t nib_bytes = up16((cells + 1) / 2);
  const size_t pk6 = nib_bytes + 64, words6 = up16(pk6 + 8 * (size_t)NU * kp.B);
  const size_t r100_off = up16(words6 + 8 * (size_t)NB * (nwords + 1));
  const size_t st_off = pk6;  // (the pairs' table)
  const size_t rate_off = up16(r100_off + 8 * 72);
  const size_t one_wave = lds2_per_wave(kp.envs_per_wave, kp.B, kp.tab_m, 1) +
                          (size_t)2 * kp.envs_per_wave * kStage2Bytes + 4;
  if (rate_off + one_wave + 8 * 64 > (size_t)kLds2BytesPerWG) return MEV_OK;
  const int cap = (int)(((size_t)kLds2BytesPerWG - rate_off) / 8);
  c->het_reach = c->d2max;
  c->het_nwords = c->d2max / 32 + 1;
  const size_t nd = (size_t)c->d2max + 1;
  if (hipMalloc(&c->het_cell, sizeof(int2) * cells) != hipSuccess ||
      hipMalloc(&c->het_flag, (size_t)NB * nd) != hipSuccess ||
      hipMalloc(&c->het_words, sizeof(uint2) * (size_t)NB * (c->het_nwords + 1)) != hipSuccess ||
      hipMalloc(&c->het_info, sizeof(int) * (2 + 2 * (size_t)NB * NU)) != hipSuccess ||
      hipMalloc(&c->het_blob, rate_off + 8 * (size_t)cap) != hipSuccess)
    return MEV_ENOMEM;
  MEV_HIP(hipMemset(c->het_blob, 0, rate_off + 8 * (size_t)cap));
  MEV_HIP(hipMemset(c->het_blob, 0xff, (cells + 1) / 2));  // no station until a layout
  double r100[72] = {0.0};
  for (int n = 1; n <= 64; ++n) r100[n] = 100.0 / (double)n;  // correctly rounded (IEEE host)
  MEV_HIP(hipMemcpy(c->het_blob + r100_off, r100, sizeof(r100), hipMemcpyHostToDevice));
  const int zero = 0;
  MEV_HIP(hipMemcpy(c->het_info, &zero, sizeof(int), hipMemcpyHostToDevice));
  c->het_r100_off = (int)r100_off;
  c->het_st_off = (int)st_off;
  c->het_nib_st = (int)nib_bytes;
  c->het_words_off = (int)words6;
  c->het_rate_off = (int)rate_off;
  c->het_rate_cap = cap;
  MEV_HIP(hipDeviceGetAttribute(&c->het_cus, hipDeviceAttributeMultiprocessorCount, c->device));
  c->het_lds = 1;
  return MEV_OK;
}

static KTables tables_of(const mev_ctx* c) {
  KTables tb{};
  tb.rate_full = c->rate_full;
  tb.jump = c->jump;
  tb.util = c->util;
  tb.assoc = c->assoc;
  tb.tab_xy = c->tab_xy;
  tb.tab_st = c->tab_st;
  tb.drawn = c->drawn;
  tb.lds_blob = c->blob;
  tb.dcount = (c->blob && c->kp.lds_mode == 3 && c->dwords)
                  ? reinterpret_cast<const int*>(c->dwords + c->nwords) : nullptr;
  tb.bs_cls = c->h_bcl;
  tb.ue_cls = c->h_ucl;
  tb.pair = c->h_pair;
  tb.mv = c->h_mv;
  tb.perm = c->h_perm;
  tb.seg = c->h_seg;
  tb.crec_g = c->crec_g;
  tb.crec_ok = c->crec_ok;
  return tb;
}

// The packed step shape (several envs per wavefront), else the block shape (a workgroup per env).
static bool packed_shape(const mev_ctx* c) {
  return c->kp.U <= 64 && (!c->kp.het || c->het_packed) && !c->block_small;
}

// The body of mev_create on a value-initialised context; on any failure the caller releases
// what was allocated so far (mev_destroy takes a partly built context), so every early return
// -- a HIP error included -- leaves nothing behind.
static int create_ctx(mev_ctx* c, const mev_params* params) {
  int rc = 0;
  c->p = *params;
  if (c->p.ue_velocity) {  // one velocity for every UE: the homogeneous kernels
    bool same = true;
    for (int u = 1; u < c->p.num_ues; ++u) same = same && c->p.ue_velocity[u] == c->p.ue_velocity[0];
    if (same) {
      c->p.velocity = c->p.ue_velocity[0];
      c->p.ue_velocity = nullptr;
    }
  }
  params = &c->p;  // (normalised; ue_velocity is read only while creating)
  MEV_HIP(hipGetDevice(&c->device));

  KParams& kp = c->kp;
  kp.E = params->num_envs;
  kp.U = params->num_ues;
  kp.B = params->num_bs;
  kp.W = params->width;
  kp.H = params->height;
  kp.t_end = params->ep_max_time < params->arrival_exit ? params->ep_max_time
                                                         : params->arrival_exit;
  kp.arr_start = params->arrival_start;
  kp.arr_exit = params->arrival_exit;
  kp.first_step_active = params->first_step_active;
  kp.movement_reseed = params->movement_reseed;
  kp.envs_per_wave = params->num_ues <= 64 ? 64 / params->num_ues : 1;
  kp.hist_lds = params->num_ues <= 64 && kp.envs_per_wave * params->num_bs <= 1024;
  // 16 station key slots {m, c} per env (2 ints each; see k_steps_packed's staging)
  kp.lbs = (params->bs_per_env && params->num_bs <= 16 && params->num_ues <= 64) ? 32 : 0;
  kp.Wd = (double)params->width;
  kp.Hd = (double)params->height;
  kp.vel = params->velocity;
  kp.lower = params->util_lower;
  kp.qoe_low = params->qoe_low;
  kp.upper = params->util_upper;
  kp.w1 = params->util_w1;
  kp.w2 = params->util_w2;
  kp.log_w3 = log(params->util_w3);
  kp.inv_w = 1.0f / (float)params->width;
  kp.inv_h = 1.0f / (float)params->height;
  kp.srv_bits = 0;
  while ((1 << kp.srv_bits) < params->num_bs) ++kp.srv_bits;
  kp.util_sat = 2.0 * (kp.upper - kp.lower) / (kp.upper - kp.lower) - 1.0;
  kp.u_log2_coef = (float)(kp.w1 * log(2.0) / kp.log_w3);
  kp.u_w2f = (float)kp.w2;
  kp.u_lowerf = (float)kp.lower;
  kp.u_upperf = (float)kp.upper;
  kp.u_scale = (float)(2.0 / (kp.upper - kp.lower));
  kp.u_offset = (float)(-2.0 * kp.lower / (kp.upper - kp.lower) - 1.0);
  // with offset 0 and w2 0 the float32 utility is ur * scale with ur = c log2(r): its relative
  // error is that of log2 at r = cents / 100 != 1 (|log2 r| >= log2 1.01), within 1e-5; otherwise
  // the sum cancels near the utility's zero and only an absolute bound holds (utility_f32r)
  kp.util_exact = (kp.u_offset != 0.f || kp.u_w2f != 0.f) ? 1 : 0;
  kp.xcd_remap = params->xcd_remap < 0 ? 0 : params->xcd_remap > 1 ? 1 + (params->xcd_remap - 1) % 8 : 1;
  kp.st8 = params->compact_state;
  if (params->num_ues > 64 && params->station_culling >= 0) {  // block kernel (block_cull_params)
    const CullP cp = block_cull_params(params->num_bs, params->width, params->height,
                                       false);
    kp.cull_log = cp.log;
    kp.cull_nx = cp.nx;
    kp.cull_nc = cp.nc;
  }
  // UEs per lane of the block kernel: 1 / 2 forced, 0 per launch (launch_block_steps)
  c->upl = params->ues_per_lane == 1 || params->ues_per_lane == 2 ? params->ues_per_lane : 0;
  if (is_het(params)) c->upl = 1;
  {
    const MoveP mp = host_move_params(params->velocity, params->width, params->height);
    kp.vel_f = mp.vel_f;
    kp.move_lim = mp.move_lim;
    kp.move_band = 0.5f - mp.move_lim;
    kp.d2snap = mp.d2snap;
    kp.axis_exact = mp.axis_exact;
  }
  // utility saturation point r_sat = w3^(upper/w1) - w2 (increasing utility only)
  kp.util_direct = 1;
  kp.util_kmax = 0;
  if (kp.w1 > 0.0 && params->util_w3 > 1.0 && kp.w2 >= 0.0) {
    const double r_sat = exp(kp.upper * kp.log_w3 / kp.w1) - kp.w2;
    const double kmax = ceil((r_sat > 0.0 ? r_sat : 0.0) * 100.0 * 1.01) + 16.0;
    if (std::isfinite(kmax) && kmax < (double)(1 << 22)) {
      kp.util_direct = 0;
      kp.util_kmax = (int)kmax;
      // the float32 utility's absolute error (utility_f32r), the sum of: the rate's float32
      // rounding and w2's (3 ulp relative, 2.2e-8 for 0.01f) through log2 (1 / ln 2 per relative
      // unit) times the slope A = |w1 ln2 / ln w3 * scale|; v_log_f32 (taken as 2^-22
      // max(|log2 x|, 1) over the table's rates, x = w2 + 0.01 .. w2 + r_sat: twice its measured
      // worst case, 0.993 * 2^-23 max(|log2 x|, 1) over every float32 x in [2^-8, 2^8),
      // tools/log2_probe.hip); the products, clip bounds and offset (2 ulp each of
      // max(|lower|, |upper|) * scale, 1, |offset|, where their roundings come to <= 1 ulp).
      // (Rounds <= 5 doubled this sum: at the defaults a band of |mean| <= 0.166 instead of
      // 0.086, which took 8.3 % of mobile-small's env-steps to the exact path instead of 2.7 %.)
      const double A = fabs(kp.w1 * log(2.0) / kp.log_w3 * (2.0 / (kp.upper - kp.lower)));
      const double lmax = std::max({1.0, fabs(log2(kp.w2 + 0.01)), fabs(log2(kp.w2 + std::max(r_sat, 0.01)))});
      const double off = fabs(-2.0 * kp.lower / (kp.upper - kp.lower) - 1.0);
      const double sc = std::max(fabs(kp.lower), fabs(kp.upper)) * 2.0 / (kp.upper - kp.lower);
      kp.u_err = (float)(A * ((3.0 * 0x1p-24 + 2.2e-8) / log(2.0) + 0x1p-22 * lmax) +
                         0x1p-22 * (1.0 + off + sc));
      if (params->reward_exact > 0) kp.u_err = INFINITY;  // (every row takes the exact path)
      // (tests: a band -reward_exact times wider, so that a subset of rows takes the exact path)
      if (params->reward_exact < -1) kp.u_err *= (float)-params->reward_exact;
      // |sum| 9.5e-6 <= nact (u_err + q) as bounds on the mean (q = 2^-24, the coarser fixed
      // point; 0.1 % wider): |mean| <= r_thr, and on the 2^-25 sum |isum| <= nact r_thr25, unsigned
      // (every |isum| <= nact 2^25 <= 2^31: the caps take every row in reward_exact)
      const double thr = (kp.u_err + 0x1p-24) / 9.5e-6 * 1.001;
      kp.r_thr = (float)std::min(thr, 4.0);
      kp.r_thr25 = (int)std::min(std::ceil(thr * 0x1p25), (double)(1 << 25));
    }
  }

  // ---- channel table: the caller's (numpy, Python host), else built here with libm ----
  if (is_het(params)) {
    c->kp.d2max = -1;
    rc = build_het(c);
    if (rc) {
      return rc;
    }
  } else {
    std::vector<double> host;
    const double* tab = params->rate_table;
    int64_t n = params->rate_table_len;
    if (tab == nullptr) {
      n = mev_build_rate_table(params, nullptr, 0);
      if (n < 0) {
        return (int)n;
      }
      host.resize((size_t)std::max<int64_t>(n, 1));
      (void)mev_build_rate_table(params, host.data(), n);
      tab = host.data();
    }
    c->d2max = (int)n - 1;
    c->kp.d2max = c->d2max;
    // (one entry at least: lanes without a server read entry 0 unconditionally)
    if (hipMalloc(&c->rate_full, sizeof(double) * (size_t)std::max<int64_t>(n, 1)) != hipSuccess) {
      return MEV_ENOMEM;
    }
    MEV_HIP(hipMemset(c->rate_full, 0, sizeof(double)));
    if (n > 0) MEV_HIP(hipMemcpy(c->rate_full, tab, sizeof(double) * (size_t)n, hipMemcpyHostToDevice));
    c->tie_free = share_tie_free(tab, n, params->num_ues);
  }
  c->scn_allowed = params->scenario_constants >= 0;
  c->dcount_h = INT_MAX;  // (mev_update_stations reads |D| back)
  c->dcount_pending = 0;

  // ---- episode draw table (packed shape, movement re-seeded every episode) ----
  c->kp.tab_m = 0;
  if (params->draw_table != 0 && params->movement_reseed)
    c->kp.tab_m = params->draw_table > 0 ? params->draw_table : 3 * params->num_ues + 8;
  if (c->kp.tab_m) {
    const size_t n = (size_t)params->num_envs * (size_t)c->kp.tab_m;
    if (c->kp.tab_m < params->num_ues || n >= ((size_t)1 << 28) ||
        hipMalloc(&c->tab_xy, sizeof(int) * n) != hipSuccess ||
        hipMalloc(&c->tab_st, sizeof(u128) * n) != hipSuccess ||
        hipMalloc(&c->drawn, sizeof(int) * (size_t)params->num_envs) != hipSuccess) {
      const bool bad = c->kp.tab_m < params->num_ues || n >= ((size_t)1 << 28);
      return bad ? MEV_EINVAL : MEV_ENOMEM;
    }
    MEV_HIP(hipMemset(c->drawn, 0, sizeof(int) * (size_t)params->num_envs));
  }

  // ---- PCG64 jump table: offsets up to 2U (reset) + 2U (waypoints), and the table pairs --
  c->jmax = max(4 * params->num_ues, 2 * c->kp.tab_m + 2);
  if (hipMalloc(&c->jump, sizeof(u128) * 2 * (size_t)(c->jmax + 1)) != hipSuccess) {
    return MEV_ENOMEM;
  }
  hipLaunchKernelGGL(k_jump_table, dim3((c->jmax + 256) / 256), dim3(256), 0, 0, c->jmax,
                     c->jump);
  MEV_HIP(hipGetLastError());

  // ---- association map of a shared layout (filled by mev_reset / mev_update_stations), only
  //      for the packed kernels (U <= 64) that gather from it: W x H x 16 B per map (268 MB at
  //      4,096^2), one per UE class with heterogeneous entities. Heterogeneous maps of 4 GiB or
  //      more (32-bit byte offsets in the gather) leave the context on the block kernel, which
  //      scans the stations instead.
  c->assoc = nullptr;
  const size_t map1 = sizeof(int4) * (size_t)params->width * (size_t)params->height;
  c->het_packed = c->kp.het && params->num_ues <= 64 && !params->bs_per_env &&
                  map1 * (size_t)c->kp.nu_cls < ((size_t)1 << 32);
  c->block_small = params->num_ues <= 64 && params->bs_per_env &&
                   (params->width > 1024 || params->height > 1024);
  if (!params->bs_per_env && params->num_ues <= 64 && (!c->kp.het || c->het_packed)) {
    const size_t bytes = map1 * (size_t)(c->het_packed ? c->kp.nu_cls : 1);
    if (bytes >= ((size_t)1 << 32)) return MEV_EINVAL;  // (32-bit byte offsets in the gather)
    if (hipMalloc(&c->assoc, bytes) != hipSuccess) {
      return MEV_ENOMEM;
    }
    MEV_HIP(hipMemset(c->assoc, 0xff, bytes));  // srv -1 everywhere until a layout is set
  }
  // ---- culling records of the block kernel kept in HBM (mev_update_layouts /
  //      mev_update_stations; one set per env, or one for a shared layout), <= 2 GiB
  c->crec_g = nullptr;
  c->crec_ok = nullptr;
  if (c->kp.U > 64 && c->kp.cull_nc > 0 && !c->kp.het) {
    const size_t n = params->bs_per_env ? (size_t)params->num_envs : 1;
    const size_t bytes = n * (size_t)pers_cull(c->kp.cull_log, c->kp.W, c->kp.H).nc * 16;
    if (bytes <= ((size_t)2 << 30)) {
      if (hipMalloc(&c->crec_g, bytes) != hipSuccess || hipMalloc(&c->crec_ok, n) != hipSuccess)
        return MEV_ENOMEM;
      MEV_HIP(hipMemset(c->crec_ok, 0, n));  // none valid until built
    }
  }
  if (!c->kp.het) {  // LDS tables: shared layouts (modes 1-3), per-env layouts (mode 4)
    rc = build_lds_tables(c);
    if (rc) {
      return rc;
    }
  }
  if (c->het_packed) {
    rc = build_het_lds(c);
    if (rc) return rc;
  }
  if ((c->blob && c->kp.lds_mode == 3) || c->het_lds) {  // |D| (mode 3) / the rate count (mode 6)
                                                       // of each layout, read back without a sync
    MEV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->dcount_pin), sizeof(int), hipHostMallocDefault));
    MEV_HIP(hipEventCreateWithFlags(&c->ev_dcount, hipEventDisableTiming));
  }

  // ---- utility table over rounded rates ----
  c->util = nullptr;
  if (!c->kp.util_direct) {
    const int kmax = c->kp.util_kmax;
    int* d_bad = nullptr;
    if (hipMalloc(&c->util, sizeof(double) * (size_t)(kmax + 1)) != hipSuccess ||
        hipMalloc(&d_bad, sizeof(int)) != hipSuccess) {
      if (d_bad) (void)hipFree(d_bad);
      return MEV_ENOMEM;
    }
    struct DevFree {  // d_bad is released on every path out of this block
      int* q;
      ~DevFree() { (void)hipFree(q); }
    } bad_guard{d_bad};
    MEV_HIP(hipMemset(d_bad, 0, sizeof(int)));
    hipLaunchKernelGGL(k_util_table, dim3((kmax + 256) / 256), dim3(256), 0, 0, c->kp, kmax,
                       c->util, d_bad);
    MEV_HIP(hipGetLastError());
    int bad = 0;
    MEV_HIP(hipMemcpy(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost));
    if (bad) {  // not saturated at kmax: fall back to in-kernel evaluation
      (void)hipFree(c->util);
      c->util = nullptr;
      c->kp.util_direct = 1;
    }
  }
  // the reward guard's constants (RewardC) in the r100 tables' spare slots of the LDS blobs
  if (c->util) {
    struct {
      const double* tab;
      double sat, kmax;
      float u_err;
      int thr25;
    } rc{c->util, c->kp.util_sat, (double)c->kp.util_kmax, c->kp.u_err, c->kp.r_thr25};
    static_assert(sizeof(rc) == 32, "RewardC: four 8-byte slots");
    if (c->blob && c->kp.lds_mode >= 1)
      MEV_HIP(hipMemcpy(reinterpret_cast<char*>(c->blob) + c->kp.lds_r100_off + 8 * kRewardCSlot, &rc,
                        sizeof(rc), hipMemcpyHostToDevice));
    if (c->het_blob)
      MEV_HIP(hipMemcpy(c->het_blob + c->het_r100_off + 8 * kRewardCSlot, &rc, sizeof(rc),
                        hipMemcpyHostToDevice));
  }
  // ---- launch shape of mev_step: one kernel per step (auto), or on request two halves on
  //      two streams (measured 3-5 % faster at 65536 large envs, but the overlapping
  //      dispatches cannot be timed one by one)
  c->parts = 1;
  if (c->kp.U <= 64 && !c->block_small && params->stream_split == 2) c->parts = 2;
  c->fuse_steps = params->fuse_steps >= 0;
  if (c->parts == 2) {
    MEV_HIP(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    MEV_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    MEV_HIP(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
  }
  MEV_HIP(hipDeviceSynchronize());
  return MEV_OK;
}

int mev_create(const mev_params* params, mev_ctx** out) {
  if (!out) return MEV_EINVAL;
  *out = nullptr;
  const int rc0 = validate(params);
  if (rc0) return rc0;
  mev_ctx* c = new (std::nothrow) mev_ctx();
  if (!c) return MEV_ENOMEM;
  const int rc = create_ctx(c, params);
  if (rc) {
    mev_destroy(c);
    return rc;
  }
  *out = c;
  return MEV_OK;
}

void mev_destroy(mev_ctx* c) {
  if (!c) return;
  (void)hipFree(c->rate_full);
  (void)hipFree(c->jump);
  if (c->util) (void)hipFree(c->util);
  if (c->assoc) (void)hipFree(c->assoc);
  if (c->crec_g) (void)hipFree(c->crec_g);
  if (c->crec_ok) (void)hipFree(c->crec_ok);
  if (c->blob) (void)hipFree(c->blob);
  if (c->rankw) (void)hipFree(c->rankw);
  if (c->dwords) (void)hipFree(c->dwords);
  if (c->dflag) (void)hipFree(c->dflag);
  if (c->tab_xy) (void)hipFree(c->tab_xy);
  if (c->tab_st) (void)hipFree(c->tab_st);
  if (c->drawn) (void)hipFree(c->drawn);
  for (void* h : {(void*)c->h_bcl, (void*)c->h_ucl, (void*)c->h_pair, (void*)c->h_mv,
                  (void*)c->h_perm, (void*)c->h_seg, (void*)c->het_cell, (void*)c->het_flag,
                  (void*)c->het_words, (void*)c->het_info, (void*)c->het_blob})
    if (h) (void)hipFree(h);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->ev_dcount) (void)hipEventDestroy(c->ev_dcount);
  if (c->dcount_pin) (void)hipHostFree(c->dcount_pin);
  delete c;
}

int mev_d2max(const mev_ctx* c) { return c ? c->d2max : MEV_EINVAL; }

int mev_launch_parts(const mev_ctx* c) { return c ? c->parts : MEV_EINVAL; }

int mev_step_shape(const mev_ctx* c) {
  if (!c) return MEV_EINVAL;
  return packed_shape(c) ? 1 : 2;
}

int mev_lds_tables_bytes(const mev_ctx* c) { return c ? c->kp.lds_assoc : MEV_EINVAL; }
int mev_state_bytes_per_ue(const mev_ctx* c) { return c ? (c->kp.st8 ? 4 : 8) : MEV_EINVAL; }

const double* mev_rate_table(const mev_ctx* c) { return c ? c->rate_full : nullptr; }

int mev_share_tie_free(const mev_ctx* c) { return c ? c->tie_free : MEV_EINVAL; }

int mev_last_launch_kind(const mev_ctx* c) { return c ? c->last_kind : MEV_EINVAL; }

int mev_rollout_instance(const mev_ctx* c) {
  if (!c) return MEV_EINVAL;
  const bool lean_ok = !c->kp.util_direct && !c->kp.util_exact;
  return (lean_ok && ((c->kp.lds_assoc > 0 && ((c->kp.lds_mode == 3 && !c->p.bs_per_env) ||
                                                (c->kp.lds_mode == 4 && c->p.bs_per_env))) ||
                      (c->kp.U > 64 && c->p.bs_per_env && !c->kp.het)))
             ? match_scn(c) : 0;
}

int mev_share_cents(const mev_ctx* c, int32_t nmax, int32_t path, double* dst, void* stream) {
  if (!c || !dst || nmax < 1 || nmax > kMaxU || path < 0 || path > 1) return MEV_EINVAL;
  if (path == 1 && nmax > 64) return MEV_EINVAL;
  const int d2n = c->d2max + 1;
  if (d2n <= 0) return MEV_OK;
  const int64_t total = (int64_t)d2n * nmax;
  hipLaunchKernelGGL(k_share_cents, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, c->rate_full, d2n, nmax, (int)path, dst);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

int mev_copy_rate_table(const mev_ctx* c, double* dst, int64_t n) {
  if (!c || !dst || n < 0 || n > (int64_t)c->d2max + 1) return MEV_EINVAL;
  MEV_HIP(hipMemcpy(dst, c->rate_full, sizeof(double) * (size_t)n, hipMemcpyDefault));
  return MEV_OK;
}

static int check_bufs(const mev_ctx* c, const mev_state* st, const mev_outputs* out) {
  if (!c || !st || !out) return MEV_EINVAL;
  if (!st->ue_state || !st->pcg || !st->t || !st->bs_xy) return MEV_EINVAL;
  if (!out->obs || !out->serving || !out->reward || !out->done) return MEV_EINVAL;
  return MEV_OK;
}

static void to_kernel(const mev_state* st, const mev_outputs* out, KState& ks, KOut& ko) {
  ks.ue_state = reinterpret_cast<int2*>(st->ue_state);
  ks.pcg = st->pcg;
  ks.t = st->t;
  ks.bs_xy = reinterpret_cast<const int2*>(st->bs_xy);
  ks.bs_count = st->bs_count;
  ko.obs = reinterpret_cast<float4*>(out->obs);
  ko.serving = out->serving;
  ko.reward = out->reward;
  ko.done = out->done;
  ko.rate64 = out->rate64;
  ko.util64 = out->util64;
  ko.metrics = reinterpret_cast<float4*>(out->metrics);
  ko.qoe_stats = reinterpret_cast<double4*>(out->qoe_stats);
}

typedef void (*StepKernel)(KParams, KState, KOut, KTables, int, int);

template <bool PER_ENV_BS, bool LEAN>
static StepKernel step_kernel_u(int U) {
  switch (U) {  // scenario sizes of the registry (small / medium / large)
    case 5: return k_step_packed<PER_ENV_BS, LEAN, 5>;
    case 15: return k_step_packed<PER_ENV_BS, LEAN, 15>;
    case 30: return k_step_packed<PER_ENV_BS, LEAN, 30>;
    default: return k_step_packed<PER_ENV_BS, LEAN, 0>;
  }
}

static StepKernel step_kernel_for(bool per_env, bool lean, int U) {
  if (per_env) return lean ? step_kernel_u<true, true>(U) : step_kernel_u<true, false>(U);
  return lean ? step_kernel_u<false, true>(U) : step_kernel_u<false, false>(U);
}


template <bool PER_ENV_BS, bool LEAN, int LDSM>
static StepsKernel steps_kernel_u(int U) {
  switch (U) {
    case 5: return k_steps_packed<PER_ENV_BS, LEAN, 5, LDSM>;
    case 15: return k_steps_packed<PER_ENV_BS, LEAN, 15, LDSM>;
    case 30: return k_steps_packed<PER_ENV_BS, LEAN, 30, LDSM>;
    default: return k_steps_packed<PER_ENV_BS, LEAN, 0, LDSM>;
  }
}

static StepsKernel steps_kernel_for(bool per_env, bool lean, int ldsm, int U) {
  if (per_env) return lean ? steps_kernel_u<true, true, 0>(U) : steps_kernel_u<true, false, 0>(U);
  if (ldsm == 3) return lean ? steps_kernel_u<false, true, 3>(U) : steps_kernel_u<false, false, 3>(U);
  if (ldsm == 2) return lean ? steps_kernel_u<false, true, 2>(U) : steps_kernel_u<false, false, 2>(U);
  if (ldsm == 1) return lean ? steps_kernel_u<false, true, 1>(U) : steps_kernel_u<false, false, 1>(U);
  return lean ? steps_kernel_u<false, true, 0>(U) : steps_kernel_u<false, false, 0>(U);
}

// Timing events of a launch (mev_rollout_timed): a single-kernel launch has its dispatch record
// them (hipExtLaunchKernelGGL: the kernel's own start and end, no separate marker packets and
// no system-scope fence of an event record); launches of several kernels record them around.
struct LaunchEv {
  hipEvent_t start, stop;
  bool on() const { return start != nullptr || stop != nullptr; }
};

template <class K, class... A>
static void launch_k(K kern, dim3 grid, dim3 block, size_t shmem, hipStream_t stream,
                     const LaunchEv& ev, A... args) {
  if (ev.on())
    hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)shmem, stream, ev.start, ev.stop, 0u, args...);
  else
    hipLaunchKernelGGL(kern, grid, block, shmem, stream, args...);
}

static int launch_packed_split(const mev_ctx* c, const KState& ks, const KOut& ko,
                               const KTables& tb, int nsteps, bool traj, hipStream_t stream,
                               StepKernel k, size_t shmem, int groups);

// |D| of the current shared layout (mode 3), INT_MAX when unknown: waits for the pinned copy
// mev_update_stations issued (normally long complete when the first rollout asks)
static int layout_dcount(const mev_ctx* c) {
  if (c->dcount_pending) {
    if (hipEventSynchronize(c->ev_dcount) != hipSuccess) return INT_MAX;
    c->dcount_h = *c->dcount_pin;
    c->dcount_pending = 0;
  }
  return c->dcount_h;
}

// Packed step kernels of `nsteps` steps. Two-half shape: the first half of the groups runs on
// the caller's stream, the second on c->aux (forked from and joined back into the caller's
// stream); the halves are independent envs, so the two streams overlap freely.
static int launch_packed_steps(const mev_ctx* c, const KState& ks, const KOut& ko,
                               const KTables& tb, int nsteps, bool traj, hipStream_t stream,
                               const LaunchEv& ev) {
  const KParams& kp = c->kp;
  const int groups = (kp.E + kp.envs_per_wave - 1) / kp.envs_per_wave;
  const bool lean = !ko.rate64 && !ko.util64 && !ko.metrics && !ko.qoe_stats && !kp.util_direct &&
                    !kp.util_exact;
  StepKernel k = step_kernel_for(c->p.bs_per_env != 0, lean, kp.U);
  // scenario constants; tie-free share with the blob's 100 / n table (k_step_packed TF)
  const bool tf1 = c->tie_free && c->blob != nullptr;
  if (lean && !c->p.bs_per_env && kp.U == 30 && match_scn(c) == 2)
    k = tf1 ? k_step_packed<false, true, 30, 2, true> : k_step_packed<false, true, 30, 2>;
  else if (lean && !c->p.bs_per_env && kp.U == 15 && match_scn(c) == 1)
    k = tf1 ? k_step_packed<false, true, 15, 1, true> : k_step_packed<false, true, 15, 1>;
  const size_t shmem =
      kp.hist_lds ? sizeof(int) * kWavesPerBlock * (size_t)kp.envs_per_wave * kp.B : 0;
  // n > 1 steps on one stream: one launch of the fused multi-step kernel
  if (nsteps > 1 && c->parts == 1 && c->fuse_steps) {
    // LDS association tables for trajectory launches (measured at 65,536 mobile-large envs:
    // 16.0 vs 19.3 us per step, where the L2 gather competes with the stream of trajectory
    // stores); a launch that overwrites its outputs keeps the L2 gather (11.9 vs 15.1 us: the
    // stores stay in L2 and the tables' LDS cost occupancy, 4 vs 5 waves per SIMD)
    const bool ldsa = kp.lds_assoc > 0 && !c->p.bs_per_env && traj;
    const int ldsm = ldsa ? kp.lds_mode : 0;
    // two env groups per wavefront when the batch fills every resident workgroup with them
    const int pairs = (groups + 1) / 2;
    // (k_steps_lds2 prefetches a pair's draw tables into at most 8 registers per lane)
    const bool pre_ok = 2 * kp.envs_per_wave * kp.tab_m <= 64 * lds2_pre_words<30, 0, 2>();
    if (c->p.bs_per_env && kp.lds_mode == 4 && lean && traj && c->lds2_wgs > 0 && pre_ok &&
        pairs >= c->lds2_wgs * kLds2Waves) {  // per-env layouts (k_steps_lds2<U, 0, true>)
      const bool c8 = kp.st8 != 0;  // (generic instances: the state form as a template flag)
      StepsKernel k2 = kp.U == 15 ? (c8 ? k_steps_lds2<15, 0, true, false, 2, true>
                                        : k_steps_lds2<15, 0, true>)
                                  : (match_scn(c) == 3 ? (c->tie_free ? k_steps_lds2<30, 3, true, true>
                                                                      : k_steps_lds2<30, 3, true>)
                                     : c8 ? k_steps_lds2<30, 0, true, false, 2, true>
                                          : k_steps_lds2<30, 0, true>);
      const int blocks = std::min((pairs + kLds2Waves - 1) / kLds2Waves, c->lds2_wgs);
      const int G = kp.envs_per_wave;
      const int srows = std::min(c->stage_rows2, nsteps);
      const size_t sh = (size_t)kp.lds_assoc +
                        kLds2Waves * lds2_per_wave(G, kp.B, kp.tab_m, 2, true) +
                        (size_t)srows * kLds2Waves * G * 2 * kStage2Bytes;
      launch_k(k2, dim3(blocks), dim3(64 * kLds2Waves), sh, stream, ev, kp, ks, ko, tb, groups,
               nsteps, 1, srows);
      MEV_HIP(hipGetLastError());
      c->last_kind = MEV_KIND_LDS2_PERENV;
      return MEV_OK;
    }
    // heterogeneous entities with a shared layout: k_steps_lds2 HET on the lds_mode 6 tables
    // (build_het_lds) when the layout's rates fit beside at least one wavefront
    if (c->het_lds && lean && traj && pre_ok && c->p.two_groups >= 0 && c->p.two_groups <= 2) {
      const int nrate = layout_dcount(c);
      if (nrate >= 0 && nrate <= c->het_rate_cap) {
        // mode 6 (the 4-bit station map: 92 KB of tables on the large layout): two groups per
        // wavefront unless two_groups = 2 -- at 65,536 mobile-large-mixed envs 2.93 vs 3.29 ms
        // per 200-step launch (the dropped mode 5, u16 cell entries of 136 KB: ~10 two-group
        // waves per workgroup, 2.93 with one group vs 4.05 ms with two; interleaved on one box)
        const int R = c->p.two_groups == 2 ? 1 : 2;
        const int G = kp.envs_per_wave;
        const int units = R == 2 ? pairs : groups;
        const size_t blob = ((size_t)c->het_rate_off + 8 * (size_t)nrate + 15) & ~(size_t)15;
        const int srows = std::max(1, std::min(c->stage_cap > 0 ? c->stage_cap : kLds2Window, nsteps));
        const bool dbl = 2 * nsteps > srows;
        const size_t row_w = (size_t)G * R * kStage2Bytes;  // a staged row, per wave
        const size_t per_w = lds2_per_wave(G, kp.B, kp.tab_m, R) + (size_t)(dbl ? 2 : 1) * srows * row_w;
        const int fit = blob + 4 + per_w <= (size_t)kLds2BytesPerWG
                            ? (int)(((size_t)kLds2BytesPerWG - blob - 4) / per_w) : 0;
        if (fit >= 1) {
          const bool c8 = kp.st8 != 0;
          StepsKernel k2 =
              kp.U == 15 ? (R == 2 ? (c8 ? k_steps_lds2<15, 0, false, false, 2, true, false, true>
                                         : k_steps_lds2<15, 0, false, false, 2, false, false, true>)
                                   : (c8 ? k_steps_lds2<15, 0, false, false, 1, true, false, true>
                                         : k_steps_lds2<15, 0, false, false, 1, false, false, true>))
                         : (R == 2 ? (c8 ? k_steps_lds2<30, 0, false, false, 2, true, false, true>
                                         : k_steps_lds2<30, 0, false, false, 2, false, false, true>)
                                   : (c8 ? k_steps_lds2<30, 0, false, false, 1, true, false, true>
                                         : k_steps_lds2<30, 0, false, false, 1, false, false, true>));
          const int nw2 = std::max(1, std::min({kLds2Waves, fit, (units + c->het_cus - 1) / c->het_cus}));
          const size_t sh = blob + nw2 * lds2_per_wave(G, kp.B, kp.tab_m, R) +
                            (((size_t)(dbl ? 2 : 1) * srows * nw2 * row_w + 3) & ~(size_t)3);
          const size_t key = (sh << 8) | ((size_t)nw2 << 2) | ((size_t)R << 1) | (c8 ? 1u : 0u);
          if (c->het_occ_key != key) {
            int n = 0;
            MEV_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &n, reinterpret_cast<const void*>(k2), 64 * nw2, sh));
            c->het_occ_key = key;
            c->het_occ_n = std::max(1, n);
          }
          const int blocks = std::min((units + nw2 - 1) / nw2, c->het_cus * c->het_occ_n);
          KParams kp5 = kp;
          kp5.lds_mode = 6;
          kp5.lds_assoc = (int)blob;
          kp5.lds_st_off = c->het_nib_st;
          kp5.lds_r16_off = c->het_st_off;     // (mode 6: the pairs' table)
          kp5.lds_rank_off = c->het_words_off;  // (mode 6)
          kp5.lds_rate_off = c->het_rate_off;
          kp5.lds_r100_off = c->het_r100_off;
          KTables tb5 = tb;
          tb5.lds_blob = reinterpret_cast<const int4*>(c->het_blob);
          tb5.dcount = nullptr;
          launch_k(k2, dim3(blocks), dim3(64 * nw2), sh, stream, ev, kp5, ks, ko, tb5, groups,
                   nsteps, 1, dbl ? -srows : srows);
          MEV_HIP(hipGetLastError());
          c->last_kind = MEV_KIND_LDS2_HET;
          return MEV_OK;
        }
      }
    }
    // two groups per wavefront once the pairs fill every resident workgroup, else the
    // one-group packed kernel below. mev_params.two_groups (A/B switches): -1 the packed kernel
    // always; 1 / 2 this kernel with two / one groups per wavefront at any batch, as many
    // waves per workgroup as fill the resident workgroups. Measured at 4,096 medium envs (1,024
    // groups: one wave per SIMD either way): packed 129 us per 200-step launch, one group per
    // wave here 136 us, two groups (two waves per CU) 230 us -- the step's dependency chain,
    // not its instruction count, bounds a wave that is alone on its SIMD.
    const int tg = c->p.two_groups;
    const bool full2 = pairs >= c->lds2_wgs * kLds2Waves;
    // the software-pipelined one-group kernel: batches that do not fill the resident workgroups
    // with pairs (or two_groups = 3), registered U = 15 / 30 scenarios whose layout has no cell
    // beyond the mode-3 table's ranks. Measured on one box (200-step launches): 4,096 medium
    // envs 116-118 vs 126 us with the one-group packed kernel; 8,192 large envs 192 vs 252 us.
    const bool pipe = (tg == 3 || tg == 4 || (tg == 0 && !full2)) && (kp.U == 15 || kp.U == 30) &&
                      match_scn(c) != 0 && layout_dcount(c) <= 4094;
    // U = 15 in 32-lane segments (two envs per wavefront, twice the wavefronts; two_groups = 4
    // only): at 4,096 medium envs two chains per SIMD instead of one, but each with the 32-lane
    // segments' LDS histogram instead of the packed DPP counts -- 126 vs 101 us per 200-step
    // launch (interleaved on one box), so the 16-lane form stays the automatic choice
    const bool seg32 = pipe && kp.U == 15 && tg == 4;
    if (ldsm == 3 && lean && c->lds2_wgs > 0 && pre_ok && (tg > 0 || (tg == 0 && full2) || pipe) &&
        ((tg != 3 && tg != 4) || pipe)) {
      const int R = tg == 1 ? 2 : (tg >= 2 || pipe) ? 1 : 2;
      const int G = seg32 ? 2 : kp.envs_per_wave;  // envs per group
      const int groups_l = seg32 ? (kp.E + 1) / 2 : groups;
      const int units = R == 2 ? pairs : groups_l;  // the waves' work units
      const int nw2 = std::max(1, std::min(kLds2Waves, (units + c->lds2_wgs - 1) / c->lds2_wgs));
      const int scn = match_scn(c);
      const bool tf = c->tie_free != 0;  // (scenario instances only)
      StepsKernel k2;
      const bool c8 = kp.st8 != 0;  // (generic instances: the state form as a template flag)
      if (seg32)
        k2 = tf ? k_steps_lds2<kSeg32 + 15, 1, false, true, 1, scn_st8(1), true>
                : k_steps_lds2<kSeg32 + 15, 1, false, false, 1, scn_st8(1), true>;
      else if (pipe)
        k2 = kp.U == 15 ? (tf ? k_steps_lds2<15, 1, false, true, 1, scn_st8(1), true>
                              : k_steps_lds2<15, 1, false, false, 1, scn_st8(1), true>)
                        : (tf ? k_steps_lds2<30, 2, false, true, 1, scn_st8(2), true>
                              : k_steps_lds2<30, 2, false, false, 1, scn_st8(2), true>);
      else if (R == 2 && tf && nsteps < 64 && (scn == 1 || scn == 2))  // (RT1: see lds2_step)
        k2 = scn == 1 ? k_steps_lds2<15, 1, false, true, 2, scn_st8(1), false, false, true>
                      : k_steps_lds2<30, 2, false, true, 2, scn_st8(2), false, false, true>;
      else if (R == 2)
        k2 = kp.U == 15 ? (scn == 1 ? (tf ? k_steps_lds2<15, 1, false, true> : k_steps_lds2<15, 1>)
                           : c8     ? k_steps_lds2<15, 0, false, false, 2, true>
                                    : k_steps_lds2<15, 0>)
                        : (scn == 2 ? (tf ? k_steps_lds2<30, 2, false, true> : k_steps_lds2<30, 2>)
                           : c8     ? k_steps_lds2<30, 0, false, false, 2, true>
                                    : k_steps_lds2<30, 0>);
      else
        k2 = kp.U == 15 ? (scn == 1 ? (tf ? k_steps_lds2<15, 1, false, true, 1>
                                          : k_steps_lds2<15, 1, false, false, 1>)
                           : c8     ? k_steps_lds2<15, 0, false, false, 1, true>
                                    : k_steps_lds2<15, 0, false, false, 1>)
                        : (scn == 2 ? (tf ? k_steps_lds2<30, 2, false, true, 1>
                                          : k_steps_lds2<30, 2, false, false, 1>)
                           : c8     ? k_steps_lds2<30, 0, false, false, 1, true>
                                    : k_steps_lds2<30, 0, false, false, 1>);
      const int blocks = std::min((units + nw2 - 1) / nw2, c->lds2_wgs);
      // staged rows: c->stage_rows2 (the count that fits beside 16 waves of two groups), or for
      // one group of 16-lane segments per wave as many as fit beside this launch's waves: 4,096
      // medium envs, 4 waves per workgroup, then flush once per 200-step launch instead of every
      // 17 rows (104.5 vs 108.5 us per launch). Not for 32-lane segments: larger windows made
      // those launches slower (8,192 large envs, pipelined: 270 vs 206 us; 65,536 with two
      // groups per wave and 126 rows: 1.72 vs 1.45 ms), all interleaved on one box.
      const size_t wave_b = (size_t)kp.lds_assoc + nw2 * lds2_per_wave(G, kp.B, kp.tab_m, R);
      const size_t row_b = (size_t)nw2 * G * R * kStage2Bytes;
      // Two groups per wave: a window of 3 rows. Each flush is a workgroup barrier, and one
      // every 3 steps keeps the workgroup's 16 waves -- adjacent envs -- in step, so their
      // trajectory stores reach the memory together: 168.8 vs 175 us per 20-step and 1.49 vs
      // 1.64 ms per 200-step launch at 65,536 large envs against the 47 rows that fit
      // (windows of 1 / 2 / 4 / 8 / 16 rows: 183 / 170.6 / 168.6 / 168 / 172.7 us and
      // 1.58 / 1.47 / 1.50 / 1.55 / 1.59 ms; interleaved on one box)
      // (mev_params.stage_rows > 0 overrides: A/B of window lengths)
      int fit = R == 2 && c->stage_cap <= 0 ? std::min(c->stage_rows2, kLds2Window) : c->stage_rows2;
      if (R == 1 && kp.U == 15) {
        fit = wave_b + row_b + 4 <= (size_t)kLds2BytesPerWG
                  ? (int)(((size_t)kLds2BytesPerWG - wave_b - 4) / row_b) : 1;
        if (c->stage_cap > 0) fit = std::min(fit, c->stage_cap);
      }
      const int srows = std::max(1, std::min(fit, nsteps));
      // two groups per wave: two windows of srows rows, one barrier per flush (k_steps_lds2's
      // stage_rows < 0)
      const bool dbl = R == 2 && 2 * nsteps > srows && 2 * srows <= c->stage_rows2;
      const size_t sh = wave_b + (((size_t)(dbl ? 2 : 1) * srows * row_b + 3) & ~(size_t)3);
      launch_k(k2, dim3(blocks), dim3(64 * nw2), sh, stream, ev, kp, ks, ko, tb, groups_l,
               nsteps, 1, dbl ? -srows : srows);
      MEV_HIP(hipGetLastError());
      c->last_kind = seg32 ? MEV_KIND_LDS2_PIPE32
                     : pipe ? MEV_KIND_LDS2_PIPE : R == 2 ? MEV_KIND_LDS2_TWO : MEV_KIND_LDS2_ONE;
      return MEV_OK;
    }
    StepsKernel kf = steps_kernel_for(c->p.bs_per_env != 0, lean, ldsm, kp.U);
    if (ldsm == 3 && lean) {  // a registered scenario's constants (scn_const)
      const int scn = match_scn(c);
      const bool tf = c->tie_free != 0;  // (share_tie_free)
      if (scn == 1) kf = tf ? k_steps_packed<false, true, 15, 3, 1, true> : k_steps_packed<false, true, 15, 3, 1>;
      if (scn == 2) kf = tf ? k_steps_packed<false, true, 30, 3, 2, true> : k_steps_packed<false, true, 30, 3, 2>;
    }
    int nw = lds_waves(ldsm);
    if (ldsa)  // few groups: fewer waves per workgroup, the workgroups on every CU
      nw = std::max(1, std::min(nw, (groups + c->lds_wgs - 1) / c->lds_wgs));
    int blocks = (groups + nw - 1) / nw;
    if (ldsa) blocks = std::min(blocks, c->lds_wgs);  // persistent: the resident workgroups
    size_t shmem_f = (ldsa ? (size_t)kp.lds_assoc : 0) + nw * lds_per_wave(kp);  // layout: k_steps_packed
    const bool stg = ldsm >= 2 && lean && stages(kp);  // k_steps_packed STG
    int srows = stg ? std::min(c->stage_rows, nsteps) : 1;
    if (stg && nw < lds_waves(ldsm))  // (more rows fit beside fewer waves)
      srows = std::min({nsteps, c->stage_cap > 0 ? c->stage_cap : nsteps,
                        (int)(((size_t)kLds2BytesPerWG - shmem_f - 4) /
                              ((size_t)nw * stage_bytes_per_row(kp)))});
    launch_k(kf, dim3(blocks), dim3(64 * nw), shmem_f + (stg ? stage_lds_bytes(kp, srows, nw) : 0),
             stream, ev, kp, ks, ko, tb, groups, nsteps, traj ? 1 : 0, srows);
    MEV_HIP(hipGetLastError());
    c->last_kind = MEV_KIND_PACKED_FUSED;
    return MEV_OK;
  }
  // (several kernels: the timing events around them)
  if (ev.start) MEV_HIP(hipEventRecord(ev.start, stream));
  const int rc = launch_packed_split(c, ks, ko, tb, nsteps, traj, stream, k, shmem, groups);
  c->last_kind = MEV_KIND_PACKED_STEP;
  if (ev.stop) MEV_HIP(hipEventRecord(ev.stop, stream));
  return rc;
}

// One-step kernels, nsteps launches, one stream or two env halves (mev_step's shapes)
static int launch_packed_split(const mev_ctx* c, const KState& ks, const KOut& ko,
                               const KTables& tb, int nsteps, bool traj, hipStream_t stream,
                               StepKernel k, size_t shmem, int groups) {
  const KParams& kp = c->kp;
  // split on a block boundary
  const int half = (groups / 2 + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;
  if (c->parts == 1 || half <= 0 || half >= groups) {
    const int blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    for (int i = 0; i < nsteps; ++i)
      k<<<dim3(blocks), dim3(kPackedBlock), shmem, stream>>>(
          kp, ks, traj ? out_row(ko, kp.E, kp.U, i) : ko, tb, 0, groups);
    MEV_HIP(hipGetLastError());
    return MEV_OK;
  }
  const int blocks0 = half / kWavesPerBlock;
  const int blocks1 = (groups - half + kWavesPerBlock - 1) / kWavesPerBlock;
  MEV_HIP(hipEventRecord(c->ev_fork, stream));
  MEV_HIP(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
  for (int i = 0; i < nsteps; ++i) {
    const KOut oi = traj ? out_row(ko, kp.E, kp.U, i) : ko;
    k<<<dim3(blocks0), dim3(kPackedBlock), shmem, stream>>>(kp, ks, oi, tb, 0, half);
    k<<<dim3(blocks1), dim3(kPackedBlock), shmem, c->aux>>>(kp, ks, oi, tb, half, groups);
  }
  MEV_HIP(hipGetLastError());
  MEV_HIP(hipEventRecord(c->ev_join, c->aux));
  MEV_HIP(hipStreamWaitEvent(stream, c->ev_join, 0));
  return MEV_OK;
}

// Block-shape steps (U > 64): ONE launch of k_steps_block for the n steps (fuse_steps), or one
// per step; one workgroup per env.
static int launch_block_steps(const mev_ctx* c, const KState& ks, const KOut& ko,
                              const KTables& tb, int nsteps, bool traj, hipStream_t stream,
                              const LaunchEv& ev) {
  const KParams& kp = c->kp;
  if (nsteps <= 0) return MEV_OK;
  const bool lean = !ko.rate64 && !ko.util64 && !ko.metrics && !ko.qoe_stats && !kp.util_direct &&
                    !kp.util_exact;
  const bool per_env = c->p.bs_per_env != 0;
  void (*kf)(KParams, KState, KOut, KTables, int, int) =
      kp.het ? (per_env ? (lean ? k_steps_block<true, true, true> : k_steps_block<true, false, true>)
                        : (lean ? k_steps_block<false, true, true> : k_steps_block<false, false, true>))
             : (per_env ? (lean ? k_steps_block<true, true, false> : k_steps_block<true, false, false>)
                        : (lean ? k_steps_block<false, true, false> : k_steps_block<false, false, false>));
  // two UEs per lane (U > 512, homogeneous) for one-step launches: 1,024 envs of 1,024 UEs then
  // take 8,192 waves, one round of the chip's resident waves instead of two, and the per-wave
  // prologue / epilogue is shared by two UEs (custom 128 x 1024 at 1,024 envs: 18.7 -> 17.3 us
  // per step() launch); rollouts keep one (at full occupancy both shapes issue the same step
  // work, and the two-UE records need cells twice as wide: 1.41 vs 1.67 ms per 200 steps)
  const bool one_step = nsteps == 1 || !c->fuse_steps;
  const int upl = kp.het ? 1 : c->upl > 0 ? c->upl : (kp.U > 512 && one_step ? 2 : 1);
  if (upl == 2)
    kf = per_env ? (lean ? k_steps_block<true, true, false, 0, false, 2> : k_steps_block<true, false, false, 0, false, 2>)
                 : (lean ? k_steps_block<false, true, false, 0, false, 2> : k_steps_block<false, false, false, 0, false, 2>);
  const CullP cp{kp.cull_log, kp.cull_nx, kp.cull_nc};
  const size_t shm = block_lds_bytes(kp.B, kp.tab_m) + block_rec_bytes(cp, kp.W, kp.H, nsteps, upl);
  if (lean && per_env && !kp.het && match_scn(c) == 4)  // mobile-custom-128x1024's constants
    kf = upl == 2 ? (c->tie_free ? k_steps_block<true, true, false, 4, true, 2> : k_steps_block<true, true, false, 4, false, 2>)
                  : (c->tie_free ? k_steps_block<true, true, false, 4, true> : k_steps_block<true, true, false, 4>);
  const int ul = (kp.U + upl - 1) / upl;  // lanes per env
  const dim3 block((unsigned)((ul + 63) / 64 * 64));
  if (c->fuse_steps || nsteps == 1) {
    launch_k(kf, dim3(kp.E), block, shm, stream, ev, kp, ks, ko, tb, nsteps, traj ? 1 : 0);
  } else {
    if (ev.start) MEV_HIP(hipEventRecord(ev.start, stream));
    for (int i = 0; i < nsteps; ++i)
      kf<<<dim3(kp.E), block, shm, stream>>>(kp, ks, traj ? out_row(ko, kp.E, kp.U, i) : ko, tb,
                                             1, 0);
    if (ev.stop) MEV_HIP(hipEventRecord(ev.stop, stream));
  }
  MEV_HIP(hipGetLastError());
  c->last_kind = MEV_KIND_BLOCK;
  return MEV_OK;
}

template <bool RESET>
static int launch(const mev_ctx* c, const mev_state* st, const mev_outputs* out,
                  const uint8_t* mask, hipStream_t stream) {
  KState ks;
  KOut ko;
  to_kernel(st, out, ks, ko);
  const KTables tb = tables_of(c);
  const KParams& kp = c->kp;
  if (packed_shape(c)) {
    const int groups = (kp.E + kp.envs_per_wave - 1) / kp.envs_per_wave;
    if (RESET) {
      const dim3 grid((unsigned)((groups + kWavesPerBlock - 1) / kWavesPerBlock));
      hipLaunchKernelGGL(k_reset_packed, grid, dim3(kPackedBlock), 0, stream, kp, ks, ko, tb,
                         mask);
    } else {
      return launch_packed_steps(c, ks, ko, tb, 1, false, stream, LaunchEv{nullptr, nullptr});
    }
  } else if (RESET) {
    const dim3 block((unsigned)((kp.U + 63) / 64 * 64));
    hipLaunchKernelGGL(k_reset_block, dim3(kp.E), block, 0, stream, kp, ks, ko, tb, mask);
  } else {
    return launch_block_steps(c, ks, ko, tb, 1, false, stream, LaunchEv{nullptr, nullptr});
  }
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

int mev_update_stations(const mev_ctx* c, const int32_t* bs_xy, void* stream) {
  if (!c || !bs_xy) return MEV_EINVAL;
  if (c->p.bs_per_env || (c->kp.het && !c->het_packed))
    return MEV_OK;  // the block kernel reads bs_xy itself
  if (c->crec_g) {  // (shared layout, block shape) the culling records of the layout
    KState ks{};
    ks.bs_xy = reinterpret_cast<const int2*>(bs_xy);
    hipLaunchKernelGGL(k_cull_build, dim3(1), dim3(256), 0, (hipStream_t)stream, c->kp, ks,
                       nullptr, 0, c->crec_g, c->crec_ok);
    MEV_HIP(hipGetLastError());
  }
  if (!c->assoc) return MEV_OK;  // (block shape: no association map, no LDS tables)
  const int cells = c->p.width * c->p.height;
  if (c->het_packed) {  // one map per UE class
    const int n = cells * c->kp.nu_cls;
    hipLaunchKernelGGL(k_assoc_map_het, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const int2*>(bs_xy), c->p.num_bs, c->p.width,
                       c->p.height, c->h_bcl, c->h_pair, c->kp.nu_cls, c->rate_full, c->assoc);
    MEV_HIP(hipGetLastError());
    if (c->het_lds) {  // the two-group rollout's tables (lds_mode 6), see build_het_lds
      const int NB = c->kp.nb_cls, NU = c->kp.nu_cls, reach = c->het_reach, nw = c->het_nwords;
      const int nd = reach + 1;
      hipStream_t s = (hipStream_t)stream;
      MEV_HIP(hipMemsetAsync(c->het_flag, 0, (size_t)NB * nd, s));
      hipLaunchKernelGGL(k_het_cells, dim3((cells + 255) / 256), dim3(256), 0, s,
                         reinterpret_cast<const int2*>(bs_xy), c->p.num_bs, c->p.width,
                         c->p.height, reach, c->h_bcl, c->het_cell, c->het_flag);
      for (int cb = 0; cb < NB; ++cb)
        hipLaunchKernelGGL(k_d2_prefix, dim3(1), dim3(1024), 0, s, c->het_flag + (size_t)cb * nd,
                           nd, c->het_words + (size_t)cb * (nw + 1), nw);
      hipLaunchKernelGGL(k_het_info, dim3(1), dim3(64), 0, s, c->het_words, nw, NB, NU,
                         c->p.num_bs, c->h_bcl, c->h_pair, reach,
                         reinterpret_cast<int2*>(c->het_blob + c->het_st_off), c->het_info,
                         reinterpret_cast<const int2*>(bs_xy),
                         reinterpret_cast<uint32_t*>(c->het_blob + c->het_nib_st));
      const int n = std::max(cells, NB * nd);
      hipLaunchKernelGGL(k_het_map, dim3((n + 255) / 256), dim3(256), 0, s, c->het_cell, cells,
                         c->het_words, nw, reach, NB, NU, c->h_bcl, c->h_pair, c->rate_full,
                         c->het_info, c->het_blob, c->het_rate_off, c->het_rate_cap);
      MEV_HIP(hipGetLastError());
      // the classes' rank indices into the blob
      MEV_HIP(hipMemcpyAsync(c->het_blob + c->het_words_off, c->het_words,
                               sizeof(uint2) * (size_t)NB * (nw + 1), hipMemcpyDeviceToDevice, s));
      MEV_HIP(hipMemcpyAsync(c->dcount_pin, c->het_info, sizeof(int), hipMemcpyDeviceToHost, s));
      MEV_HIP(hipEventRecord(c->ev_dcount, s));
      c->dcount_pending = 1;
    }
    return MEV_OK;
  }
  hipLaunchKernelGGL(k_assoc_map, dim3((cells + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const int2*>(bs_xy), c->p.num_bs, c->p.width,
                     c->p.height, c->d2max, c->rate_full, c->assoc);
  MEV_HIP(hipGetLastError());
  if (c->blob && c->kp.lds_mode == 3) {
    MEV_HIP(hipMemsetAsync(c->dflag, 0, (size_t)c->d2max + 1, (hipStream_t)stream));
    hipLaunchKernelGGL(k_d2_mark, dim3((cells + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       c->assoc, cells, c->dflag);
    hipLaunchKernelGGL(k_d2_prefix, dim3(1), dim3(1024), 0, (hipStream_t)stream, c->dflag,
                       c->d2max + 1, c->dwords, c->nwords);
    const int n = std::max(cells, c->d2max + 1);
    hipLaunchKernelGGL(k_lds_map3, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       c->assoc, cells, c->dwords, c->d2max, c->rate_full,
                       reinterpret_cast<uint8_t*>(c->blob), c->kp.lds_rate_off);
    MEV_HIP(hipGetLastError());
    // |D| for the host's kernel choice (the pipelined rollout takes layouts without cells
    // beyond the table's ranks): copied to pinned memory in stream order; the first launch
    // whose choice depends on it waits for that copy's event (layout_dcount), nothing else does
    MEV_HIP(hipMemcpyAsync(c->dcount_pin, c->dwords + c->nwords, sizeof(int),
                           hipMemcpyDeviceToHost, (hipStream_t)stream));
    MEV_HIP(hipEventRecord(c->ev_dcount, (hipStream_t)stream));
    c->dcount_pending = 1;
  } else if (c->blob) {
    const int bytes = (cells + 1) / 2;
    hipLaunchKernelGGL(k_lds_map, dim3((bytes + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const int2*>(bs_xy), c->p.num_bs, cells, c->assoc,
                       reinterpret_cast<uint8_t*>(c->blob), c->kp.lds_mode, c->kp.lds_st_off,
                       c->kp.lds_r16_off, c->rankw);
    MEV_HIP(hipGetLastError());
  }
  return MEV_OK;
}

int mev_update_layouts(const mev_ctx* c, const mev_state* st, const uint8_t* env_mask,
                       void* stream) {
  if (!c || !st || !st->bs_xy) return MEV_EINVAL;
  if (!c->p.bs_per_env || !c->crec_g) return MEV_OK;  // nothing kept per env
  KState ks;
  KOut ko{};
  mev_outputs none{};
  to_kernel(st, &none, ks, ko);
  hipLaunchKernelGGL(k_cull_build, dim3((unsigned)c->kp.E), dim3(256), 0, (hipStream_t)stream,
                     c->kp, ks, env_mask, 1, c->crec_g, c->crec_ok);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

int mev_prepare_draws(const mev_ctx* c, const mev_state* st, const uint8_t* env_mask,
                      void* stream) {
  if (!c || !st || !st->pcg) return MEV_EINVAL;
  if (!c->kp.tab_m) return MEV_OK;
  const int64_t n = (int64_t)c->kp.E * c->kp.tab_m;
  hipLaunchKernelGGL(k_draw_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, c->kp, st->pcg, env_mask, c->jump, c->tab_xy,
                     c->tab_st);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

#ifdef MEV_TIMING
extern "C" int mev_debug_timestamps(void* dev_buf) {
  MEV_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_mev_ts), &dev_buf, sizeof(void*)));
  return MEV_OK;
}
#endif

int mev_sync_stream_state(const mev_ctx* c, const mev_state* st, void* stream) {
  if (!c || !st || !st->pcg) return MEV_EINVAL;
  if (!c->kp.tab_m) return MEV_OK;  // without the table the rows are always current
  hipLaunchKernelGGL(k_sync_stream_state, dim3((unsigned)((c->kp.E + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, c->kp.E, c->kp.tab_m, c->drawn, c->tab_st, st->pcg);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

int mev_restore_stream_state(const mev_ctx* c, const mev_state* st, const uint8_t* env_mask,
                             void* stream) {
  if (!c || !st || !st->pcg) return MEV_EINVAL;
  if (!c->kp.tab_m) return MEV_OK;  // without the table every draw reads the row already
  // the episode draw tables of the restored streams (state0), for the envs' next episodes
  const int rc = mev_prepare_draws(c, st, env_mask, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_restore_stream_state, dim3((unsigned)((c->kp.E + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, c->kp.E, c->kp.tab_m, env_mask, c->drawn);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

int mev_reset(const mev_ctx* c, const mev_state* st, const mev_outputs* out,
              const uint8_t* env_mask, void* stream) {
  int rc = check_bufs(c, st, out);
  if (rc) return rc;
  rc = mev_update_stations(c, st->bs_xy, stream);
  if (rc) return rc;
  rc = mev_update_layouts(c, st, env_mask, stream);
  if (rc) return rc;
  rc = mev_prepare_draws(c, st, env_mask, stream);
  if (rc) return rc;
  return launch<true>(c, st, out, env_mask, (hipStream_t)stream);
}

static int run_steps(const mev_ctx* c, const mev_state* st, const mev_outputs* out,
                     int32_t nsteps, bool traj, void* stream, LaunchEv ev = LaunchEv{nullptr, nullptr}) {
  int rc = check_bufs(c, st, out);
  if (rc) return rc;
  if (nsteps < 0) return MEV_EINVAL;
  KState ks;
  KOut ko;
  to_kernel(st, out, ks, ko);
  const KTables tb = tables_of(c);
  if (nsteps == 0 && ev.on()) {  // nothing to launch: the events still bracket the (empty) work
    if (ev.start) MEV_HIP(hipEventRecord(ev.start, (hipStream_t)stream));
    if (ev.stop) MEV_HIP(hipEventRecord(ev.stop, (hipStream_t)stream));
    return MEV_OK;
  }
  if (packed_shape(c))
    return launch_packed_steps(c, ks, ko, tb, nsteps, traj, (hipStream_t)stream, ev);
  return launch_block_steps(c, ks, ko, tb, nsteps, traj, (hipStream_t)stream, ev);
}

int mev_step(const mev_ctx* c, const mev_state* st, const mev_outputs* out, int32_t nsteps,
             void* stream) {
  return run_steps(c, st, out, nsteps, false, stream);
}

int mev_rollout(const mev_ctx* c, const mev_state* st, const mev_outputs* traj,
                int32_t nsteps, void* stream) {
  return run_steps(c, st, traj, nsteps, true, stream);
}

int mev_rollout_timed(const mev_ctx* c, const mev_state* st, const mev_outputs* traj,
                      int32_t nsteps, void* stream, void* start_event, void* stop_event) {
  return run_steps(c, st, traj, nsteps, true, stream,
                   LaunchEv{(hipEvent_t)start_event, (hipEvent_t)stop_event});
}

// --------------------------------------------------------------------------------------
// numpy-compatible seeding (host): SeedSequence(seed).generate_state(4, uint64) ->
// PCG64 srandom (numpy/random/bit_generator.pyx, numpy/random/src/pcg64/pcg64.c).
// --------------------------------------------------------------------------------------
__host__ __device__ static uint32_t ss_hashmix(uint32_t value, uint32_t* hash_const) {
  value ^= *hash_const;
  *hash_const *= 0x931e8875u;  // MULT_A
  value *= *hash_const;
  value ^= value >> 16;
  return value;
}

__host__ __device__ static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;  // MIX_MULT_L, MIX_MULT_R
  r ^= r >> 16;
  return r;
}

__host__ __device__ static void seed_sequence_state(uint64_t seed, uint64_t out_words[4]) {
  uint32_t entropy[2];
  int n_ent = 0;
  uint64_t v = seed;
  do {  // _coerce_to_uint32_array: little-endian 32-bit words, at least one
    entropy[n_ent++] = (uint32_t)(v & 0xffffffffu);
    v >>= 32;
  } while (v && n_ent < 2);
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;  // INIT_A
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < n_ent ? entropy[i] : 0u, &hc);
  for (int src = 0; src < 4; ++src)
    for (int dst = 0; dst < 4; ++dst)
      if (src != dst) pool[dst] = ss_mix(pool[dst], ss_hashmix(pool[src], &hc));
  for (int src = 4; src < n_ent; ++src)
    for (int dst = 0; dst < 4; ++dst) pool[dst] = ss_mix(pool[dst], ss_hashmix(entropy[src], &hc));
  uint32_t st32[8];
  uint32_t hb = 0x8b51f9ddu;  // INIT_B
  for (int i = 0; i < 8; ++i) {
    uint32_t d = pool[i % 4];
    d ^= hb;
    hb *= 0x58f38dedu;  // MULT_B
    d *= hb;
    d ^= d >> 16;
    st32[i] = d;
  }
  for (int i = 0; i < 4; ++i) out_words[i] = (uint64_t)st32[2 * i] | ((uint64_t)st32[2 * i + 1] << 32);
}

// One pcg row {state, inc, state0} of PCG64(SeedSequence(seed)): pcg64_set_seed with
// initstate = (w0 << 64) | w1, initseq = (w2 << 64) | w3.
__host__ __device__ static void seed_row(uint64_t seed, uint64_t* r) {
  const u128 mult = ((u128)PCG_MULT_HI << 64) | PCG_MULT_LO;
  uint64_t w[4];
  seed_sequence_state(seed, w);
  const u128 initstate = ((u128)w[0] << 64) | w[1];
  const u128 initseq = ((u128)w[2] << 64) | w[3];
  const u128 inc = (initseq << 1) | 1;
  u128 s = 0;
  s = s * mult + inc;
  s += initstate;
  s = s * mult + inc;
  r[0] = (uint64_t)s;
  r[1] = (uint64_t)(s >> 64);
  r[2] = (uint64_t)inc;
  r[3] = (uint64_t)(inc >> 64);
  r[4] = r[0];
  r[5] = r[1];
}

int mev_seed_pcg64(const uint64_t* seeds, int64_t n, uint64_t* rows) {
  if ((!seeds || !rows) && n > 0) return MEV_EINVAL;
  for (int64_t i = 0; i < n; ++i) {
    if (seeds[i] >> 63) return MEV_EINVAL;
    seed_row(seeds[i], rows + 6 * i);
  }
  return MEV_OK;
}

// Device SeedSequence -> PCG64 rows, one thread per env (batched init of large batches).
__global__ void k_seed_pcg64(const uint64_t* __restrict__ seeds, int64_t n, uint64_t* rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t sd = seeds[i];
  uint64_t* r = rows + 6 * i;
  if (sd >> 63) {  // not a valid numpy seed here: an all-zero row (inc = 0 marks it)
    for (int k = 0; k < 6; ++k) r[k] = 0;
    return;
  }
  seed_row(sd, r);
}

int mev_seed_pcg64_device(const uint64_t* seeds, int64_t n, uint64_t* rows, void* stream) {
  if (n < 0 || ((!seeds || !rows) && n > 0)) return MEV_EINVAL;
  if (n == 0) return MEV_OK;
  hipLaunchKernelGGL(k_seed_pcg64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, seeds, n, rows);
  MEV_HIP(hipGetLastError());
  return MEV_OK;
}

