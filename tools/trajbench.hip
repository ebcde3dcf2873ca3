// Dev tool: write pattern of a fused rollout launch (no env math), to find what couples the
// per-step output stores to the step's compute.
// Every wave owns G = 2 envs x 30 UEs (lane = UE, pitch 32) and runs `n` steps; each step does
// `work` x 4 independent FMAs per lane (stand-in for the step's compute) and writes obs
// (16 B / UE), serving (4 B / UE), reward (4 B / env), done (1 B / env) to step-major rows
// [n][E][U] (layout 0) or one overwritten row (layout 2).
//   mode 0: no loads in the loop
//   mode 1: a 16 B gather per lane per step from an L2-resident 640 KB table, consumed before
//           the step's stores (the step kernel's association-map read)
//   mode 2: mode 1 with the stores of step i issued after the gather of step i + 1
//   mode 3: mode 1 with a store wave per workgroup: 4 compute waves hand their outputs to a
//           5th wave through an LDS ring of RING slots; only the store wave issues global
//           stores, so the compute waves' gathers never wait behind stores
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int U = 30, P = 32, G = 2, RING = 4;

__device__ __forceinline__ float spin(float x, int work) {
  float a = x, b = x + 1.f, c = x + 2.f, d = x + 3.f;
  for (int k = 0; k < work; ++k) {
    a = __builtin_fmaf(a, 1.0000001f, 0.5f);
    b = __builtin_fmaf(b, 1.0000001f, 0.5f);
    c = __builtin_fmaf(c, 1.0000001f, 0.5f);
    d = __builtin_fmaf(d, 1.0000001f, 0.5f);
  }
  return a + b + c + d;
}

__global__ __launch_bounds__(256) void k_traj(float4* obs, int* srv, float* rew, uint8_t* done,
                                             const int4* tab, int E, int n, int layout, int mode,
                                             int work) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int seg = lane / P, u = lane - seg * P;
  const int e = wave * G + seg;
  if (e >= E) return;
  float x = (float)lane;
  uint32_t h = (uint32_t)(e * 31 + u) * 2654435761u;
  float4 po = make_float4(0, 0, 0, 0);
  int ps = 0;
  float pr = 0.f;
  size_t pui = 0, pei = 0;
  bool have = false;
  for (int i = 0; i < n; ++i) {
    int4 r = make_int4(0, 0, 0, 0);
    if (mode >= 1) {
      h = h * 1664525u + 1013904223u;
      r = tab[(h >> 8) % 40000u];
    }
    const size_t ui = layout == 0 ? ((size_t)i * E + e) * U + u : (size_t)e * U + u;
    const size_t ei = layout == 0 ? (size_t)i * E + e : (size_t)e;
    if (mode == 2 && have) {  // previous step's stores after this step's gather
      if (u < U) {
        obs[pui] = po;
        srv[pui] = ps;
      }
      if (u == P - 1) {
        rew[pei] = pr;
        done[pei] = (uint8_t)i;
      }
    }
    x = spin(x + (float)r.x, work);
    const float4 o = make_float4(x, (float)i, (float)u, (float)r.y);
    if (mode == 2) {
      po = o;
      ps = (int)x;
      pr = x;
      pui = ui;
      pei = ei;
      have = true;
    } else {
      if (u < U) {
        obs[ui] = o;
        srv[ui] = (int)x;
      }
      if (u == P - 1) {
        rew[ei] = x;
        done[ei] = (uint8_t)i;
      }
    }
  }
  if (mode == 2 && have) {
    if (u < U) {
      obs[pui] = po;
      srv[pui] = ps;
    }
    if (u == P - 1) {
      rew[pei] = pr;
      done[pei] = (uint8_t)n;
    }
  }
}

// mode 3: 5 waves per workgroup (waves 0-3 compute, wave 4 stores)
struct Slot {
  float4 obs[4][64];
  int srv[4][64];
};

__global__ __launch_bounds__(320) void k_traj_sw(float4* obs, int* srv, float* rew,
                                                uint8_t* done, const int4* tab, int E, int n,
                                                int layout, int work) {
  __shared__ Slot ring[RING];
  __shared__ int full[RING];  // compute waves that filled the slot for its current step
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  if (threadIdx.x < RING) full[threadIdx.x] = 0;
  __syncthreads();
  if (w < 4) {
    const int wave = blockIdx.x * 4 + w;
    const int seg = lane / P, u = lane - seg * P;
    const int e = min(wave * G + seg, E - 1);
    float x = (float)lane;
    uint32_t h = (uint32_t)(e * 31 + u) * 2654435761u;
    for (int i = 0; i < n; ++i) {
      h = h * 1664525u + 1013904223u;
      const int4 r = tab[(h >> 8) % 40000u];
      x = spin(x + (float)r.x, work);
      const int sl = i % RING;
      // wait until the store wave has drained this slot's previous use (step i - RING):
      // full[sl] gains 4 from the compute waves and 4 from the store wave per use; it is
      // >= 8 * (i / RING) when free for step i
      // (bounded spin: a protocol bug ends the kernel instead of hanging the GPU)
      for (int it = 0; it < (1 << 22) && __hip_atomic_load(&full[sl], __ATOMIC_ACQUIRE,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP) <
                                             8 * (i / RING); ++it)
        __builtin_amdgcn_s_sleep(1);
      ring[sl].obs[w][lane] = make_float4(x, (float)i, (float)u, (float)r.y);
      ring[sl].srv[w][lane] = (int)x;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_fetch_add(&full[sl], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
    // store wave: step i's slot is ready when full == 8 * (i / RING) + 4
    for (int i = 0; i < n; ++i) {
      const int sl = i % RING;
      const int want = 8 * (i / RING) + 4;
      for (int it = 0; it < (1 << 22) && __hip_atomic_load(&full[sl], __ATOMIC_ACQUIRE,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP) < want;
           ++it)
        __builtin_amdgcn_s_sleep(1);
      for (int cw = 0; cw < 4; ++cw) {
        const int wave = blockIdx.x * 4 + cw;
        const int seg = lane / P, u = lane - seg * P;
        const int e = wave * G + seg;
        if (e < E) {
          const size_t ui = layout == 0 ? ((size_t)i * E + e) * U + u : (size_t)e * U + u;
          const size_t ei = layout == 0 ? (size_t)i * E + e : (size_t)e;
          const float4 o = ring[sl].obs[cw][lane];
          const int s = ring[sl].srv[cw][lane];
          if (u < U) {
            obs[ui] = o;
            srv[ui] = s;
          }
          if (u == P - 1) {
            rew[ei] = o.x;
            done[ei] = (uint8_t)i;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // slot reads done before release
      if (lane == 0) __hip_atomic_fetch_add(&full[sl], 4, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

extern "C" int tb_run(void* obs, void* srv, void* rew, void* done, void* tab, int E, int n,
                      int layout, int mode, int work, int reps, void* stream) {
  const int waves = (E + 1) / 2;
  for (int r = 0; r < reps; ++r) {
    if (mode == 3)
      hipLaunchKernelGGL(k_traj_sw, dim3((waves + 3) / 4), dim3(320), 0, (hipStream_t)stream,
                         (float4*)obs, (int*)srv, (float*)rew, (uint8_t*)done, (const int4*)tab,
                         E, n, layout, work);
    else
      hipLaunchKernelGGL(k_traj, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                         (float4*)obs, (int*)srv, (float*)rew, (uint8_t*)done, (const int4*)tab,
                         E, n, layout, mode, work);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
