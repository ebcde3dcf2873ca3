// Dev tool: memory floor of the step kernel's access pattern on MI355X (no compute).
//  kind 0: same lane mapping / loads / stores as the packed step kernel, trivial math
//  kind 1: ideal streaming with the same read:write byte ratio (float4 read, 2x float4 write)
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void k_pattern(int2* st, uint64_t* pcg, int* t, float4* obs,
                                                int* serving, float* reward, uint8_t* done,
                                                int E, int U) {
  // the step kernel's layout: int16x4 UE state (8 B), segments of pitch P (32 for U = 30)
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int P = U > 16 && U <= 32 ? 32 : (U > 8 && U <= 16 ? 16 : U);
  const int G = 64 / P;
  const int seg = lane / P;
  const int u = lane - seg * P;
  const int e = wave * G + seg;
  if (seg >= G || e >= E) return;
  const int uc = u < U ? u : U - 1;
  const size_t idx = (size_t)e * U + uc;
  const ulonglong2* pr = reinterpret_cast<const ulonglong2*>(pcg + 6 * (size_t)e);
  const ulonglong2 a = pr[0], b = pr[1];
  const int tt = t[e];
  int2 s = st[idx];
  s.x += 1;
  s.y += (int)(a.x & 1);
  if (u < U) {
    st[idx] = s;
    serving[idx] = s.y;
    obs[idx] = make_float4((float)s.x, (float)s.y, (float)tt, (float)(b.y & 7));
  }
  if (u == U - 1 && tt % 3 == 0)  // the stream moves in about a third of the env-steps
    *reinterpret_cast<ulonglong2*>(pcg + 6 * (size_t)e) = make_ulonglong2(a.x + 1, a.y);
  if (u == P - 1) {
    t[e] = tt + 1;
    reward[e] = (float)tt;
    done[e] = (uint8_t)(tt > 19);
  }
}

__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ in, float4* __restrict__ out,
                                               size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 v = in[i];
  out[2 * i] = v;
  out[2 * i + 1] = make_float4(v.y, v.x, v.w, v.z);
}

extern "C" int mb_pattern(void* st, void* pcg, void* t, void* obs, void* serving, void* reward,
                          void* done, int E, int U, int reps, void* stream) {
  const int G = 64 / U;
  const int waves = (E + G - 1) / G;
  for (int r = 0; r < reps; ++r)
  hipLaunchKernelGGL(k_pattern, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     (int2*)st, (uint64_t*)pcg, (int*)t, (float4*)obs, (int*)serving,
                     (float*)reward, (uint8_t*)done, E, U);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mb_stream(const void* in, void* out, size_t n, int reps, void* stream) {
  for (int r = 0; r < reps; ++r)
  hipLaunchKernelGGL(k_stream, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)in, (float4*)out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// launch-overhead probes: same grid as the step kernel
__global__ __launch_bounds__(256) void k_empty(int* p) {
  if (threadIdx.x == 1000) p[0] = 1;
}
__global__ __launch_bounds__(256) void k_touch(const int4* __restrict__ st, int* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int4 v = st[i];
    if (v.x == 123456789) out[0] = v.y;
  }
}
extern "C" int mb_empty(void* p, int blocks, int reps, void* stream) {
  for (int r = 0; r < reps; ++r)
  hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (int*)p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int mb_touch(const void* st, void* out, int n, int reps, void* stream) {
  for (int r = 0; r < reps; ++r)
  hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const int4*)st, (int*)out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
