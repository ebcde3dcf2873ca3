// Dev probe (GPU box): the accuracy of the float32 log2 the fast utility uses (__log2f, the
// hardware v_log_f32) over every float32 x in [2^-8, 2^8) -- the rates of the utility tables
// (0.01 .. 100 Mbit/s at the default BoundedLog) and more. Against float64 log2 of the same x,
// per x: err = |log2f(x) - log2(x)|, reported as
//   a) err / max(|log2 x|, 1) in units of 2^-23 (the form of DESIGN 4's u_err term), and
//   b) err in ulps of the float32 result.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/log2_probe tools/log2_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void k_probe(uint32_t lo, uint32_t n, uint32_t per, float* out_a, float* out_b,
                        uint32_t* arg_a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  float ma = 0.f, mb = 0.f;
  uint32_t xa = 0;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t k = t * per + i;
    if (k >= n) break;
    const uint32_t bits = lo + k;
    const float x = __uint_as_float(bits);
    const float y = __log2f(x);
    const double yd = log2((double)x);
    const double err = fabs((double)y - yd);
    const double a = err / fmax(fabs(yd), 1.0) * 0x1p23;
    const double ulp = (double)fabsf(nextafterf(y, INFINITY) - y);
    const double b = yd == 0.0 ? (y == 0.f ? 0.0 : 1e9) : err / (ulp > 0.0 ? ulp : 1e-45);
    if (a > ma) { ma = (float)a; xa = bits; }
    if (b > mb) mb = (float)b;
  }
  out_a[t] = ma;
  out_b[t] = mb;
  arg_a[t] = xa;
}

int main() {
  const float xlo = 0x1p-8f, xhi = 0x1p8f;
  uint32_t lo, hi;
  memcpy(&lo, &xlo, 4);
  memcpy(&hi, &xhi, 4);
  const uint32_t n = hi - lo, threads = 1u << 20, per = (n + threads - 1) / threads;
  float *a, *b;
  uint32_t* xa;
  if (hipMalloc(&a, 4 * threads) || hipMalloc(&b, 4 * threads) || hipMalloc(&xa, 4 * threads)) return 1;
  hipLaunchKernelGGL(k_probe, dim3(threads / 256), dim3(256), 0, 0, lo, n, per, a, b, xa);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<float> ha(threads), hb(threads);
  std::vector<uint32_t> hx(threads);
  if (hipMemcpy(ha.data(), a, 4 * threads, hipMemcpyDeviceToHost) ||
      hipMemcpy(hb.data(), b, 4 * threads, hipMemcpyDeviceToHost) ||
      hipMemcpy(hx.data(), xa, 4 * threads, hipMemcpyDeviceToHost)) return 3;
  float ma = 0.f, mb = 0.f;
  uint32_t xm = 0;
  for (uint32_t i = 0; i < threads; ++i) {
    if (ha[i] > ma) { ma = ha[i]; xm = hx[i]; }
    if (hb[i] > mb) mb = hb[i];
  }
  float xw;
  memcpy(&xw, &xm, 4);
  printf("{\"probe\": \"log2f\", \"values\": %u, \"max_err_over_max_abs_log2_1_in_2^-23\": %.4f, "
         "\"at_x\": %.9g, \"max_err_ulps_of_result\": %.4f}\n", n, ma, xw, mb);
  return 0;
}
