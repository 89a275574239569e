// Mean signed error of the cells' gate activations on gfx950 (device_common.h fast_sigmoid /
// fast_tanh on v_exp_f32 / v_rcp_f32, and the libm expf / tanhf / IEEE-division forms) against
// the exact value (double on the host), in ulps of the exact result, over inputs spread like
// gate pre-activations (|z| < 8) and cell states (|c| < 2).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../aa-rmvsnet_amd/csrc/device_common.h"

__global__ void fn_kernel(const float* x, float* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  o[6 * i + 0] = aarmvs::fast_sigmoid(v);
  o[6 * i + 1] = aarmvs::fast_tanh(v);
  o[6 * i + 2] = 1.0f / (1.0f + expf(-v));
  o[6 * i + 3] = tanhf(v);
  o[6 * i + 4] = aarmvs::precise_sigmoid(v);
  o[6 * i + 5] = aarmvs::precise_tanh(v);
}

int main() {
  const int n = 1 << 20;
  std::mt19937 rng(3);
  std::uniform_real_distribution<float> ud(-8.f, 8.f);
  std::vector<float> x(n), o(6 * n);
  for (auto& v : x) v = ud(rng);
  float *dx, *dy;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dy, 6 * n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(fn_kernel, dim3(n / 256), dim3(256), 0, 0, dx, dy, n);
  hipMemcpy(o.data(), dy, 6 * n * 4, hipMemcpyDeviceToHost);
  const char* names[6] = {"fast_sigmoid", "fast_tanh", "sigmoid(expf, div)", "tanhf", "precise_sigmoid", "precise_tanh"};
  for (int f = 0; f < 6; ++f) {
    double s = 0, a = 0, s_small = 0;
    long ns = 0;
    for (int i = 0; i < n; ++i) {
      const double v = x[i];
      double ex = f == 0 || f == 2 || f == 4 ? 1.0 / (1.0 + std::exp(-v)) : std::tanh(v);
      const double ulp = std::ldexp(1.0, std::ilogb((float)ex) - 23);
      const double e = ((double)o[6 * i + f] - ex) / ulp;
      s += e;
      a += std::fabs(e);
      if (std::fabs(v) < 0.5) { s_small += e; ++ns; }
    }
    printf("%-20s mean err %+.4f ulp, mean |err| %.3f ulp; |x| < 0.5: mean err %+.4f ulp\n", names[f], s / n, a / n,
           s_small / ns);
  }
  return 0;
}
