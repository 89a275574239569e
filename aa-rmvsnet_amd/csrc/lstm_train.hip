// ConvLSTMCell gate math for the BPTT recompute (module.py:76-92; models.module.ConvLSTMCell
// on the GPU): the forward from the conv output z to (h, c), and its backward from (dh, dc)
// to (dz, dc_prev) in one pass each, instead of ATen's ~20 pointwise launches per cell.
//
// z is NCHW [B][4 hid][HW] (gates i, f, o, g in channel blocks, torch.split order), c_prev /
// h / c / dh / dc / dc_prev are [B][hid][HW].  Activations are the accurate libm forms
// (1 / (1 + exp(-x)), tanhf), as torch's.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "aarmvs_internal.h"

namespace aarmvs {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

struct GateIdx {
  size_t zi, zf, zo, zg, s;   // offsets of the four gates and of the state element
};

__device__ __forceinline__ GateIdx gate_idx(size_t e, int hid, int HW) {
  const size_t per_b = (size_t)hid * HW;
  const size_t b = e / per_b, r = e - b * per_b;   // r = ch * HW + p
  GateIdx g;
  g.s = e;
  g.zi = b * 4 * per_b + r;
  g.zf = g.zi + per_b;
  g.zo = g.zf + per_b;
  g.zg = g.zo + per_b;
  return g;
}

__global__ void __launch_bounds__(256) lstm_gates_fwd_kernel(const float* __restrict__ z,
                                                             const float* __restrict__ c_prev,
                                                             size_t n, int hid, int HW,
                                                             float* __restrict__ h,
                                                             float* __restrict__ c) {
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
    const GateIdx q = gate_idx(e, hid, HW);
    const float i = sigm(z[q.zi]), f = sigm(z[q.zf]), o = sigm(z[q.zo]), g = tanhf(z[q.zg]);
    const float cn = f * c_prev[q.s] + i * g;   // module.py:88
    c[q.s] = cn;
    h[q.s] = o * tanhf(cn);                      // module.py:89
  }
}

__global__ void __launch_bounds__(256) lstm_gates_bwd_kernel(
    const float* __restrict__ z, const float* __restrict__ c_prev, const float* __restrict__ dh,
    const float* __restrict__ dc, size_t n, int hid, int HW, float* __restrict__ dz,
    float* __restrict__ dc_prev) {
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
    const GateIdx q = gate_idx(e, hid, HW);
    const float i = sigm(z[q.zi]), f = sigm(z[q.zf]), o = sigm(z[q.zo]), g = tanhf(z[q.zg]);
    const float cp = c_prev[q.s];
    const float cn = f * cp + i * g;
    const float tc = tanhf(cn);
    const float gh = dh ? dh[q.s] : 0.0f;
    const float gc = (dc ? dc[q.s] : 0.0f) + gh * o * (1.0f - tc * tc);
    dz[q.zi] = gc * g * i * (1.0f - i);
    dz[q.zf] = gc * cp * f * (1.0f - f);
    dz[q.zo] = gh * tc * o * (1.0f - o);
    dz[q.zg] = gc * i * (1.0f - g * g);
    dc_prev[q.s] = gc * f;
  }
}

static inline unsigned gates_blocks(size_t n) {
  return (unsigned)std::min<size_t>((n + 255) / 256, 65535);
}

hipError_t launch_lstm_gates_fwd(const float* z, const float* c_prev, int B, int hid, int HW,
                                 float* h, float* c, hipStream_t s) {
  const size_t n = (size_t)B * hid * HW;
  hipLaunchKernelGGL(lstm_gates_fwd_kernel, dim3(gates_blocks(n)), dim3(256), 0, s, z, c_prev, n,
                     hid, HW, h, c);
  return hipGetLastError();
}

hipError_t launch_lstm_gates_bwd(const float* z, const float* c_prev, const float* dh,
                                 const float* dc, int B, int hid, int HW, float* dz, float* dc_prev,
                                 hipStream_t s) {
  const size_t n = (size_t)B * hid * HW;
  hipLaunchKernelGGL(lstm_gates_bwd_kernel, dim3(gates_blocks(n)), dim3(256), 0, s, z, c_prev, dh,
                     dc, n, hid, HW, dz, dc_prev);
  return hipGetLastError();
}

}  // namespace aarmvs
