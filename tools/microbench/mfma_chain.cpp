// Bias of a long split-fp16 accumulation on v_mfma_f32_32x32x16_f16 (gfx950), as the BPTT's
// input-gradient conv runs it: out = sum over T steps of (a_hi b_hi + a_hi b_lo + a_lo b_hi)
// with fp32 a, b split into fp16 hi + lo.  Variants:
//   0 one accumulator (every MFMA adds into it)
//   1 sign-balanced: step t's products go to acc_p (+a) on even t and to acc_n (-a) on odd t,
//     out = acc_p - acc_n
//   2 sign-balanced within a step: even t: hh, hl -> acc_p, lh -> acc_n (-a_lo); odd t: hh, hl
//     -> acc_n (-a_hi), lh -> acc_p
// Reports the mean signed error and mean |error| in units of the largest partial-sum
// magnitude's ulp, against the exact sum of the split products (long double on the host).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int V>
__global__ void chain_kernel(const _Float16* Ah, const _Float16* Al, const _Float16* Bh, const _Float16* Bl,
                             int T, float* D) {
  const int l = threadIdx.x;
  floatx16 p, n;
  for (int r = 0; r < 16; ++r) p[r] = n[r] = 0.f;
  for (int t = 0; t < T; ++t) {
    half8 ah, al, bh, bl;
    for (int i = 0; i < 8; ++i) {
      const int ai = (t * 32 + (l & 31)) * 16 + 8 * (l >> 5) + i;
      const int bi = (t * 16 + 8 * (l >> 5) + i) * 32 + (l & 31);
      ah[i] = Ah[ai];
      al[i] = Al[ai];
      bh[i] = Bh[bi];
      bl[i] = Bl[bi];
    }
    if (V == 0) {
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, p, 0, 0, 0);
    } else if (V == 1) {
      if (t & 1) {
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-ah, bh, n, 0, 0, 0);
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-ah, bl, n, 0, 0, 0);
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-al, bh, n, 0, 0, 0);
      } else {
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, p, 0, 0, 0);
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, p, 0, 0, 0);
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, p, 0, 0, 0);
      }
    } else {
      if (t & 1) {
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-ah, bh, n, 0, 0, 0);
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-ah, bl, n, 0, 0, 0);
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, p, 0, 0, 0);
      } else {
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, p, 0, 0, 0);
        p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, p, 0, 0, 0);
        n = __builtin_amdgcn_mfma_f32_32x32x16_f16(-al, bh, n, 0, 0, 0);
      }
    }
  }
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    D[row * 32 + col] = V == 0 ? p[r] : p[r] - n[r];
  }
}

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int T = 36, trials = 60;
  std::vector<float> A(T * 512), B(T * 512);
  std::vector<_Float16> Ah(T * 512), Al(T * 512), Bh(T * 512), Bl(T * 512);
  _Float16 *dAh, *dAl, *dBh, *dBl;
  float* dD;
  hipMalloc(&dAh, T * 1024);
  hipMalloc(&dAl, T * 1024);
  hipMalloc(&dBh, T * 1024);
  hipMalloc(&dBl, T * 1024);
  hipMalloc(&dD, 4096);
  for (int v = 0; v < 3; ++v) {
    double sum_s = 0, sum_a = 0;
    long cnt = 0;
    std::mt19937 r2(11);
    for (int tr = 0; tr < trials; ++tr) {
      for (int i = 0; i < T * 512; ++i) {
        A[i] = nd(r2) * 4096.f;          // weights scaled towards 2^14 as packed
        B[i] = nd(r2) * 4096.f * (1 + (r2() % 3));
        Ah[i] = (_Float16)A[i];
        Al[i] = (_Float16)(A[i] - (float)Ah[i]);
        Bh[i] = (_Float16)B[i];
        Bl[i] = (_Float16)(B[i] - (float)Bh[i]);
      }
      hipMemcpy(dAh, Ah.data(), T * 1024, hipMemcpyHostToDevice);
      hipMemcpy(dAl, Al.data(), T * 1024, hipMemcpyHostToDevice);
      hipMemcpy(dBh, Bh.data(), T * 1024, hipMemcpyHostToDevice);
      hipMemcpy(dBl, Bl.data(), T * 1024, hipMemcpyHostToDevice);
      if (v == 0) hipLaunchKernelGGL(chain_kernel<0>, dim3(1), dim3(64), 0, 0, dAh, dAl, dBh, dBl, T, dD);
      if (v == 1) hipLaunchKernelGGL(chain_kernel<1>, dim3(1), dim3(64), 0, 0, dAh, dAl, dBh, dBl, T, dD);
      if (v == 2) hipLaunchKernelGGL(chain_kernel<2>, dim3(1), dim3(64), 0, 0, dAh, dAl, dBh, dBl, T, dD);
      std::vector<float> D(1024);
      hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
      for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
          long double ex = 0, mx = 0;
          for (int t = 0; t < T; ++t) {
            for (int k = 0; k < 16; ++k) {
              const int ai = (t * 32 + m) * 16 + k, bi = (t * 16 + k) * 32 + n;
              ex += (long double)(float)Ah[ai] * (float)Bh[bi] + (long double)(float)Ah[ai] * (float)Bl[bi] +
                    (long double)(float)Al[ai] * (float)Bh[bi];
            }
            mx = std::max(mx, std::fabs(ex));
          }
          const double u = std::ldexp(1.0, std::ilogb((double)mx) - 23);
          const double e = (double)((long double)D[m * 32 + n] - ex) / u;
          sum_s += e;
          sum_a += std::fabs(e);
          ++cnt;
        }
    }
    printf("variant %d (T=%d steps, 3 MFMAs each): mean err %+.3f ulp(max partial), mean |err| %.3f\n", v, T,
           sum_s / cnt, sum_a / cnt);
  }
  return 0;
}
