// How v_mfma_f32_32x32x16_f16 rounds (gfx950): D = C + A B with random fp16 A, B and fp32 C,
// compared with the exact result (long double on the host) and its round-to-nearest-even fp32.
// Prints the fraction of outputs equal to RNE(exact), and the mean signed error in units of the
// output's ulp: a correctly rounded unit gives ~0 mean; truncation toward zero gives a
// negative mean of the error's projection on sign(exact).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// one wave: A [32][16] (row-major by M), B [16][32], C/D [32][32]; lane layout as the library's
// (A: lane l holds row l & 31, k = 8 (l >> 5) .. +7; B: column l & 31, same k; D: 16 values per lane)
__global__ void mfma_kernel(const _Float16* A, const _Float16* B, const float* C, float* D, int reps) {
  const int l = threadIdx.x;
  half8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = A[(l & 31) * 16 + 8 * (l >> 5) + i];
    b[i] = B[(8 * (l >> 5) + i) * 32 + (l & 31)];
  }
  floatx16 acc;
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    acc[r] = C[row * 32 + col];
  }
  for (int i = 0; i < reps; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    D[row * 32 + col] = acc[r];
  }
}

int main() {
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int trials = 200;
  long eq = 0, tot = 0, toward0 = 0, away = 0;
  double sum_err_ulp = 0.0, sum_signed = 0.0, sum_plain = 0.0, sum_pos = 0.0, sum_neg = 0.0;
  double sum_maxulp = 0.0;
  long npos = 0, nneg = 0;
  _Float16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, 512 * 2);
  hipMalloc(&dB, 512 * 2);
  hipMalloc(&dC, 1024 * 4);
  hipMalloc(&dD, 1024 * 4);
  for (int t = 0; t < trials; ++t) {
    std::vector<_Float16> A(512), B(512);
    std::vector<float> C(1024), D(1024);
    // mixed magnitudes: products spanning several binades, C of either sign and size
    for (auto& v : A) v = (_Float16)(nd(rng) * std::ldexp(1.0f, (int)(rng() % 8) - 4));
    for (auto& v : B) v = (_Float16)(nd(rng) * std::ldexp(1.0f, (int)(rng() % 8) - 4));
    for (auto& v : C) v = nd(rng) * std::ldexp(1.0f, (int)(rng() % 10) - 5);
    hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, 1);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    for (int m = 0; m < 32; ++m)
      for (int n = 0; n < 32; ++n) {
        long double ex = C[m * 32 + n];
        double mx = std::fabs((double)C[m * 32 + n]);
        for (int k = 0; k < 16; ++k) {
          const long double pr = (long double)(float)A[m * 16 + k] * (long double)(float)B[k * 32 + n];
          ex += pr;
          mx = std::max(mx, (double)std::fabs((double)pr));
        }
        const float rne = (float)ex;
        const float d = D[m * 32 + n];
        const double ulp = std::ldexp(1.0, std::ilogb(rne == 0.f ? 1e-30f : rne) - 23);
        const double err = (double)((long double)d - ex) / ulp;
        ++tot;
        if (d == rne) ++eq;
        sum_err_ulp += std::fabs(err);
        const double s = (ex > 0 ? err : -err);   // error along the sign of the exact value
        sum_signed += s;
        sum_plain += err;
        (ex > 0 ? sum_pos : sum_neg) += err;
        (ex > 0 ? npos : nneg)++;
        sum_maxulp += (double)((long double)d - ex) / std::ldexp(1.0, std::ilogb(mx) - 23);
        if (d != rne) (std::fabs((double)d) < std::fabs((double)ex) ? toward0 : away)++;
      }
  }
  printf("v_mfma_f32_32x32x16_f16: %ld outputs, %.4f equal to RNE(exact); mean |err| %.3f ulp; "
         "mean err along sign(exact) %+.4f ulp; of the inexact: %ld toward zero, %ld away\n",
         tot, (double)eq / tot, sum_err_ulp / tot, sum_signed / tot, toward0, away);
  printf("  mean signed err %+.4f ulp (exact > 0: %+.4f, exact < 0: %+.4f); in ulps of the largest addend %+.4f\n",
         sum_plain / tot, sum_pos / npos, sum_neg / nneg, sum_maxulp / tot);
  return 0;
}
