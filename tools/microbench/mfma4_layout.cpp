// Operand / result lane layout of v_mfma_f32_4x4x4_16b_f16 on gfx950 (round 6: the omega
// conv's centre tap).  A[i][k] of block b is assumed at lane 4 b + i (k = 0..3 in the half4),
// B[k][j] at lane 4 b + j, D[i][j] at lane 4 b + j, register i.  The probe fills A and B with
// distinct small integers and checks every D element against that assumption.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  half4 a, b;
  for (int k = 0; k < 4; ++k) {
    a[k] = (_Float16)(float)((l & 3) * 4 + k + 1 + (l >> 2) * 0);    // A[i = l & 3][k], block-independent
    b[k] = (_Float16)(float)(k == (l & 3) ? 1 + (l >> 2) : 0);        // B = (1 + b) I
  }
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x4f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  // expected under the assumption: D[i][j] of block b = (1 + b) A[i][j] = (1 + b)(4 i + j + 1),
  // at lane 4 b + j, register i
  int bad = 0, badT = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int b = l >> 2, j = l & 3, i = r;
      const float e = (float)((1 + b) * (4 * i + j + 1));
      const float eT = (float)((1 + b) * (4 * j + i + 1));   // transposed: D[i = l & 3][j = r]
      bad += h[l * 4 + r] != e;
      badT += h[l * 4 + r] != eT;
    }
  printf("mfma_f32_4x4x4f16 layout: assumed %s (%d mismatches), transposed %s (%d)\n",
         bad ? "WRONG" : "OK", bad, badT ? "WRONG" : "OK", badT);
  if (bad)
    for (int l = 0; l < 64; ++l) printf("lane %2d: %g %g %g %g\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  return bad ? 1 : 0;
}
