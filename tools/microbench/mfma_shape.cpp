// Does the MFMA shape change the clock the chip holds on the cells' kind of loop?  Two
// kernels of equal FLOPs and equal LDS bytes per FLOP, every CU busy with one 8-wave block
// (two waves per SIMD, as the ConvLSTM cells), random f16 operands re-read from LDS:
//   A: per step 6 ds_read_b128 + 6 v_mfma_f32_32x32x16_f16 on 2 accumulators (h3_mfma_chunk)
//   B: per step 6 ds_read_b128 + 12 v_mfma_f32_16x16x32_f16 on 4 accumulators
// usage: mfma_shape [steps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__);                      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kSlots = 1024;   // half8 slots in LDS (16 KB)

template <int SHAPE>
__global__ void __launch_bounds__(512) shape_kernel(const half8* __restrict__ src, int T, float* out) {
  __shared__ half8 sh[kSlots];
  for (int i = threadIdx.x; i < kSlots; i += 512) sh[i] = src[i];
  __syncthreads();
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (SHAPE == 0) {
    floatx16 a0, a1;
    for (int i = 0; i < 16; ++i) a0[i] = a1[i] = 0.f;
    for (int t = 0; t < T; ++t) {
      const int base = ((t * 6 + w) * 64) & (kSlots - 1);
      const half8 ah0 = sh[(base + l) & (kSlots - 1)], al0 = sh[(base + 64 + l) & (kSlots - 1)];
      const half8 ah1 = sh[(base + 128 + l) & (kSlots - 1)], al1 = sh[(base + 192 + l) & (kSlots - 1)];
      const half8 bh = sh[(base + 256 + l) & (kSlots - 1)], bl = sh[(base + 320 + l) & (kSlots - 1)];
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bh, a0, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bl, a0, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al0, bh, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bh, a1, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bl, a1, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al1, bh, a1, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += a0[i] + a1[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  } else {
    floatx4 c[4];
    for (int k = 0; k < 4; ++k)
      for (int i = 0; i < 4; ++i) c[k][i] = 0.f;
    for (int t = 0; t < T; ++t) {
      const int base = ((t * 6 + w) * 64) & (kSlots - 1);
      const half8 ah0 = sh[(base + l) & (kSlots - 1)], al0 = sh[(base + 64 + l) & (kSlots - 1)];
      const half8 ah1 = sh[(base + 128 + l) & (kSlots - 1)], al1 = sh[(base + 192 + l) & (kSlots - 1)];
      const half8 bh = sh[(base + 256 + l) & (kSlots - 1)], bl = sh[(base + 320 + l) & (kSlots - 1)];
      // 2 m-tiles x 2 n-tiles x 3 products: 12 MFMAs (the n-tiles reuse B with swapped halves)
      const half8 bh2 = bl, bl2 = bh;
      c[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah0, bh, c[0], 0, 0, 0);
      c[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah0, bl, c[0], 0, 0, 0);
      c[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al0, bh, c[0], 0, 0, 0);
      c[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah0, bh2, c[1], 0, 0, 0);
      c[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah0, bl2, c[1], 0, 0, 0);
      c[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al0, bh2, c[1], 0, 0, 0);
      c[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bh, c[2], 0, 0, 0);
      c[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bl, c[2], 0, 0, 0);
      c[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al1, bh, c[2], 0, 0, 0);
      c[3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bh2, c[3], 0, 0, 0);
      c[3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bl2, c[3], 0, 0, 0);
      c[3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al1, bh2, c[3], 0, 0, 0);
    }
    float s = 0.f;
    for (int k = 0; k < 4; ++k)
      for (int i = 0; i < 4; ++i) s += c[k][i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  }
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 20000;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<_Float16> h(kSlots * 8);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : h) x = (_Float16)U(rng);
  half8* src;
  float* out;
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)cus * 512 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    for (int shape = 0; shape < 2; ++shape) {
      auto launch = [&] {
        if (shape == 0)
          hipLaunchKernelGGL(shape_kernel<0>, dim3(cus), dim3(512), 0, 0, src, T, out);
        else
          hipLaunchKernelGGL(shape_kernel<1>, dim3(cus), dim3(512), 0, 0, src, T, out);
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double flop = 6.0 * 32768.0 * T * 8 * cus;   // both shapes: 196,608 FLOP per wave-step
      printf("rep %d %s: %.3f ms, %.1f TFLOP/s (f16), cycles/step/SIMD at 2.4 GHz %.1f\n", rep,
             shape == 0 ? "32x32x16" : "16x16x32", ms, flop / ms / 1e9, ms * 1e-3 * 2.4e9 / (T * 2.0));
    }
  return 0;
}
