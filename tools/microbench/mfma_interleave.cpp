// Does a chain of dependent v_mfma_f32_32x32x16_f16 give the same bits whatever else runs on
// the SIMD?  Every wave of a large grid computes the same chain (T steps of 3 split-fp16
// products, the inputs from global memory as in the library's kernels) and writes its result;
// the results are compared bit for bit with the one of a lone wave.  Variants:
//   0 one accumulator, the three products of a step back to back (h3_mfma_chunk's pattern)
//   1 three accumulators, one per product (no MFMA reads the result of the one before it)
//   2 like 0 with a v_nop-free VALU op on the accumulator between steps (acc = acc * 1)
// Waves start after a wave-dependent s_sleep so that their MFMAs interleave differently.
// Then the same with a second kernel running concurrently on another stream: chains of
// v_mfma_f32_16x16x32_f16 (the weight gradient's shape) with 64 KB of LDS per block.
// usage: mfma_interleave [blocks] [waves per block]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int V>
__global__ void chain_kernel(const half8* A, const half8* B, int T, float* D, int stagger) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gw = blockIdx.x * (blockDim.x >> 6) + w;
  if (stagger) {
    for (int i = 0; i < (gw * 7) % 13; ++i) __builtin_amdgcn_s_sleep(1);
  }
  floatx16 p, q, r;
  for (int i = 0; i < 16; ++i) p[i] = q[i] = r[i] = 0.f;
  for (int t = 0; t < T; ++t) {
    const half8 ah = A[(t * 2 + 0) * 64 + l], al = A[(t * 2 + 1) * 64 + l];
    const half8 bh = B[(t * 2 + 0) * 64 + l], bl = B[(t * 2 + 1) * 64 + l];
    if (V == 1) {
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, p, 0, 0, 0);
      q = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, q, 0, 0, 0);
      r = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, r, 0, 0, 0);
    } else {
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, p, 0, 0, 0);
      p = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, p, 0, 0, 0);
      if (V == 2) {
        float one = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, 1.0f)));
        for (int i = 0; i < 16; ++i) p[i] *= one;
      }
    }
  }
  float* d = D + (size_t)gw * 1024;
  for (int i = 0; i < 16; ++i) d[i * 64 + l] = V == 1 ? (p[i] + q[i]) + r[i] : p[i];
}

typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void noise_kernel(const half8* A, int T, float* out) {
  extern __shared__ half8 sh[];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) sh[i] = A[i % 1024];
  __syncthreads();
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < T; ++t) {
    const half8 a = sh[(t * 64 + l) & 4095], b = sh[(t * 64 + l + 17) & 4095];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc, 0, 0, 0);
  }
  if (acc[0] == 1234.5f) out[0] = acc[1];
}

template <int V>
static void run_noisy(const half8* dA, const half8* dB, int T, float* dD, int blocks, int wpb) {
  std::vector<float> ref(1024), all((size_t)blocks * wpb * 1024);
  hipLaunchKernelGGL(chain_kernel<V>, dim3(1), dim3(64), 0, 0, dA, dB, T, dD, 0);
  hipDeviceSynchronize();
  hipMemcpy(ref.data(), dD, 4096, hipMemcpyDeviceToHost);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipFuncSetAttribute((const void*)noise_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  long bad_waves = 0, bad_vals = 0, total = 0;
  for (int rep = 0; rep < 8; ++rep) {
    hipMemsetAsync(dD, 0, all.size() * 4, s1);
    hipStreamSynchronize(s1);
    for (int k = 0; k < 4; ++k)
      hipLaunchKernelGGL(noise_kernel, dim3(1024), dim3(512), 65536, s2, dA, 2000, dD + all.size());
    hipLaunchKernelGGL(chain_kernel<V>, dim3(blocks), dim3(64 * wpb), 0, s1, dA, dB, T, dD, rep & 1);
    hipDeviceSynchronize();
    hipMemcpy(all.data(), dD, all.size() * 4, hipMemcpyDeviceToHost);
    for (int g = 0; g < blocks * wpb; ++g) {
      long b = 0;
      for (int i = 0; i < 1024; ++i) b += memcmp(&all[(size_t)g * 1024 + i], &ref[i], 4) != 0;
      bad_vals += b;
      bad_waves += b != 0;
    }
    total += (long)blocks * wpb;
  }
  printf("variant %d beside the 16x16x32 noise kernel: %ld of %ld waves differ from the lone wave (%ld values)\n",
         V, bad_waves, total, bad_vals);
}

template <int V>
static void run(const half8* dA, const half8* dB, int T, float* dD, int blocks, int wpb) {
  std::vector<float> ref(1024), all((size_t)blocks * wpb * 1024);
  hipLaunchKernelGGL(chain_kernel<V>, dim3(1), dim3(64), 0, 0, dA, dB, T, dD, 0);
  hipDeviceSynchronize();
  hipMemcpy(ref.data(), dD, 4096, hipMemcpyDeviceToHost);
  for (int stagger = 0; stagger < 2; ++stagger) {
    hipMemset(dD, 0, all.size() * 4);
    hipLaunchKernelGGL(chain_kernel<V>, dim3(blocks), dim3(64 * wpb), 0, 0, dA, dB, T, dD, stagger);
    hipDeviceSynchronize();
    hipMemcpy(all.data(), dD, all.size() * 4, hipMemcpyDeviceToHost);
    long bad_waves = 0, bad_vals = 0;
    for (int g = 0; g < blocks * wpb; ++g) {
      long b = 0;
      for (int i = 0; i < 1024; ++i) b += memcmp(&all[(size_t)g * 1024 + i], &ref[i], 4) != 0;
      bad_vals += b;
      bad_waves += b != 0;
    }
    printf("variant %d stagger %d: %d waves, %ld differ from the lone wave (%ld of %ld values)\n", V, stagger,
           blocks * wpb, bad_waves, bad_vals, (long)blocks * wpb * 1024);
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048, wpb = argc > 2 ? atoi(argv[2]) : 8;
  const int T = 48;
  std::mt19937 rng(5);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<_Float16> A(T * 2 * 64 * 8), B(T * 2 * 64 * 8);
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 512; ++i) {
      const float a = nd(rng) * 4096.f, b = nd(rng) * 4096.f;
      const _Float16 ah = (_Float16)a, bh = (_Float16)b;
      A[(t * 2) * 512 + i] = ah;
      A[(t * 2 + 1) * 512 + i] = (_Float16)(a - (float)ah);
      B[(t * 2) * 512 + i] = bh;
      B[(t * 2 + 1) * 512 + i] = (_Float16)(b - (float)bh);
    }
  half8 *dA, *dB;
  float* dD;
  hipMalloc(&dA, A.size() * 2);
  hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dD, (size_t)blocks * wpb * 4096 + 4096);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  run<0>(dA, dB, T, dD, blocks, wpb);
  run<1>(dA, dB, T, dD, blocks, wpb);
  run<2>(dA, dB, T, dD, blocks, wpb);
  run_noisy<0>(dA, dB, T, dD, blocks, wpb);
  run_noisy<1>(dA, dB, T, dD, blocks, wpb);
  return 0;
}
