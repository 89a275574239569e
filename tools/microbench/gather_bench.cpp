// Microbenchmark: bilinear gather of 32-channel fp32 features (1600x1184) in the
// access patterns the cost-slice kernel could use.  Diagnostic only (not shipped).
//   V1  NCHW, one thread per pixel, 32 ch x 4 taps dword loads
//   V2  NHWC, one thread per pixel, 4 taps x 8 dwordx4 loads
//   V3  NHWC, 8 lanes per pixel (lane = 4 channels), 4 taps x 1 dwordx4 load
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int H = 1184, W = 1600, C = 32;

__device__ __forceinline__ void pos(int x, int y, float& ix, float& iy) {
  ix = x * 0.997f + 23.3f;   // smooth, homography-like
  iy = y * 1.001f + 0.37f;
}

__global__ void v1(const float* __restrict__ src, float* __restrict__ out) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= H * W) return;
  float ix, iy; pos(p % W, p / W, ix, iy);
  int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  float wx = ix - x0, wy = iy - y0;
  bool okx0 = x0 >= 0 && x0 < W, okx1 = x0 + 1 >= 0 && x0 + 1 < W, oky0 = y0 >= 0 && y0 < H, oky1 = y0 + 1 >= 0 && y0 + 1 < H;
  int i00 = (okx0 && oky0) ? y0 * W + x0 : 0, i01 = (okx1 && oky0) ? y0 * W + x0 + 1 : 0;
  int i10 = (okx0 && oky1) ? (y0 + 1) * W + x0 : 0, i11 = (okx1 && oky1) ? (y0 + 1) * W + x0 + 1 : 0;
  float acc = 0.f;
#pragma unroll 8
  for (int c = 0; c < C; ++c) {
    const float* s = src + (size_t)c * H * W;
    float v = s[i00] * (1 - wx) * (1 - wy) + s[i01] * wx * (1 - wy) + s[i10] * (1 - wx) * wy + s[i11] * wx * wy;
    acc += v * v;
  }
  out[p] = acc;
}

__global__ void v2(const float4* __restrict__ src, float* __restrict__ out) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= H * W) return;
  float ix, iy; pos(p % W, p / W, ix, iy);
  int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  float wx = ix - x0, wy = iy - y0;
  x0 = min(max(x0, 0), W - 2); y0 = min(max(y0, 0), H - 2);
  const float4* a = src + ((size_t)y0 * W + x0) * 8;
  const float4* b = a + (size_t)W * 8;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float4 q00 = a[k], q01 = a[8 + k], q10 = b[k], q11 = b[8 + k];
    float w00 = (1 - wx) * (1 - wy), w01 = wx * (1 - wy), w10 = (1 - wx) * wy, w11 = wx * wy;
    float4 v;
    v.x = q00.x * w00 + q01.x * w01 + q10.x * w10 + q11.x * w11;
    v.y = q00.y * w00 + q01.y * w01 + q10.y * w10 + q11.y * w11;
    v.z = q00.z * w00 + q01.z * w01 + q10.z * w10 + q11.z * w11;
    v.w = q00.w * w00 + q01.w * w01 + q10.w * w10 + q11.w * w11;
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  out[p] = acc;
}

__global__ void v3(const float4* __restrict__ src, float* __restrict__ out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  int p = t >> 3, k = t & 7;
  if (p >= H * W) return;
  float ix, iy; pos(p % W, p / W, ix, iy);
  int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  float wx = ix - x0, wy = iy - y0;
  x0 = min(max(x0, 0), W - 2); y0 = min(max(y0, 0), H - 2);
  const float4* a = src + ((size_t)y0 * W + x0) * 8 + k;
  const float4* b = a + (size_t)W * 8;
  float4 q00 = a[0], q01 = a[8], q10 = b[0], q11 = b[8];
  float w00 = (1 - wx) * (1 - wy), w01 = wx * (1 - wy), w10 = (1 - wx) * wy, w11 = wx * wy;
  float4 v;
  v.x = q00.x * w00 + q01.x * w01 + q10.x * w10 + q11.x * w11;
  v.y = q00.y * w00 + q01.y * w01 + q10.y * w10 + q11.y * w11;
  v.z = q00.z * w00 + q01.z * w01 + q10.z * w10 + q11.z * w11;
  v.w = q00.w * w00 + q01.w * w01 + q10.w * w10 + q11.w * w11;
  float acc = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  acc += __shfl_xor(acc, 1); acc += __shfl_xor(acc, 2); acc += __shfl_xor(acc, 4);
  if (k == 0) out[p] = acc;
}

int main() {
  size_t n = (size_t)C * H * W;
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  float *src, *out;
  CK(hipMalloc(&src, n * 4)); CK(hipMalloc(&out, (size_t)H * W * 4));
  CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 20;
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= R;
    printf("%-40s %8.3f ms  %7.1f GB/s (src bytes once)\n", name, ms, n * 4 / ms / 1e6);
  };
  int px = H * W;
  run("V1 NCHW dword thread/pixel", [&] { hipLaunchKernelGGL(v1, dim3((px + 255) / 256), dim3(256), 0, 0, src, out); });
  run("V2 NHWC dwordx4 thread/pixel", [&] { hipLaunchKernelGGL(v2, dim3((px + 255) / 256), dim3(256), 0, 0, (const float4*)src, out); });
  run("V3 NHWC dwordx4 8 lanes/pixel", [&] { hipLaunchKernelGGL(v3, dim3((px * 8 + 255) / 256), dim3(256), 0, 0, (const float4*)src, out); });
  CK(hipGetLastError());
  return 0;
}
