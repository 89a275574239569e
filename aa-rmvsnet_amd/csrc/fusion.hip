// Depth-map fusion core (fusion.py:71-220) for gfx950: per reference pixel, the geometric
// consistency against every source view's depth map (reproject_with_depth +
// check_geometric_consistency) and filter_depth's vote / mask / averaged-depth logic, in
// one pass (one thread per reference pixel, the source views in a loop).
//
// Arithmetic follows the reference's numpy types: projections in float64 on the float32
// camera matrices (the host packs them exactly as numpy forms them: float32 inverses and
// float32 matrix products), the maps, the reprojected depth and coordinates rounded to
// float32 where the reference casts, cv2.remap's INTER_LINEAR as OpenCV computes it for
// float maps (coordinates rounded to 1/32 px, table weights, left-to-right float32 sum,
// out-of-image taps 0), relative depth differences and depth sums in float32.
// Algorithmic bytes per reference pixel: depth + confidence (8) + one depth read per source
// view (4 nsrc) + three masks and the float64 average (11).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "aarmvs_internal.h"

namespace aarmvs {

struct FusionArgs {
  int H, W, nsrc;
  const float* ref_depth;
  const float* confidence;
  const float* src_depth[AARMVS_MAX_FUSION_SRC];
  float cams[AARMVS_FUSION_CAM_FLOATS(AARMVS_MAX_FUSION_SRC)];
  float photo_threshold;
  unsigned char* photo_mask;
  unsigned char* geo_mask;
  unsigned char* final_mask;
  double* depth_avg;
};

// rows r of a row-major float32 matrix (columns cols) times a float64 vector, as numpy's
// float64 matmul of the up-cast matrix (an fma chain over k)
template <int COLS>
__device__ __forceinline__ double mrow(const float* m, int r, const double (&v)[COLS]) {
  double s = (double)m[r * COLS] * v[0];
#pragma unroll
  for (int k = 1; k < COLS; ++k) s = fma((double)m[r * COLS + k], v[k], s);
  return s;
}

// cv2.remap(src, map_x, map_y, INTER_LINEAR) at one pixel (BORDER_CONSTANT 0)
__device__ __forceinline__ float remap_linear(const float* __restrict__ src, int H, int W, float mx,
                                              float my) {
  auto to_fixed = [](float v) -> long long {
    const float t = __fmul_rn(v, 32.0f);
    // cvRound: nearest, ties to even; non-finite / out-of-int range -> INT_MIN (outside)
    if (!(fabsf(t) < 2147483520.0f)) return -2147483648LL;
    return (long long)rintf(t);
  };
  const long long X = to_fixed(mx), Y = to_fixed(my);
  const long long sx = X >> 5, sy = Y >> 5;
  const float fx = (float)(X & 31) * (1.0f / 32.0f), fy = (float)(Y & 31) * (1.0f / 32.0f);
  const float cx0 = __fsub_rn(1.0f, fx), cy0 = __fsub_rn(1.0f, fy);
  const float w0 = __fmul_rn(cy0, cx0), w1 = __fmul_rn(cy0, fx), w2 = __fmul_rn(fy, cx0),
              w3 = __fmul_rn(fy, fx);
  auto tap = [&](long long yy, long long xx) {
    return (xx >= 0 && xx < W && yy >= 0 && yy < H) ? src[yy * W + xx] : 0.0f;
  };
  float r = __fmul_rn(tap(sy, sx), w0);
  r = __fadd_rn(r, __fmul_rn(tap(sy, sx + 1), w1));
  r = __fadd_rn(r, __fmul_rn(tap(sy + 1, sx), w2));
  r = __fadd_rn(r, __fmul_rn(tap(sy + 1, sx + 1), w3));
  return r;
}

__global__ void __launch_bounds__(256) fusion_filter_kernel(FusionArgs a) {
  const int H = a.H, W = a.W, nsrc = a.nsrc, n = nsrc + 1;
  // cams: invK_ref[9], K_ref[9], then per source view K[9], invK[9], M1[12] = (E_src
  // inv(E_ref))[:3], M2[12] = (E_ref inv(E_src))[:3]
  const float* invK_ref = a.cams;
  const float* K_ref = a.cams + 9;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < H * W; p += gridDim.x * blockDim.x) {
    const int y = p / W, x = p - y * W;
    const float dref = a.ref_depth[p];
    const double dd = (double)dref;
    const double b0[3] = {(double)x * dd, (double)y * dd, dd};
    const double xr[4] = {mrow<3>(invK_ref, 0, b0), mrow<3>(invK_ref, 1, b0), mrow<3>(invK_ref, 2, b0),
                          1.0};
    int votes[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int geo_sum = 0;
    float depth_sum = 0.0f;
    for (int v = 0; v < nsrc; ++v) {
      const float* c = a.cams + 18 + 42 * v;
      const float *K = c, *invK = c + 9, *M1 = c + 18, *M2 = c + 30;
      // step 1: reference pixel -> source view (fusion.py:75-87)
      const double xs3[3] = {mrow<4>(M1, 0, xr), mrow<4>(M1, 1, xr), mrow<4>(M1, 2, xr)};
      const double kx = mrow<3>(K, 0, xs3), ky = mrow<3>(K, 1, xs3), kz = mrow<3>(K, 2, xs3);
      const double xsrc = kx / kz, ysrc = ky / kz;
      // step 2: source depth at that point, back to the reference view (:89-108)
      const float sampled = remap_linear(a.src_depth[v], H, W, (float)xsrc, (float)ysrc);
      const double sd = (double)sampled;
      const double b2[3] = {xsrc * sd, ysrc * sd, sd};
      const double xs2[4] = {mrow<3>(invK, 0, b2), mrow<3>(invK, 1, b2), mrow<3>(invK, 2, b2), 1.0};
      const double xq[3] = {mrow<4>(M2, 0, xs2), mrow<4>(M2, 1, xs2), mrow<4>(M2, 2, xs2)};
      float depth_rep = (float)xq[2];
      const double qx = mrow<3>(K_ref, 0, xq), qy = mrow<3>(K_ref, 1, xq), qz = mrow<3>(K_ref, 2, xq);
      const float xrep = (float)(qx / qz), yrep = (float)(qy / qz);
      // check_geometric_consistency (:117-131)
      const double ex = (double)xrep - (double)x, ey = (double)yrep - (double)y;
      const double dist = sqrt(ex * ex + ey * ey);
      const float rel = __fdiv_rn(fabsf(__fsub_rn(depth_rep, dref)), dref);
      bool m = false;
#pragma unroll
      for (int i = 2; i <= 10; ++i) {
        m = dist < (double)i / 4.0 && rel < (float)((double)i / 1300.0);
        if (i < n) votes[i - 2] += m ? 1 : 0;   // filter_depth counts masks[0 .. n-3]
      }
      if (!m) depth_rep = 0.0f;   // depth_reprojected[~mask] = 0 (mask: i = 10)
      geo_sum += m ? 1 : 0;
      depth_sum = __fadd_rn(depth_sum, depth_rep);
    }
    // filter_depth (:207-220)
    bool geo = geo_sum >= n;
#pragma unroll
    for (int i = 2; i <= 10; ++i)
      if (i < n) geo = geo || votes[i - 2] >= i;
    const bool photo = a.confidence[p] > a.photo_threshold;
    a.photo_mask[p] = photo ? 1 : 0;
    a.geo_mask[p] = geo ? 1 : 0;
    a.final_mask[p] = (photo && geo) ? 1 : 0;
    a.depth_avg[p] = (double)__fadd_rn(depth_sum, dref) / (double)(geo_sum + 1);
  }
}

hipError_t launch_fusion_filter(const aarmvs_fusion_args* in, hipStream_t s) {
  FusionArgs a{};
  a.H = in->H;
  a.W = in->W;
  a.nsrc = in->nsrc;
  a.ref_depth = in->ref_depth;
  a.confidence = in->confidence;
  for (int v = 0; v < in->nsrc; ++v) a.src_depth[v] = in->src_depth[v];
  for (int i = 0; i < AARMVS_FUSION_CAM_FLOATS(in->nsrc); ++i) a.cams[i] = in->cams[i];
  a.photo_threshold = in->photo_threshold;
  a.photo_mask = in->photo_mask;
  a.geo_mask = in->geo_mask;
  a.final_mask = in->final_mask;
  a.depth_avg = in->depth_avg;
  const int HW = a.H * a.W;
  const int blocks = std::max(1, std::min((HW + 255) / 256, 65535));
  ProfScope ps(s, K_FUSION);
  hipLaunchKernelGGL(fusion_filter_kernel, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace aarmvs
