// Diagnostic harness: times the cost-slice pipeline kernels (cost_x, omega_conv) at the
// headline geometry (1600x1184, 6 source views).  Includes the kernel source; links
// libaarmvs.so for the parameter layout / workspace carve.  Not shipped; numbers are
// for design decisions.
#include "../../aa-rmvsnet_amd/csrc/warp_cost.hip"

#include <cstdio>
#include <vector>

using namespace aarmvs;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int B = 1, H = 1184, W = 1600, nsrc = 6, D = 4;
  const size_t HW = (size_t)H * W, fn = (size_t)kC * HW;
  std::vector<float> h(fn);
  uint32_t st = 1;
  auto rnd = [&] { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xFFFF) / 65536.0f - 0.5f; };
  float* feats[7];
  for (int v = 0; v < 7; ++v) {
    for (size_t i = 0; i < fn; ++i) h[i] = rnd();
    CK(hipMalloc(&feats[v], fn * 4));
    CK(hipMemcpy(feats[v], h.data(), fn * 4, hipMemcpyHostToDevice));
  }
  // cameras as in aarmvs.synthetic: f = W, baseline -20 mm * v, small yaw
  std::vector<float> rel(nsrc * B * 12);
  for (int v = 0; v < nsrc; ++v) {
    float th = 0.02f * (v + 1) * ((v + 1) % 2 ? 1 : -1);
    float f = W, cx = W / 2.f, cy = H / 2.f;
    // rel = K [R|t] K^-1 (ref = identity), rows 0..2
    float R[3][3] = {{cosf(th), 0, sinf(th)}, {0, 1, 0}, {-sinf(th), 0, cosf(th)}};
    float t[3] = {-20.f * (v + 1), 0.3f * (v + 1), 0};
    float Ki[3][3] = {{1 / f, 0, -cx / f}, {0, 1 / f, -cy / f}, {0, 0, 1}};
    float K[3][3] = {{f, 0, cx}, {0, f, cy}, {0, 0, 1}};
    float KR[3][3], M[3][3], Kt[3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) { KR[i][j] = 0; for (int k = 0; k < 3; ++k) KR[i][j] += K[i][k] * R[k][j]; }
    for (int i = 0; i < 3; ++i) {
      Kt[i] = 0; for (int k = 0; k < 3; ++k) Kt[i] += K[i][k] * t[k];
      for (int j = 0; j < 3; ++j) { M[i][j] = 0; for (int k = 0; k < 3; ++k) M[i][j] += KR[i][k] * Ki[k][j]; }
    }
    for (int i = 0; i < 3; ++i) { for (int j = 0; j < 3; ++j) rel[v * 12 + i * 4 + j] = M[i][j]; rel[v * 12 + i * 4 + 3] = Kt[i]; }
  }
  float *drel, *ddv, *dpar;
  CK(hipMalloc(&drel, rel.size() * 4)); CK(hipMemcpy(drel, rel.data(), rel.size() * 4, hipMemcpyHostToDevice));
  float dvh[D] = {600.f, 601.f, 602.f, 603.f};
  CK(hipMalloc(&ddv, sizeof(dvh))); CK(hipMemcpy(ddv, dvh, sizeof(dvh), hipMemcpyHostToDevice));
  size_t pb = aarmvs_packed_param_bytes();
  std::vector<float> ph(pb / 4);
  for (auto& x : ph) x = 0.1f * rnd();
  CK(hipMalloc(&dpar, pb)); CK(hipMemcpy(dpar, ph.data(), pb, hipMemcpyHostToDevice));
  size_t wsb = aarmvs_sweep_workspace_bytes(B, H, W, nsrc);
  void* wsp; CK(hipMalloc(&wsp, wsb)); CK(hipMemset(wsp, 0, wsb));
  Workspace ws = carve_workspace(wsp, B, H, W, nsrc);
  SweepGeom g{B, H, W, nsrc, D, 256};
  CostArgs ca{};
  ca.ref = feats[0];
  for (int v = 0; v < nsrc; ++v) ca.src[v] = feats[v + 1];
  ca.rel = drel; ca.depth_values = ddv; ca.params = dpar;
  CK(launch_to_c8(feats[0], ws.feat8[0], B, (int)HW, 0));
  for (int v = 0; v < nsrc; ++v) CK(launch_to_c8(feats[v + 1], ws.feat8[v + 1], B, (int)HW, 0));
  CK(launch_omega_next(ca, g, ws, 0, 0));
  CK(hipDeviceSynchronize());
  PipeArgs a0 = pipe_args(ca, g, ws);
  a0.d_prev = 0; a0.d_next = 1;
  a0.ref = ws.feat8[0];
  for (int v = 0; v < nsrc; ++v) a0.src[v] = ws.feat8[v + 1];
  a0.t1_prev = reinterpret_cast<const float4*>(ws.t1[0]); a0.st_prev = ws.omega_stats[0];
  a0.t1_next = reinterpret_cast<float4*>(ws.t1[1]); a0.st_next = ws.omega_stats[1];
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int tiles_x = (W + kTileW - 1) / kTileW;
  auto run = [&](const char* name, auto kern, dim3 grid, int threads, double bytes) {
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, grid, dim3(threads), 0, 0, a0, dpar, drel);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 10;
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(kern, grid, dim3(threads), 0, 0, a0, dpar, drel);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-36s %8.3f ms  %7.0f GB/s algorithmic\n", name, ms / R, bytes / (ms / R) / 1e6);
  };
  const dim3 gx(tiles_x * ((H + kXRows - 1) / kXRows), B);
  const double bx = 128.0 * (nsrc + 2) * HW;
  run("cost_x", cost_x_kernel<0>, gx, 2 * kXRows * kTileW, bx);
  run("cost_x pair sample_pos (1)", cost_x_kernel<1>, gx, 2 * kXRows * kTileW, bx);
  run("cost_x pair omega (2)", cost_x_kernel<2>, gx, 2 * kXRows * kTileW, bx);
  run("cost_x pair both (3)", cost_x_kernel<3>, gx, 2 * kXRows * kTileW, bx);
  run("cost_x pair omega, 5 waves/SIMD (6)", cost_x_kernel<6>, gx, 2 * kXRows * kTileW, bx);
  run("cost_x pair omega, 6 waves/SIMD (10)", cost_x_kernel<10>, gx, 2 * kXRows * kTileW, bx);
  const dim3 gc(tiles_x * ((H + kTileH - 1) / kTileH) * nsrc, 1, B);
  const double bc = (128.0 * (nsrc + 1) + 16.0 * nsrc) * HW;
  run("omega_conv", omega_conv_kernel<0>, gc, kTileThreads, bc);
  run("omega_conv no conv (1)", omega_conv_kernel<1>, gc, kTileThreads, bc);
  run("omega_conv no sq (2)", omega_conv_kernel<2>, gc, kTileThreads, bc);
  run("omega_conv no box loads (4)", omega_conv_kernel<4>, gc, kTileThreads, bc);
  run("omega_conv no sq/box (6)", omega_conv_kernel<6>, gc, kTileThreads, bc);
  run("omega_conv skeleton (7)", omega_conv_kernel<7>, gc, kTileThreads, bc);
  run("omega_conv MFMA off-centre taps (16)", omega_conv_kernel<16>, gc, kTileThreads, bc);
  run("omega_conv conv rolled (8)", omega_conv_kernel<8>, gc, kTileThreads, bc);
  a0.box_cap = 64;
  run("omega_conv (box cap 64: global gathers)", omega_conv_kernel<0>, gc, kTileThreads, bc);
  {
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) CK(launch_to_c8(feats[0], ws.feat8[0], B, (int)HW, 0));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-36s %8.3f ms (%.0f GB/s)\n", "to_c8 one view", ms / 10, 2.0 * fn * 4 / (ms / 10) / 1e6);
  }
  CK(hipGetLastError());
  return 0;
}
