// Diagnostic harness: times the cost-slice pipeline kernels (cost_x, omega_conv) at the
// headline geometry (1600x1184, 6 source views).  Includes the kernel source; links
// libaarmvs.so for the parameter layout / workspace carve.  Not shipped; numbers are
// for design decisions.
#include "../../aa-rmvsnet_amd/csrc/warp_cost.hip"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace aarmvs;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int B = 1, H = 1184, W = 1600, nsrc = 6, D = 16;
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
  float dvh[D];
  for (int d = 0; d < D; ++d) dvh[d] = 600.f + d;
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
  CK(launch_omega_group(ca, g, ws, 0, 1, 0));
  CK(hipDeviceSynchronize());
  PipeArgs a0 = pipe_args(ca, g, ws);
  a0.part = ws.omega_part; a0.part_n = ws.omega_part_n;   // GN partials (npl <= kPlaneGroup)
  a0.d_prev = 0; a0.d_next = 1;
  a0.ref = ws.feat8[0];
  for (int v = 0; v < nsrc; ++v) a0.src[v] = ws.feat8[v + 1];
  a0.t1_prev = reinterpret_cast<const float4*>(ws.t1); a0.st_prev = ws.omega_stats;
  a0.t1_next = nullptr; a0.st_next = nullptr;
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
  // omega_mfma ablations at npl = 8 (tools: what bounds the kernel)
  auto ablate = [&](const char* name, auto kern, float4* t1o, double* sto) {
    PipeArgs a = a0;
    a.npl = 8; a.t1_kstride = (size_t)B * nsrc * HW; a.st_kstride = ws.omega_stats_bytes / 8;
    a.d_next = 1; a.t1_next = t1o; a.st_next = sto;
    const int ntm = OmegaTile<16>::tiles(H, W);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, dim3(ntm * nsrc * 8, 1, B), dim3(OmegaTile<16>::NT), 0, 0, a, dpar, drel, ws.xbound);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(ntm * nsrc * 8, 1, B), dim3(OmegaTile<16>::NT), 0, 0, a, dpar, drel, ws.xbound);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("omega_mfma npl=8 %-34s %8.3f ms/plane\n", name, ms / 5 / 8);
  };
  // plane batching: one launch over npl planes (per-plane time = launch / npl)
  const size_t t1k = (size_t)B * nsrc * HW, stk = ws.omega_stats_bytes / 8, xk = (size_t)B * kC * HW;
  float4* t1b; double* stb; float* xb;
  CK(hipMalloc(&t1b, 8 * t1k * 16)); CK(hipMalloc(&stb, 8 * stk * 8)); CK(hipMalloc(&xb, 8 * xk * 4));
  CK(hipMemset(stb, 0, 8 * stk * 8));
  const int ntm = OmegaTile<16>::tiles(H, W);
  const double bc = (128.0 * (nsrc + 1) + 16.0 * nsrc) * HW;
  const double bx = 128.0 * (nsrc + 2) * HW;
  for (int npl : {1, 2, 4, 8}) {
    PipeArgs a = a0;
    a.npl = npl; a.t1_kstride = t1k; a.st_kstride = stk; a.x_kstride = xk;
    a.d_next = 1; a.t1_next = t1b; a.st_next = stb;
    auto om = [&] { hipLaunchKernelGGL((omega_mfma_kernel<0, 16>), dim3(ntm * nsrc * npl, 1, B), dim3(OmegaTile<16>::NT), 0, 0, a, dpar, drel, ws.xbound); };
    for (int i = 0; i < 2; ++i) om();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) om();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("omega_mfma npl=%d  %8.3f ms/plane  %7.0f GB/s algorithmic\n", npl, ms / 10 / npl, bc * npl / (ms / 10) / 1e6);
    if (npl == 8) {
      ablate("default (0)", omega_mfma_kernel<0, 16>, t1b, stb);
      ablate("no MFMA (1)", omega_mfma_kernel<1, 16>, t1b, stb);
      ablate("no box DMA (2)", omega_mfma_kernel<2, 16>, t1b, stb);
      ablate("no sampling (4)", omega_mfma_kernel<4, 16>, t1b, stb);
      ablate("no ref loads (8)", omega_mfma_kernel<8, 16>, t1b, stb);
      ablate("no divisions (16)", omega_mfma_kernel<16, 16>, t1b, stb);
      ablate("no DMA, no sampling (6)", omega_mfma_kernel<6, 16>, t1b, stb);
      ablate("no DMA/sampling/MFMA/ref (15)", omega_mfma_kernel<15, 16>, t1b, stb);
      ablate("skeleton (31)", omega_mfma_kernel<31, 16>, t1b, stb);
      ablate("skeleton, no Y image (63)", omega_mfma_kernel<63, 16>, t1b, stb);
      ablate("skeleton, no stats atomics (95)", omega_mfma_kernel<95, 16>, t1b, stb);
      ablate("skeleton, no B loads (159)", omega_mfma_kernel<159, 16>, t1b, stb);
      ablate("skeleton - Y/atomics/B (255)", omega_mfma_kernel<255, 16>, t1b, stb);
      ablate("no Y image (32)", omega_mfma_kernel<32, 16>, t1b, stb);
      ablate("no B loads (128)", omega_mfma_kernel<128, 16>, t1b, stb);
    }
    // plane npl-1 must equal a single-plane launch at d_next = npl
    if (npl > 1) {
      std::vector<float4> hb(t1k), hs(t1k);
      CK(hipMemcpy(hb.data(), t1b + (npl - 1) * t1k, t1k * 16, hipMemcpyDeviceToHost));
      PipeArgs a1 = a; a1.npl = 1; a1.d_next = npl;
      hipLaunchKernelGGL((omega_mfma_kernel<0, 16>), dim3(ntm * nsrc, 1, B), dim3(OmegaTile<16>::NT), 0, 0, a1, dpar, drel, ws.xbound);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hs.data(), t1b, t1k * 16, hipMemcpyDeviceToHost));
      printf("  plane %d vs single launch: %s\n", npl - 1, memcmp(hb.data(), hs.data(), t1k * 16) ? "DIFFERENT" : "identical");
    }
    PipeArgs c = a0;
    c.npl = npl; c.t1_kstride = 0; c.st_kstride = 0; c.x_kstride = xk; c.x = xb; c.omega_k = -1;
    auto cx = [&] { hipLaunchKernelGGL(cost_x_kernel<2>, dim3(tiles_x * ((H + kXRows - 1) / kXRows) * npl, B), dim3(2 * kXRows * kTileW), 0, 0, c, dpar, drel); };
    for (int i = 0; i < 2; ++i) cx();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) cx();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("cost_x npl=%d      %8.3f ms/plane  %7.0f GB/s algorithmic\n", npl, ms / 10 / npl, bx * npl / (ms / 10) / 1e6);
    if (npl == 8) {
      auto c4 = [&] { hipLaunchKernelGGL((cost_x_kernel<2, 4>), dim3(tiles_x * ((H + 3) / 4) * npl, B), dim3(2 * 4 * kTileW), 0, 0, c, dpar, drel); };
      for (int i = 0; i < 2; ++i) c4();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) c4();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("cost_x npl=8 4-row tiles (256 threads) %8.3f ms/plane\n", ms / 10 / npl);
      // co-running: omega_mfma (the library's 16x16 tiles) on one stream and cost_x (4-row
      // tiles) on another, independent buffers -- do the two kernels' limits (latency / L1
      // gathers) overlap on shared CUs?
      PipeArgs ao = a0;
      ao.npl = 8; ao.t1_kstride = t1k; ao.st_kstride = stk; ao.d_next = 1; ao.t1_next = t1b; ao.st_next = stb;
      const int nt16 = OmegaTile<16>::tiles(H, W);
      ao.part_n = nt16;
      hipStream_t s1, s2;
      CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
      CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      auto om16 = [&](hipStream_t st) { hipLaunchKernelGGL((omega_mfma_kernel<0, 16>), dim3(nt16 * nsrc * 8, 1, B), dim3(OmegaTile<16>::NT), 0, st, ao, dpar, drel, ws.xbound); };
      auto cx4 = [&](hipStream_t st) { hipLaunchKernelGGL((cost_x_kernel<2, 4>), dim3(tiles_x * ((H + 3) / 4) * npl, B), dim3(2 * 4 * kTileW), 0, st, c, dpar, drel); };
      auto timed = [&](const char* name, auto body) {
        body(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 5; ++i) body();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float mm; CK(hipEventElapsedTime(&mm, e0, e1));
        printf("corun %-40s %8.3f ms per (8-plane) launch pair\n", name, mm / 5);
      };
      timed("omega alone", [&] { om16(s1); });
      timed("cost_x alone", [&] { cx4(s2); });
      timed("omega then cost_x (one stream)", [&] { om16(s1); cx4(s1); });
      timed("omega || cost_x (two streams)", [&] { om16(s1); cx4(s2); });
      CK(hipStreamDestroy(s1)); CK(hipStreamDestroy(s2));
    }
  }
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
