// Diagnostic harness (round 6): why a training cell costs more per pixel than an inference
// cell.  Cell 0 (the double-buffered kernel, the library's config) at config 4's 640x512 and at
// the headline's 1600x1184, in four forms: inference (fast gates, one accumulator), the
// training kernel (PRECISE: sign-balanced accumulator pair, unbiased gates) without and with
// the gate pre-activation record (z_out, 256 B per pixel), and PRECISE with the gate math
// ablated.  Random NHWC inputs; weights as in cell_bench.  Not shipped.
#include "../../aa-rmvsnet_amd/csrc/convlstm.hip"

#include <cstdio>
#include <vector>

using namespace aarmvs;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float* rnd_buf(size_t n, float scale) {
  std::vector<float> h(n);
  uint32_t st = (uint32_t)n * 2654435761u + 7;
  for (auto& x : h) { st = st * 1664525u + 1013904223u; x = scale * (((st >> 8) & 0xFFFF) / 65536.0f - 0.5f); }
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

int main() {
  _Float16* wh;
  {
    std::vector<_Float16> hh(2 * 3 * 9 * 2 * 64 * 8);
    uint32_t st = 99;
    for (auto& x : hh) { st = st * 1664525u + 1013904223u; x = (_Float16)(((st >> 8) & 0xFFFF) / 65536.0f * 20.f - 10.f); }
    CK(hipMalloc(&wh, hh.size() * 2)); CK(hipMemcpy(wh, hh.data(), hh.size() * 2, hipMemcpyHostToDevice));
  }
  float* invs = rnd_buf(1, 0.f);
  { float v = 1.0f / 1024; CK(hipMemcpy(invs, &v, 4, hipMemcpyHostToDevice)); }
  float* bias = rnd_buf(64, 0.1f);
  unsigned* xb; CK(hipMalloc(&xb, 4));
  { const float v = 16.0f; CK(hipMemcpy(xb, &v, 4, hipMemcpyHostToDevice)); }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int cu = cu_count();
  const int geo[2][2] = {{512, 640}, {1184, 1600}};
  for (const auto& g : geo) {
    const int H = g[0], W = g[1];
    const size_t HW = (size_t)H * W;
    float* x32 = rnd_buf(32 * HW, 4.f);
    float* f16a = rnd_buf(16 * HW, 2.f);
    float* hout = rnd_buf(16 * HW, 1.f);
    float* cst = rnd_buf(16 * HW, 1.f);
    float* z; CK(hipMalloc(&z, 64 * HW * 4));
    CellArgs a{};
    a.B = 1; a.H = H; a.W = W;
    a.h_new = hout; a.c = cst; a.c_in = cst; a.wpk = reinterpret_cast<const float*>(wh); a.bias = bias;
    a.part[0] = {x32, 32, SRC_PLAIN, nullptr, nullptr, nullptr};
    a.part[1] = {f16a, 16, SRC_PLAIN, nullptr, nullptr, nullptr};
    a.nparts = 2;
    a.xbound = xb;
    auto run = [&](const char* name, auto fn) {
      for (int i = 0; i < 2; ++i) CK(fn());
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      const int R = 20;
      for (int i = 0; i < R; ++i) CK(fn());
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= R;
      printf("%4dx%-4d %-44s %8.1f us  %6.3f ns/px\n", W, H, name, ms * 1e3, ms * 1e6 / HW);
    };
    CellArgs az = a;
    az.z_out = z;
    run("inference (fast gates)", [&] { return run_cell_h3_<0, 1, 8, 0, 1, 1, false>(a, invs, cu, K_CELL0, 0); });
    run("PRECISE, no record", [&] { return run_cell_h3_<0, 1, 8, 0, 1, 1, true>(a, invs, cu, K_CELL0, 0); });
    run("PRECISE + z record (the training cell)", [&] { return run_cell_h3_<0, 1, 8, 0, 1, 1, true>(az, invs, cu, K_CELL0, 0); });
    run("PRECISE, gate math ablated (4)", [&] { return run_cell_h3_<0, 1, 8, 4, 1, 1, true>(a, invs, cu, K_CELL0, 0); });
    run("inference, gate math ablated (4)", [&] { return run_cell_h3_<0, 1, 8, 4, 1, 1, false>(a, invs, cu, K_CELL0, 0); });
    run("PRECISE, no MFMA (1)", [&] { return run_cell_h3_<0, 1, 8, 1, 1, 1, true>(a, invs, cu, K_CELL0, 0); });
    run("inference, no MFMA (1)", [&] { return run_cell_h3_<0, 1, 8, 1, 1, 1, false>(a, invs, cu, K_CELL0, 0); });
    CK(hipFree(x32)); CK(hipFree(f16a)); CK(hipFree(hout)); CK(hipFree(cst)); CK(hipFree(z));
  }
  return 0;
}
