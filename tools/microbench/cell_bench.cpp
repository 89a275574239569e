// Diagnostic harness: times the ConvLSTM cell kernels at the headline geometry
// (1600x1184) for the library's tile configs and experimental variants (CellDef
// specialisations >= 10 defined here).  Not shipped.
#include "../../aa-rmvsnet_amd/csrc/convlstm.hip"

#include <cstdio>
#include <vector>

namespace aarmvs {
// variants: same parts as the base kind, other tile shapes
template <> struct CellDef<10> : CellDef<0> { static constexpr int TH = 4, NT = 1; };
template <> struct CellDef<14> : CellDef<4> { static constexpr int TH = 4, NT = 1; };
template <> struct CellDef<24> : CellDef<4> { static constexpr int TH = 16, NT = 1; };
template <> struct CellDef<34> : CellDef<4> { static constexpr int TH = 8, NT = 2; };
template <> struct CellDef<11> : CellDef<1> { static constexpr int TH = 4, NT = 1; };
}  // namespace aarmvs

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
  const int H = 1184, W = 1600, B = 1;
  const size_t HW = (size_t)H * W;
  float* x32 = rnd_buf(32 * HW, 4.f);
  float* f16a = rnd_buf(16 * HW, 2.f);
  float* f16b = rnd_buf(16 * HW, 2.f);
  float* f8 = rnd_buf(8 * HW, 2.f);
  float* hout = rnd_buf(16 * HW, 1.f);
  float* cst = rnd_buf(16 * HW, 1.f);
  float* wts = rnd_buf(64 * 48 * 9, 0.1f);
  float* bias = rnd_buf(64, 0.1f);
  float* gamma = rnd_buf(16, 1.f);
  double* stats; CK(hipMalloc(&stats, 4 * kSlots * 2 * 8)); CK(hipMemset(stats, 0, 4 * kSlots * 2 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto args = [&](int kind, int scale) {
    CellArgs a{};
    a.B = B; a.H = H / scale; a.W = W / scale;
    a.h_new = hout; a.c = cst; a.wpk = wts; a.bias = bias;
    if (kind == 0) { a.part[0] = {x32, 32, SRC_PLAIN, nullptr, nullptr, nullptr}; a.part[1] = {f16a, 16, SRC_PLAIN, nullptr, nullptr, nullptr}; a.nparts = 2; }
    if (kind == 1) { a.part[0] = {f16a, 16, SRC_POOL, nullptr, nullptr, nullptr}; a.part[1] = {f16b, 16, SRC_PLAIN, nullptr, nullptr, nullptr}; a.nparts = 2; }
    if (kind == 3 || kind == 4) {
      a.part[0] = {f16a, 16, SRC_GNRELU, stats, gamma, gamma};
      a.part[1] = {f16b, 16, SRC_PLAIN, nullptr, nullptr, nullptr};
      a.part[2] = {kind == 4 ? f8 : x32, kind == 4 ? 8 : 16, SRC_PLAIN, nullptr, nullptr, nullptr};
      a.nparts = 3;
    }
    return a;
  };
  auto run = [&](const char* name, auto fn, double flops) {
    for (int i = 0; i < 2; ++i) CK(fn());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 10;
    for (int i = 0; i < R; ++i) CK(fn());
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= R;
    printf("%-34s %8.3f ms  %7.1f TFLOP/s\n", name, ms, flops / ms / 1e9);
  };
  const double fl0 = 2.0 * 9 * 48 * 64 * HW, fl1 = 2.0 * 9 * 32 * 64 * HW / 4, fl3 = 2.0 * 9 * 48 * 64 * HW / 4,
               fl4 = 2.0 * 9 * 40 * 32 * HW;
  run("cell0 (TH4 NT1)", [&] { return run_cell<0>(args(0, 1), 256, K_CELL0, 0); }, fl0);
  run("cell1 (TH8 NT1)", [&] { return run_cell<1>(args(1, 2), 256, K_CELL1, 0); }, fl1);
  run("cell1 var TH4", [&] { return run_cell<11>(args(1, 2), 256, K_CELL1, 0); }, fl1);
  run("cell3 (TH4 NT1)", [&] { return run_cell<3>(args(3, 2), 256, K_CELL3, 0); }, fl3);
  run("cell4 (TH8 NT1)", [&] { return run_cell<4>(args(4, 1), 256, K_CELL4, 0); }, fl4);
  run("cell4 var TH4 NT1", [&] { return run_cell<14>(args(4, 1), 256, K_CELL4, 0); }, fl4);
  run("cell4 var TH16 NT1", [&] { return run_cell<24>(args(4, 1), 256, K_CELL4, 0); }, fl4);
  run("cell4 var TH8 NT2", [&] { return run_cell<34>(args(4, 1), 256, K_CELL4, 0); }, fl4);
  return 0;
}
