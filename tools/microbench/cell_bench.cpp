// Diagnostic harness: times the ConvLSTM cell kernels at the headline geometry
// (1600x1184, NHWC inputs of random values) for the library's configs, the other buffer
// mode and the ablations.  Not shipped.
#include "../../aa-rmvsnet_amd/csrc/convlstm.hip"

#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
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
  // CB_H / CB_W: another geometry (e.g. config 1's 128 x 160), CB_SMALL=1: the library configs
  // and the cell-0 ablations only
  const int H = getenv("CB_H") ? atoi(getenv("CB_H")) : 1184, W = getenv("CB_W") ? atoi(getenv("CB_W")) : 1600, B = 1;
  const bool small = getenv("CB_SMALL") && atoi(getenv("CB_SMALL"));
  const size_t HW = (size_t)H * W;
  float* x32 = rnd_buf(32 * HW, 4.f);
  float* f16a = rnd_buf(16 * HW, 2.f);
  float* f16b = rnd_buf(16 * HW, 2.f);
  float* f8 = rnd_buf(8 * HW, 2.f);
  float* hout = rnd_buf(16 * HW, 1.f);
  float* cst = rnd_buf(16 * HW, 1.f);
  float* wts = rnd_buf(64 * 48 * 9, 0.1f);
  // split-fp16 weights (valid halves) for the h3 kernels + a scale
  _Float16* wh;
  {
    std::vector<_Float16> hh(2 * 3 * 9 * 2 * 64 * 8);
    uint32_t st = 99;
    for (auto& x : hh) { st = st * 1664525u + 1013904223u; x = (_Float16)(((st >> 8) & 0xFFFF) / 65536.0f * 20.f - 10.f); }
    CK(hipMalloc(&wh, hh.size() * 2)); CK(hipMemcpy(wh, hh.data(), hh.size() * 2, hipMemcpyHostToDevice));
  }
  float* invs = rnd_buf(1, 0.f);
  {
    float v = 1.0f / 1024; CK(hipMemcpy(invs, &v, 4, hipMemcpyHostToDevice));
  }
  float* bias = rnd_buf(64, 0.1f);
  float* gamma = rnd_buf(16, 1.f);
  double* stats; CK(hipMalloc(&stats, 4 * kSlots * 2 * 8)); CK(hipMemset(stats, 0, 4 * kSlots * 2 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto args = [&](int kind, int scale) {
    CellArgs a{};
    a.B = B; a.H = H / scale; a.W = W / scale;
    a.h_new = hout; a.c = cst; a.c_in = cst; a.wpk = wts; a.bias = bias;   // c updated in place, as the eval sweep does
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
  auto h3 = [&](CellArgs a) { a.wpk = reinterpret_cast<const float*>(wh); return a; };
  if (small) {
    {   // MS=2 against the library config: h and c bit-identical (fresh c for each)
      std::vector<float> c0(16 * HW), h1(16 * HW), h2(16 * HW), c1(16 * HW), c2(16 * HW);
      CK(hipMemcpy(c0.data(), cst, 16 * HW * 4, hipMemcpyDeviceToHost));
      auto once = [&](auto fn, std::vector<float>& ho, std::vector<float>& co) {
        CK(hipMemcpy(cst, c0.data(), 16 * HW * 4, hipMemcpyHostToDevice));
        CK(fn()); CK(hipDeviceSynchronize());
        CK(hipMemcpy(ho.data(), hout, 16 * HW * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(co.data(), cst, 16 * HW * 4, hipMemcpyDeviceToHost));
      };
      auto cmp = [&](const char* name, auto f1, auto f2, size_t n) {
        once(f1, h1, c1); once(f2, h2, c2);
        const bool same = !memcmp(h1.data(), h2.data(), n * 4) && !memcmp(c1.data(), c2.data(), n * 4);
        printf("  %s: MS2 vs library %s\n", name, same ? "bit-identical" : "DIFFERENT");
      };
      cmp("cell0", [&] { return run_cell_h3<0, 1, 8, 0, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); },
          [&] { return run_cell_h3<0, 1, 16, 0, 1, 1, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, 16 * HW);
      cmp("cell1", [&] { return run_cell_h3<1, 1, 8, 0, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); },
          [&] { return run_cell_h3<1, 1, 16, 0, 1, 1, 2>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, 16 * HW / 4);
      cmp("cell3", [&] { return run_cell_h3<3, 1, 8, 0, 1, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); },
          [&] { return run_cell_h3<3, 1, 16, 0, 1, 1, 2>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, 16 * HW / 4);
      CK(hipMemcpy(cst, c0.data(), 16 * HW * 4, hipMemcpyHostToDevice));
    }
    run("cell0 h3 DB1 PIPE1 (library)", [&] { return run_cell_h3<0, 1, 8, 0, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 DB1 no MFMA (1)", [&] { return run_cell_h3<0, 1, 8, 1, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 DB1 no staging (2)", [&] { return run_cell_h3<0, 1, 8, 2, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 DB1 no gates (4)", [&] { return run_cell_h3<0, 1, 8, 4, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 DB1 skeleton (7)", [&] { return run_cell_h3<0, 1, 8, 7, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 RW1 W4 DB1", [&] { return run_cell_h3<0, 1, 4, 0, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 W16 MS2 DB1 PIPE1", [&] { return run_cell_h3<0, 1, 16, 0, 1, 1, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 W16 MS2 DB1 PIPE0", [&] { return run_cell_h3<0, 1, 16, 0, 1, 0, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 W16 MS2 DB0 PIPE1", [&] { return run_cell_h3<0, 1, 16, 0, 0, 1, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell0 W8 MS2 DB1 PIPE1", [&] { return run_cell_h3<0, 1, 8, 0, 1, 1, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
    run("cell1 W16 MS2 DB1 PIPE1", [&] { return run_cell_h3<1, 1, 16, 0, 1, 1, 2>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
    run("cell1 W8 MS2 DB1 PIPE1", [&] { return run_cell_h3<1, 1, 8, 0, 1, 1, 2>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
    run("cell3 W16 MS2 DB1 PIPE1", [&] { return run_cell_h3<3, 1, 16, 0, 1, 1, 2>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
    run("cell3 W8 MS2 DB1 PIPE1", [&] { return run_cell_h3<3, 1, 8, 0, 1, 1, 2>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
    run("cell1 h3 DB1 PIPE1 (library)", [&] { return run_cell_h3<1, 1, 8, 0, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
    run("cell1 DB1 skeleton (7)", [&] { return run_cell_h3<1, 1, 8, 7, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
    run("cell3 h3 DB1 PIPE1 (library)", [&] { return run_cell_h3<3, 1, 8, 0, 1, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
    run("cell4 h3 DB0 PIPE0 (library)", [&] { return run_cell_h3<4, 1, 8, 0, 0, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
    run("cell4 DB0 skeleton (7)", [&] { return run_cell_h3<4, 1, 8, 7, 0, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
    return 0;
  }
  {
    const int Hi = H / 2, Wi = W / 2;
    const dim3 grid((Wi + kDpTW - 1) / kDpTW, (Hi + kDpTH - 1) / kDpTH, B);
    double* gp; CK(hipMalloc(&gp, (size_t)grid.x * grid.y * 4 * 8));
    const double fld = 2.0 * 16 * 16 * 9 * Hi * Wi;
    auto dc = [&](auto kern) { return [=] { hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, f16a, wts, bias, Hi, Wi, hout, gp); return hipGetLastError(); }; };
    // packed parameters from one random raw blob: dct (VALU) and dcm (MFMA) of deconv_1
    const ParamLayout& PL = param_layout();
    float* raw = rnd_buf(PL.raw_total, 0.2f);
    float* pk; CK(hipMalloc(&pk, PL.pk_total * 4));
    CK(launch_pack_params(raw, pk, 0));
    float* hin = rnd_buf(16 * HW / 4, 1.9f);   // |h| < 1 like the tanh outputs
    auto dv = [&](auto kern, const float* wp) { return [=] { hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, hin, wp, pk + PL.pk_off[P_D1B], Hi, Wi, hout, gp); return hipGetLastError(); }; };
    {
      const size_t no = (size_t)16 * 4 * Hi * Wi;
      std::vector<float> o1(no), o2(no);
      std::vector<double> g1((size_t)grid.x * grid.y * 4), g2(g1.size());
      CK(dv(deconv_px2_kernel<0>, pk + PL.dct_off[1])()); CK(hipDeviceSynchronize());
      CK(hipMemcpy(o1.data(), hout, no * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(g1.data(), gp, g1.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemset(hout, 0, no * 4));
      CK(dv(deconv_mfma_kernel<0>, pk + PL.dcm_off[1])()); CK(hipDeviceSynchronize());
      CK(hipMemcpy(o2.data(), hout, no * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(g2.data(), gp, g2.size() * 8, hipMemcpyDeviceToHost));
      double mx = 0, mref = 0, gs1 = 0, gs2 = 0;
      for (size_t i = 0; i < no; ++i) { mx = fmax(mx, fabs((double)o1[i] - o2[i])); mref = fmax(mref, fabs((double)o1[i])); }
      for (size_t i = 0; i < g1.size(); i += 4) { gs1 += g1[i]; gs2 += g2[i]; }
      printf("  deconv_mfma vs deconv_px2: max|diff| %.3g (max|out| %.3g), GN sum %.9g vs %.9g\n", mx, mref, gs1, gs2);
    }
    run("deconv1 mfma", dv(deconv_mfma_kernel<0>, pk + PL.dcm_off[1]), fld);
    run("deconv1 mfma no stores (1)", dv(deconv_mfma_kernel<1>, pk + PL.dcm_off[1]), fld);
    run("deconv1 mfma no MFMA (2)", dv(deconv_mfma_kernel<2>, pk + PL.dcm_off[1]), fld);
    run("deconv1 (H/2 -> H)", dc(deconv_px2_kernel<0>), fld);
    run("deconv1 no stores (1)", dc(deconv_px2_kernel<1>), fld);
    run("deconv1 no channel loop (2)", dc(deconv_px2_kernel<2>), fld);
    run("deconv1 no staging loads (4)", dc(deconv_px2_kernel<4>), fld);
    run("deconv1 skeleton (7)", dc(deconv_px2_kernel<7>), fld);
  }
  run("cell0 h3 DB0 PIPE0", [&] { return run_cell_h3<0, 1, 8, 0, 0, 0>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB0 PIPE1", [&] { return run_cell_h3<0, 1, 8, 0, 0, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 PIPE0", [&] { return run_cell_h3<0, 1, 8, 0, 1, 0>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 PIPE1", [&] { return run_cell_h3<0, 1, 8, 0, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell1 h3 DB0 PIPE0", [&] { return run_cell_h3<1, 1, 8, 0, 0, 0>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB0 PIPE1", [&] { return run_cell_h3<1, 1, 8, 0, 0, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB1 PIPE0", [&] { return run_cell_h3<1, 1, 8, 0, 1, 0>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB1 PIPE1", [&] { return run_cell_h3<1, 1, 8, 0, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell3 h3 DB0 PIPE0", [&] { return run_cell_h3<3, 1, 8, 0, 0, 0>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell3 h3 DB0 PIPE1", [&] { return run_cell_h3<3, 1, 8, 0, 0, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell3 h3 DB1 PIPE0", [&] { return run_cell_h3<3, 1, 8, 0, 1, 0>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell3 h3 DB1 PIPE1", [&] { return run_cell_h3<3, 1, 8, 0, 1, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell4 h3 DB0 PIPE0", [&] { return run_cell_h3<4, 1, 8, 0, 0, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell4 h3 DB0 PIPE1", [&] { return run_cell_h3<4, 1, 8, 0, 0, 1>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell4 h3 DB1 PIPE0", [&] { return run_cell_h3<4, 1, 8, 0, 1, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell4 h3 DB1 PIPE1", [&] { return run_cell_h3<4, 1, 8, 0, 1, 1>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell0 h3 RW2 W4 DB1", [&] { return run_cell_h3<0, 2, 4, 0, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 RW2 W4 DB0", [&] { return run_cell_h3<0, 2, 4, 0, 0, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 RW2 W8 DB0", [&] { return run_cell_h3<0, 2, 8, 0, 0, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 RW2 W8 DB0 nopipe", [&] { return run_cell_h3<0, 2, 8, 0, 0, 0>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell4 h3 RW2 W8 DB0", [&] { return run_cell_h3<4, 2, 8, 0, 0, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell4 h3 RW2 W4 DB0", [&] { return run_cell_h3<4, 2, 4, 0, 0, 0>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell3 h3 RW2 W8 DB0", [&] { return run_cell_h3<3, 2, 8, 0, 0, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell1 h3 RW2 W8 DB0", [&] { return run_cell_h3<1, 2, 8, 0, 0, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell0 h3 DB1 A once (8)", [&] { return run_cell_h3<0, 1, 8, 8, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 B once (16)", [&] { return run_cell_h3<0, 1, 8, 16, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 A+B once (24)", [&] { return run_cell_h3<0, 1, 8, 24, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 MFMA only, A once (14)", [&] { return run_cell_h3<0, 1, 8, 14, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 DB1 MFMA only, A+B once (30)", [&] { return run_cell_h3<0, 1, 8, 30, 1, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 no MFMA (1)", [&] { return run_cell_h3<0, 1, 8, 1>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 no staging (2)", [&] { return run_cell_h3<0, 1, 8, 2>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 MFMA only (6)", [&] { return run_cell_h3<0, 1, 8, 6>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell0 h3 skeleton (7)", [&] { return run_cell_h3<0, 1, 8, 7>(h3(args(0, 1)), invs, 256, K_CELL0, 0); }, fl0);
  run("cell1 h3 DB1 no MFMA (1)", [&] { return run_cell_h3<1, 1, 8, 1, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB1 no staging (2)", [&] { return run_cell_h3<1, 1, 8, 2, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB1 MFMA only (6)", [&] { return run_cell_h3<1, 1, 8, 6, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell1 h3 DB1 skeleton (7)", [&] { return run_cell_h3<1, 1, 8, 7, 1, 1>(h3(args(1, 2)), invs, 256, K_CELL1, 0); }, fl1);
  run("cell3 h3 no MFMA (1)", [&] { return run_cell_h3<3, 1, 8, 1, 0, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell3 h3 MFMA only (6)", [&] { return run_cell_h3<3, 1, 8, 6, 0, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell3 h3 skeleton (7)", [&] { return run_cell_h3<3, 1, 8, 7, 0, 1>(h3(args(3, 2)), invs, 256, K_CELL3, 0); }, fl3);
  run("cell4 h3 no MFMA (1)", [&] { return run_cell_h3<4, 1, 8, 1>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  run("cell4 h3 MFMA only (6)", [&] { return run_cell_h3<4, 1, 8, 6>(h3(args(4, 1)), invs, 256, K_CELL4, 0); }, fl4);
  return 0;
}
