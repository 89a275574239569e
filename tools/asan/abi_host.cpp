// Host-side AddressSanitizer harness of the C ABI (SURVEY §5 "Sanitizers": a
// -fsanitize=address host variant).  Links libaarmvs_asan.so, whose host code is built
// with AddressSanitizer (device code unchanged), and drives every host path that runs
// without a GPU: shape validation, the workspace carve (sizes and every state region
// written end to end inside a heap buffer of exactly aarmvs_sweep_workspace_bytes),
// argument rejection of each entry point, error strings, the profiling bookkeeping.
// A heap overflow or use-after-free in that code aborts with an ASan report.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aarmvs.h"

static int g_fail = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

static bool has_error() {
  const char* e = aarmvs_last_error();
  return e && std::strlen(e) > 0;
}

// every h / c region of the workspace, written over its full extent
static void carve(int B, int H, int W, int nsrc) {
  const size_t bytes = aarmvs_sweep_workspace_bytes(B, H, W, nsrc);
  CHECK(bytes > 0);
  std::vector<unsigned char> ws(bytes);
  const int hid[5] = {16, 16, 16, 16, 8}, sc[5] = {1, 2, 4, 2, 1};
  for (int par = 0; par < 8; ++par)   // planes processed: every slot of the rings (up to 6)
    for (int k = 0; k < 5; ++k)
      for (int which = 0; which < 2; ++which) {
        float* p = aarmvs_state_ptr(ws.data(), B, H, W, nsrc, par, k, which);
        CHECK(p != nullptr);
        if (!p) continue;
        const size_t n = (size_t)B * (H / sc[k]) * (W / sc[k]) * hid[k];
        const unsigned char* b = reinterpret_cast<unsigned char*>(p);
        CHECK(b >= ws.data() && b + n * sizeof(float) <= ws.data() + bytes);
        std::memset(p, 0x5a, n * sizeof(float));   // ASan: stays inside the buffer
      }
  CHECK(aarmvs_state_ptr(ws.data(), B, H, W, nsrc, 0, 5, 0) == nullptr);
  CHECK(aarmvs_state_ptr(ws.data(), B, H, W, nsrc, 0, -1, 0) == nullptr);
  CHECK(aarmvs_state_ptr(nullptr, B, H, W, nsrc, 0, 0, 0) == nullptr);
}

int main() {
  CHECK(aarmvs_version() != nullptr);
  CHECK(aarmvs_param_count() > 0);
  CHECK(aarmvs_packed_param_bytes() >= aarmvs_param_count() * sizeof(float));

  // valid geometries: the workspace grows with every dimension
  carve(1, 8, 8, 1);
  carve(2, 64, 80, 6);
  carve(1, 96, 200, 10);
  carve(3, 36, 44, 16);
  CHECK(aarmvs_sweep_workspace_bytes(1, 64, 80, 6) < aarmvs_sweep_workspace_bytes(2, 64, 80, 6));
  CHECK(aarmvs_sweep_workspace_bytes(1, 64, 80, 2) < aarmvs_sweep_workspace_bytes(1, 64, 80, 6));

  // rejected geometries: 0 bytes and a message
  const int bad[][4] = {{0, 8, 8, 1},   {1, 6, 8, 1},  {1, 8, 10, 1}, {1, 0, 8, 1},
                        {1, 8, 8, 0},   {1, 8, 8, 17}, {-1, 8, 8, 1}, {1, 65536, 65536, 1},
                        {1, 8, -4, 1}};
  for (const auto& g : bad) {
    CHECK(aarmvs_sweep_workspace_bytes(g[0], g[1], g[2], g[3]) == 0);
    CHECK(has_error());
  }

  // every entry point rejects bad arguments before touching the device
  float dummy[64] = {};
  const float* srcs[AARMVS_MAX_SRC] = {dummy};
  CHECK(aarmvs_pack_params(nullptr, dummy, nullptr) == AARMVS_ERR_INVALID && has_error());
  CHECK(aarmvs_aux_stream(nullptr) == AARMVS_ERR_INVALID && has_error());
  CHECK(aarmvs_homo_warp(nullptr, dummy, dummy, 1, 32, 8, 8, dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_homo_warp(dummy, dummy, dummy, 1, 32, 1, 8, dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_homo_warp_backward(dummy, dummy, dummy, 0, 32, 8, 8, dummy, dummy, nullptr) ==
        AARMVS_ERR_INVALID);
  CHECK(aarmvs_homo_warp_backward(dummy, dummy, dummy, 1, 32, 8, 8, dummy, nullptr, nullptr) ==
        AARMVS_ERR_INVALID);   // no workspace
  CHECK(aarmvs_homo_warp_backward_workspace_bytes(1, 32, 8, 8) == 256 + 32 * 64 * 8);
  CHECK(aarmvs_homo_warp_backward_workspace_bytes(65, 32, 8, 8) == 256 + 64 * 32 * 64 * 8);
  CHECK(aarmvs_homo_warp_backward_workspace_bytes(1, 0, 8, 8) == 0);
  CHECK(aarmvs_sweep(nullptr, nullptr) == AARMVS_ERR_INVALID);
  aarmvs_sweep_args a;
  std::memset(&a, 0, sizeof(a));
  a.B = 1, a.C = 32, a.H = 8, a.W = 8, a.nsrc = 1, a.D = 4, a.d_begin = 0, a.d_end = 4;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID);   // null pointers
  a.ref_fea = dummy, a.src_fea[0] = dummy, a.rel_proj = dummy, a.depth_values = dummy;
  a.packed_params = dummy, a.workspace = dummy;
  a.C = 16;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID);   // C != 32
  a.C = 32, a.d_end = 5;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID);   // d_end > D
  a.d_end = 4, a.d_begin = 4;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID);   // empty plane range
  a.d_begin = 0, a.nsrc = 2;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID);   // src_fea[1] null
  // training record: sizes grow with the frame; a record with a null buffer is rejected
  CHECK(aarmvs_train_record_bytes(1, 8, 8, 1) > 0 && aarmvs_train_record_bytes(1, 8, 8, 7) == 0);
  CHECK(aarmvs_train_record_bytes(1, 8, 8, 5) == 8 * 8 * 16 && aarmvs_train_record_bytes(1, 8, 8, 6) > 0);
  CHECK(aarmvs_train_record_bytes(1, 8, 8, 2) < aarmvs_train_record_bytes(1, 16, 8, 2));
  CHECK(aarmvs_train_record_bytes(1, 6, 8, 0) == 0 && has_error());
  aarmvs_train_record rec;
  std::memset(&rec, 0, sizeof(rec));
  a.nsrc = 1, a.record = &rec;
  CHECK(aarmvs_sweep(&a, nullptr) == AARMVS_ERR_INVALID && has_error());   // null record buffers
  a.record = nullptr;
  // backward: argument rejection before any launch
  CHECK(aarmvs_backward_scratch_bytes(1, 64, 80, 2) > 0 && aarmvs_backward_scratch_bytes(1, 6, 8, 1) == 0);
  CHECK(aarmvs_sweep_backward(nullptr, nullptr) == AARMVS_ERR_INVALID);
  aarmvs_backward_args ba;
  std::memset(&ba, 0, sizeof(ba));
  ba.B = 1, ba.C = 32, ba.H = 8, ba.W = 8, ba.nsrc = 1, ba.D = 4;
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // null pointers
  ba.ref_fea = dummy, ba.src_fea[0] = dummy, ba.rel_proj = dummy, ba.depth_values = dummy;
  ba.packed_params = dummy, ba.grad_cost = dummy, ba.workspace = dummy, ba.scratch = dummy;
  ba.record = &rec;
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // record buffers null
  float* rb = dummy;
  rec.x = rb, rec.state = rb, rec.z = rb, rec.u = rb, rec.stats = reinterpret_cast<double*>(rb);
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // t1 / ostats null
  rec.t1 = rb, rec.ostats = reinterpret_cast<double*>(rb);
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // grad_ref required
  ba.C = 16;
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // C != 32
  ba.C = 32, ba.H = 6;
  CHECK(aarmvs_sweep_backward(&ba, nullptr) == AARMVS_ERR_INVALID);   // H % 4
  a.nsrc = 2;
  CHECK(aarmvs_cost_slice(dummy, srcs, dummy, dummy, dummy, 1, 32, 8, 8, 2, dummy, dummy,
                          nullptr, nullptr) == AARMVS_ERR_INVALID);   // src_fea[1] null
  CHECK(aarmvs_cost_slice(dummy, srcs, dummy, dummy, dummy, 1, 8, 8, 8, 1, dummy, dummy,
                          nullptr, nullptr) == AARMVS_ERR_INVALID);   // C != 32
  CHECK(aarmvs_cost_slice(dummy, nullptr, dummy, dummy, dummy, 1, 32, 8, 8, 1, dummy, dummy,
                          nullptr, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_wta_update(dummy, dummy, dummy, dummy, nullptr, 1, 64, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_wta_update(dummy, dummy, dummy, dummy, dummy, 1, 0, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_unet_step(dummy, 1, 8, 8, 1, -1, dummy, dummy, dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_unet_step(dummy, 1, 8, 9, 1, 0, dummy, dummy, dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_softmax_depth(dummy, dummy, 1, 0, 64, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_softmax_depth(nullptr, dummy, 1, 4, 64, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_lstm_gates_forward(nullptr, dummy, 1, 8, 64, dummy, dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_lstm_gates_backward(dummy, dummy, nullptr, nullptr, 1, 0, 64, dummy, dummy, nullptr) ==
        AARMVS_ERR_INVALID);
  CHECK(aarmvs_group_norm_scratch_bytes(0, 16, 64) == 0);
  CHECK(aarmvs_group_norm_scratch_bytes(1, 16, 64) > 0);
  CHECK(aarmvs_group_norm_forward(dummy, nullptr, nullptr, 1, 16, 64, 3, 1e-5f, dummy, dummy, dummy,
                                  nullptr) == AARMVS_ERR_INVALID);   // 3 does not divide 16
  CHECK(aarmvs_group_norm_forward(nullptr, nullptr, nullptr, 1, 16, 64, 2, 1e-5f, dummy, dummy, dummy,
                                  nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_group_norm_backward(dummy, dummy, nullptr, dummy, 1, 16, 64, 2, dummy, dummy, nullptr,
                                   dummy, nullptr) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_fusion_filter(nullptr, nullptr) == AARMVS_ERR_INVALID);
  aarmvs_fusion_args f;
  std::memset(&f, 0, sizeof(f));
  f.H = 8, f.W = 8, f.nsrc = 11;
  CHECK(aarmvs_fusion_filter(&f, nullptr) == AARMVS_ERR_INVALID);   // nsrc > 10
  f.nsrc = 2, f.ref_depth = f.confidence = f.cams = dummy, f.src_depth[0] = dummy;
  f.photo_mask = f.geo_mask = f.final_mask = reinterpret_cast<unsigned char*>(dummy);
  f.depth_avg = reinterpret_cast<double*>(dummy);
  CHECK(aarmvs_fusion_filter(&f, nullptr) == AARMVS_ERR_INVALID);   // src_depth[1] null

  // profiling bookkeeping with nothing recorded
  const int nk = aarmvs_profile_kernel_count();
  CHECK(nk > 0);
  aarmvs_profile_enable(1);
  aarmvs_profile_reset();
  for (int k = 0; k < nk; ++k) {
    long long n = -1;
    double ms = -1.0;
    CHECK(aarmvs_profile_kernel_name(k) != nullptr);
    CHECK(aarmvs_profile_read(k, &n, &ms) == AARMVS_OK && n == 0 && ms == 0.0);
  }
  aarmvs_profile_enable(0);
  CHECK(aarmvs_profile_kernel_name(nk) == nullptr && aarmvs_profile_kernel_name(-1) == nullptr);
  long long n;
  double ms;
  CHECK(aarmvs_profile_read(nk, &n, &ms) == AARMVS_ERR_INVALID);
  CHECK(aarmvs_profile_read(0, nullptr, &ms) == AARMVS_ERR_INVALID);

  std::printf("abi_host: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
