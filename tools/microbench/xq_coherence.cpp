// Kernel-boundary visibility across HIP streams (diagnostic, not shipped): a buffer is updated
// read-modify-write by kernels that alternate between two streams, ordered by events both ways
// (or host waits), while a third stream keeps the chip busy with unrelated traffic.  Every chunk
// of the buffer is handled by a different block (so a different CU / XCD) in every launch.  After
// K rounds every element must equal the number of increments; a lower value means a kernel read
// a stale copy of what an earlier kernel, ordered before it, had written.
//   ./xq_coherence [mode]   mode 0: one stream (control), 1: two streams + events,
//                           2: two streams + host waits, 3: two streams + events, no noise
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kChunk = 1024;   // floats per block

__global__ void __launch_bounds__(256) rmw_kernel(float* x, int nchunk, int rot) {
  const int c = (blockIdx.x + rot) % nchunk;
  float* p = x + (size_t)c * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += 256) p[i] = p[i] + 1.0f;
}

__global__ void __launch_bounds__(256) noise_kernel(float* y, size_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
      y[i] = y[i] * 0.999f + 1.0f;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 1;
  const int nchunk = 2048, K = 400;
  const size_t n = (size_t)nchunk * kChunk;   // 8 MB
  const size_t nn = (size_t)64 << 20;         // 256 MB of noise traffic
  float *x, *y;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, nn * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, nn * 4));
  hipStream_t qa, qb, qc;
  CK(hipStreamCreateWithFlags(&qa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&qb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&qc, hipStreamNonBlocking));
  hipEvent_t ea, eb;
  CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  const bool two = mode != 0, host = mode == 2, noise = mode != 3;
  for (int it = 0; it < K; ++it) {
    if (noise && it % 8 == 0) hipLaunchKernelGGL(noise_kernel, dim3(1024), dim3(256), 0, qc, y, nn, 1);
    hipLaunchKernelGGL(rmw_kernel, dim3(nchunk), dim3(256), 0, qa, x, nchunk, (it * 37) % nchunk);
    hipStream_t q2 = two ? qb : qa;
    if (two) {
      CK(hipEventRecord(ea, qa));
      if (host) CK(hipEventSynchronize(ea));
      else CK(hipStreamWaitEvent(qb, ea, 0));
    }
    hipLaunchKernelGGL(rmw_kernel, dim3(nchunk), dim3(256), 0, q2, x, nchunk, (it * 37 + 11) % nchunk);
    if (two) {
      CK(hipEventRecord(eb, qb));
      if (host) CK(hipEventSynchronize(eb));
      else CK(hipStreamWaitEvent(qa, eb, 0));
    }
  }
  CK(hipDeviceSynchronize());
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), x, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  float mn = 1e30f;
  for (size_t i = 0; i < n; ++i) {
    if (h[i] != 2.0f * K) ++bad;
    mn = h[i] < mn ? h[i] : mn;
  }
  printf("mode %d: %zu of %zu elements differ from %d (min %.0f)\n", mode, bad, n, 2 * K, mn);
  return bad ? 3 : 0;
}
