// Torch-free check of HIP-graph replay with a forked side stream (the pattern of a captured training step: the
// weight-gradient stream forks from the compute stream after every layer and joins at the end).
//
// Captured program (race-free by construction):
//   main stream s0:  m[l] = f(m[l-1])            for l = 0..L-1   (m[-1] = x)
//   side stream s1:  s[l] = g(m[l], s[l-1])      after an event recorded on s0 behind m[l]   (s[-1] = 0)
//   join:            out = m[L-1] + s[L-1]       on s0 after an event recorded on s1
// Mode "u" (the pattern of tools/diag_fork_graph.py variant B): the side stream only scales an UNRELATED buffer at
// three fork points, every main layer starts with a memset node (a zeroed scratch it then reads), join at the end.
// Every replay first rewrites x (a kernel outside the graph), then the result is compared bit for bit with the same
// kernels launched eagerly on ONE stream. Prints the mismatching replays and the largest difference.
//   hipcc --offload-arch=gfx950 -O2 tools/graph_fork_repro.hip -o tools/graph_fork_repro.bin
//   tools/graph_fork_repro.bin [replays] [layers] [mode f|u]   (DEBUG_HIP_FORCE_GRAPH_QUEUES=1: one-queue executor)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

__global__ void fill_x(float* x, int n, int rep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = sinf(0.001f * (float)i + 0.37f * (float)rep);
}

// a fixed amount of dependent arithmetic per element (kernels long enough to overlap across streams)
__global__ void step_main(const float* __restrict__ in, float* __restrict__ out, int n, int iters, float a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = in[i];
  for (int k = 0; k < iters; ++k) v = fmaf(v, a, 0.001f * (float)(k & 7)) * 0.999f;
  out[i] = v;
}

__global__ void step_side(const float* __restrict__ m, const float* __restrict__ prev, float* __restrict__ out, int n,
                          int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = m[i] + (prev ? prev[i] : 0.f);
  for (int k = 0; k < iters; ++k) v = fmaf(v, 0.9995f, 0.0001f);
  out[i] = v;
}

__global__ void scale_unrelated(float* __restrict__ z, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) z[i] *= 1.0001f;
}

__global__ void step_main_tmp(const float* __restrict__ in, const float* __restrict__ tmp, float* __restrict__ out,
                              int n, int iters, float a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = in[i] + tmp[i];
  for (int k = 0; k < iters; ++k) v = fmaf(v, a, 0.001f * (float)(k & 7)) * 0.999f;
  out[i] = v;
}

__global__ void join_add(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

int main(int argc, char** argv) {
  const int replays = argc > 1 ? std::atoi(argv[1]) : 200;
  const int L = argc > 2 ? std::atoi(argv[2]) : 8;
  const bool unrelated = argc > 3 && argv[3][0] == 'u';
  const int n = 1 << 21, iters = 64, tpb = 256, blocks = (n + tpb - 1) / tpb;
  const char* q = std::getenv("DEBUG_HIP_FORCE_GRAPH_QUEUES");
  std::printf("graph_fork_repro: mode %s, %d replays, %d layers, n = %d, DEBUG_HIP_FORCE_GRAPH_QUEUES=%s\n",
              unrelated ? "u" : "f", replays, L, n, q ? q : "(unset)");
  float *x, *out, *ref, *z;
  std::vector<float*> m(L), s(L), tmp(L);
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMalloc(&out, n * 4));
  CHECK(hipMalloc(&ref, n * 4));
  for (int l = 0; l < L; ++l) {
    CHECK(hipMalloc(&m[l], n * 4));
    CHECK(hipMalloc(&s[l], n * 4));
    CHECK(hipMalloc(&tmp[l], n * 4));
  }
  CHECK(hipMalloc(&z, n * 4));
  CHECK(hipMemset(z, 0, n * 4));
  hipStream_t s0, s1;
  CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(L + 1);
  for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  auto program = [&](hipStream_t a, hipStream_t b, bool fork) {
    const float* prev = x;
    if (unrelated) {
      for (int l = 0; l < L; ++l) {
        CHECK(hipMemsetAsync(tmp[l], 0, n * 4, a));
        step_main_tmp<<<blocks, tpb, 0, a>>>(prev, tmp[l], m[l], n, iters, 1.0f + 0.01f * (float)l);
        if (fork && (l == L / 4 || l == L / 2 || l == 3 * L / 4)) {
          CHECK(hipEventRecord(ev[l], a));
          CHECK(hipStreamWaitEvent(b, ev[l], 0));
          scale_unrelated<<<blocks, tpb, 0, b>>>(z, n);
        }
        prev = m[l];
      }
      if (fork) {
        CHECK(hipEventRecord(ev[L], b));
        CHECK(hipStreamWaitEvent(a, ev[L], 0));
      }
      join_add<<<blocks, tpb, 0, a>>>(m[L - 1], m[0], fork ? out : ref, n);
      return;
    }
    for (int l = 0; l < L; ++l) {
      step_main<<<blocks, tpb, 0, a>>>(prev, m[l], n, iters, 1.0f + 0.01f * (float)l);
      if (fork) {
        CHECK(hipEventRecord(ev[l], a));
        CHECK(hipStreamWaitEvent(b, ev[l], 0));
      }
      step_side<<<blocks, tpb, 0, fork ? b : a>>>(m[l], l ? s[l - 1] : nullptr, s[l], n, iters);
      prev = m[l];
    }
    if (fork) {
      CHECK(hipEventRecord(ev[L], b));
      CHECK(hipStreamWaitEvent(a, ev[L], 0));
    }
    join_add<<<blocks, tpb, 0, a>>>(m[L - 1], s[L - 1], fork ? out : ref, n);
  };

  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  program(s0, s1, true);
  CHECK(hipStreamEndCapture(s0, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));

  std::vector<float> h_out(n), h_ref(n);
  int bad = 0;
  double worst = 0.0;
  for (int r = 0; r < replays; ++r) {
    fill_x<<<blocks, tpb, 0, s0>>>(x, n, r);
    CHECK(hipGraphLaunch(ge, s0));
    program(s0, s0, false);           // eager reference on the one stream, after the replay (stream order)
    CHECK(hipStreamSynchronize(s0));
    CHECK(hipMemcpy(h_out.data(), out, n * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h_ref.data(), ref, n * 4, hipMemcpyDeviceToHost));
    int diff = 0;
    double md = 0.0;
    for (int i = 0; i < n; ++i)
      if (h_out[i] != h_ref[i]) {
        ++diff;
        md = std::fmax(md, std::fabs((double)h_out[i] - (double)h_ref[i]));
      }
    if (diff) {
      ++bad;
      worst = std::fmax(worst, md);
      if (bad <= 5) std::printf("  replay %d: %d elements differ, max |diff| %.3g\n", r, diff, md);
    }
  }
  std::printf("RESULT mismatching replays %d / %d, max |diff| %.3g\n", bad, replays, worst);
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return 0;
}
