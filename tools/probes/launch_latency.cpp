// launch_latency.cpp -- what a one-kernel call costs end to end on this box, by the
// way the host learns that the kernel finished:
//   event      hipLaunchKernelGGL + hipEventRecord + hipEventSynchronize
//   stream     hipLaunchKernelGGL + hipStreamSynchronize
//   flag_kern  the kernel itself stores a sequence number to pinned host memory (vector
//              store, system scope); the host spins on it
//   flag_wv    hipStreamWriteValue32 to pinned host memory after the kernel; host spins
//   graph      a one-node hipGraph, hipGraphLaunch + hipStreamSynchronize
// Each: 2000 calls after 200 warm-up, median and p90 in microseconds, one JSON line.
// Then the aggregate rate of T threads (1 .. 16), each on its own stream: "mt_flag" =
// launch + spin on the thread's own word per call; "mt_async" = launches only, one
// stream synchronize at the end (the dispatch rate).
//   hipcc --offload-arch=gfx950 -O2 launch_latency.cpp -o launch_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <thread>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void empty_kernel(uint32_t *unused) {
  if (unused && threadIdx.x == 1024) unused[threadIdx.x] = 0;  // never taken
}

// thread 0 of block 0 publishes `seq` once every wave of the grid has passed the barrier
// of its own block (one block: the grid)
__global__ void flag_kernel(uint32_t *flag, uint32_t seq) {
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double us_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

template <class F>
static int measure(const char *name, F f, bool last) {
  std::vector<double> t;
  for (int i = 0; i < 2200; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (f((uint32_t)i + 1)) return 1;
    if (i >= 200) t.push_back(us_since(t0));
  }
  std::sort(t.begin(), t.end());
  printf("\"%s\": {\"median_us\": %.2f, \"p90_us\": %.2f, \"min_us\": %.2f}%s", name, t[t.size() / 2],
         t[t.size() * 9 / 10], t[0], last ? "" : ", ");
  return 0;
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t *flag = nullptr;
  CHECK(hipHostMalloc((void **)&flag, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t *dflag = nullptr;
  CHECK(hipHostGetDevicePointer((void **)&dflag, flag, 0));
  volatile uint32_t *vf = flag;
  *vf = 0;
  // graph of one empty kernel
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  printf("{");
  int rc = 0;
  rc |= measure("event", [&](uint32_t) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    if (hipEventRecord(ev, s) != hipSuccess) return 1;
    return hipEventSynchronize(ev) != hipSuccess ? 1 : 0;
  }, false);
  rc |= measure("stream", [&](uint32_t) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    return hipStreamSynchronize(s) != hipSuccess ? 1 : 0;
  }, false);
  rc |= measure("flag_kern", [&](uint32_t seq) {
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
    const auto t0 = std::chrono::steady_clock::now();
    while (*vf != seq)
      if (us_since(t0) > 1e6) return 1;  // 1 s: the flag never came
    return 0;
  }, false);
  *vf = 0;
  rc |= measure("flag_wv", [&](uint32_t seq) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    if (hipStreamWriteValue32(s, dflag, seq, 0) != hipSuccess) return 1;
    const auto t0 = std::chrono::steady_clock::now();
    while (*vf != seq)
      if (us_since(t0) > 1e6) return 1;
    return 0;
  }, false);
  rc |= measure("graph", [&](uint32_t) {
    if (hipGraphLaunch(ge, s) != hipSuccess) return 1;
    return hipStreamSynchronize(s) != hipSuccess ? 1 : 0;
  }, true);
  // T threads, each with its own stream and word
  for (int mode = 0; mode < 2; ++mode) {
    printf(", \"%s\": {", mode ? "mt_async" : "mt_flag");
    for (int T : {1, 2, 4, 8, 16}) {
      std::vector<std::thread> th;
      std::vector<int> bad(T, 0);
      const int calls = 4000;
      const auto t0 = std::chrono::steady_clock::now();
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          hipStream_t q;
          if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) { bad[t] = 1; return; }
          uint32_t *word = dflag + 16 * (t + 1);  // (own 64-byte line)
          volatile uint32_t *hw = flag + 16 * (t + 1);
          *hw = 0;
          for (int i = 1; i <= calls && !bad[t]; ++i) {
            if (mode == 0) {
              hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, q, word, (uint32_t)i);
              const auto w0 = std::chrono::steady_clock::now();
              while (*hw != (uint32_t)i)
                if (us_since(w0) > 1e6) { bad[t] = 1; break; }
            } else {
              hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, q, nullptr);
            }
          }
          if (hipStreamSynchronize(q) != hipSuccess) bad[t] = 1;
          (void)hipStreamDestroy(q);
        });
      for (auto &x : th) x.join();
      const double us = us_since(t0);
      for (int b : bad) rc |= b;
      printf("\"%d\": %.0f%s", T, T * calls / us * 1e3, T == 16 ? "" : ", ");  // kcalls/s
    }
    printf("}");
  }
  printf("}\n");
  CHECK(hipStreamSynchronize(s));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  CHECK(hipHostFree(flag));
  CHECK(hipEventDestroy(ev));
  CHECK(hipStreamDestroy(s));
  return rc;
}
