// doorbell.cpp -- can a resident kernel serve small calls without a launch each?
//
// A kernel of W workgroups stays resident on its own stream; workgroup w serves slot w
// of a ring in pinned host memory: thread 0 polls the slot's sequence word (a
// system-scope load over PCIe), the workgroup meets at a barrier, and thread 0 stores
// the sequence to the slot's done word (system-scope release).  Every workgroup leaves
// when the host sets the stop word or when its lease (s_memrealtime, 100 MHz) runs
// out, whichever comes first, so the grid always drains.  The host measures:
//   rt         one thread posting to one slot and spinning on its done word: the round
//              trip (median / p90 of 2000 after 200 warm-up)
//   mt         T threads (1 .. 16), each on its own slot: calls per second
//   side       while the resident kernel runs, an empty kernel on each of 8 ordinary
//              streams: microseconds until it completes (a stream on the resident
//              kernel's hardware queue would wait for the lease)
// for the resident kernel on a CU-masked stream (every CU in the mask: the runtime gives
// such a stream a hardware queue of its own) and, as the control, on an ordinary
// stream.  One JSON object per variant.  "vram" (run alone): the slots in fine-grained
// device memory, written by the host through its mapping of the BAR (the kernel polls
// HBM instead of reading over PCIe).  (A mask of CUs 0-31 hung: on gfx950 the
// workgroups are dealt round robin to the 8 XCDs, and those of an XCD without a CU in
// the mask never start -- a mask must cover every XCD.)
//   hipcc --offload-arch=gfx950 -O2 doorbell.cpp -o doorbell -lpthread
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

struct alignas(128) Slot {
  uint32_t seq;
  uint32_t pad0[31];
  uint32_t done;
  uint32_t pad1[31];
};

__global__ void empty_kernel(uint32_t *unused) {
  if (unused && threadIdx.x == 1024) unused[threadIdx.x] = 0;  // never taken
}

__global__ __launch_bounds__(256) void resident_kernel(Slot *slots, const uint32_t *stop, uint64_t lease_ticks) {
  __shared__ uint32_t s_go, s_seq;
  Slot *sl = slots + blockIdx.x;
  const uint64_t t0 = wall_clock64();
  uint32_t last = 0;
  if (threadIdx.x == 0) last = __hip_atomic_load(&sl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (threadIdx.x == 0) {
      uint32_t go = 0, q = last;
      for (uint32_t i = 0;; ++i) {
        q = __hip_atomic_load(&sl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (q != last) {
          go = 1;
          break;
        }
        if ((i & 15u) == 0u &&
            (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
             wall_clock64() - t0 > lease_ticks))
          break;
        __builtin_amdgcn_s_sleep(1);
      }
      s_go = go;
      s_seq = q;
    }
    __syncthreads();
    const uint32_t go = s_go, q = s_seq;
    __syncthreads();
    if (!go) return;  // (workgroup-uniform)
    if (threadIdx.x == 0) {
      __hip_atomic_store(&sl->done, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      last = q;
    }
  }
}

static double us_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

static bool call(Slot *s, uint32_t seq) {  // post and spin; false after 100 ms
  __atomic_store_n(&s->seq, seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) == seq) return true;
    if ((i & 1023u) == 0u && us_since(t0) > 100000.0) return false;
    __builtin_ia32_pause();
  }
}

static int variant(const char *name, bool masked, int cus, int total_cus, bool vram = false) {
  constexpr int W = 16;
  Slot *slots = nullptr;
  uint32_t *stop = nullptr;
  if (vram) {  // (fine-grained device memory the host writes through its BAR mapping)
    CHECK(hipExtMallocWithFlags((void **)&slots, sizeof(Slot) * W, hipDeviceMallocFinegrained));
    fprintf(stderr, "%s: device slots at %p, host write test\n", name, (void *)slots);
  } else {
    CHECK(hipHostMalloc((void **)&slots, sizeof(Slot) * W, hipHostMallocCoherent));
  }
  CHECK(hipHostMalloc((void **)&stop, 64, hipHostMallocCoherent));
  for (int i = 0; i < W; ++i) slots[i].seq = slots[i].done = 0;
  *stop = 0;
  hipStream_t rs;
  if (masked) {
    std::vector<uint32_t> mask((total_cus + 31) / 32, 0u);
    for (int c = 0; c < cus; ++c) mask[c / 32] |= 1u << (c % 32);
    CHECK(hipExtStreamCreateWithCUMask(&rs, (uint32_t)mask.size(), mask.data()));
  } else {
    CHECK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
  }
  const uint64_t lease = 100ull * 1000ull * 2500ull;  // 2.5 s at 100 MHz
  const auto tl = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(resident_kernel, dim3(W), dim3(256), 0, rs, slots, stop, lease);
  CHECK(hipGetLastError());
  printf("{\"variant\": \"%s\", \"masked_cus\": %d", name, masked ? cus : 0);
  if (vram) {  // host stores of a request's 2 KiB of descriptors into the mapped VRAM
    static uint8_t src[2048];
    for (int i = 0; i < 2048; ++i) src[i] = (uint8_t)i;
    uint8_t *dstp = nullptr;
    CHECK(hipExtMallocWithFlags((void **)&dstp, 2048, hipDeviceMallocFinegrained));
    std::vector<double> t;
    for (int r = 0; r < 1100; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 2048; i += 16) __builtin_memcpy(dstp + i, src + i, 16);
      __builtin_ia32_sfence();
      if (r >= 100) t.push_back(us_since(t0));
    }
    std::sort(t.begin(), t.end());
    printf(", \"host_store_2k_us\": %.3f", t[t.size() / 2]);
    CHECK(hipFree(dstp));
  }
  fflush(stdout);
  fprintf(stderr, "%s: launched\n", name);
  // first answer (the kernel's start)
  {
    const bool ok = call(&slots[0], 1);
    printf(", \"first_answer_us\": %.1f", ok ? us_since(tl) : -1.0);
    if (!ok) {
      printf(", \"error\": \"no answer\"}\n");
      *stop = 1;
      CHECK(hipStreamSynchronize(rs));
      return 0;
    }
  }
  fprintf(stderr, "%s: first answer\n", name);
  // round trip, one thread
  {
    std::vector<double> t;
    for (uint32_t i = 2; i < 2202; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      if (!call(&slots[0], i)) {
        printf(", \"error\": \"lost call\"");
        break;
      }
      if (i >= 202) t.push_back(us_since(t0));
    }
    std::sort(t.begin(), t.end());
    if (!t.empty())
      printf(", \"rt_median_us\": %.2f, \"rt_p90_us\": %.2f, \"rt_min_us\": %.2f", t[t.size() / 2],
             t[t.size() * 9 / 10], t[0]);
  }
  fflush(stdout);
  fprintf(stderr, "%s: round trips done\n", name);
  // T threads, one slot each
  printf(", \"mt_calls_per_s\": {");
  for (int T : {1, 2, 4, 8, 16}) {
    std::atomic<int> lost{0};
    const int K = 4000;
    std::vector<std::thread> th;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < T; ++k)
      th.emplace_back([&, k] {
        Slot *s = &slots[k];
        const uint32_t base = s->done;
        for (int i = 1; i <= K; ++i)
          if (!call(s, base + (uint32_t)i)) {
            ++lost;
            return;
          }
      });
    for (auto &x : th) x.join();
    const double us = us_since(t0);
    printf("%s\"%d\": %.0f", T == 1 ? "" : ", ", T, lost ? -1.0 : T * K / (us * 1e-6));
    fflush(stdout);
    fprintf(stderr, "%s: T=%d done\n", name, T);
  }
  printf("}");
  // ordinary streams while the resident kernel runs
  printf(", \"side_us\": [");
  for (int k = 0; k < 8; ++k) {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    double us = -1.0;
    while (us_since(t0) < 500000.0) {
      if (hipStreamQuery(s) == hipSuccess) {
        us = us_since(t0);
        break;
      }
    }
    printf("%s%.1f", k ? ", " : "", us);
    fflush(stdout);
    fprintf(stderr, "%s: side %d %.1f us\n", name, k, us);
    CHECK(hipStreamSynchronize(s));  // (a blocked one: after the lease)
    CHECK(hipStreamDestroy(s));
  }
  printf("]");
  *stop = 1;
  fprintf(stderr, "%s: stop\n", name);
  const auto ts = std::chrono::steady_clock::now();
  CHECK(hipStreamSynchronize(rs));
  printf(", \"stop_us\": %.1f}\n", us_since(ts));
  fflush(stdout);
  CHECK(hipStreamDestroy(rs));
  if (vram) CHECK(hipFree(slots));
  else CHECK(hipHostFree(slots));
  CHECK(hipHostFree(stop));
  return 0;
}

int main(int argc, char **argv) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const char *only = argc > 1 ? argv[1] : nullptr;
  auto want = [&](const char *v) { return !only || std::string(only) == v; };
  if (want("masked_all") && variant("masked_all", true, cus, cus)) return 1;
  if (want("plain_stream") && variant("plain_stream", false, 0, cus)) return 1;
  if (only && std::string(only) == "vram" && variant("vram", false, 0, cus, true)) return 1;
  return 0;
}
