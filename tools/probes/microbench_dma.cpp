// microbench_dma.cpp -- copy-engine rates between pinned host memory and HBM, the
// data movement under the batched Tunn's pipeline (wg_tunn.cpp): one direction
// alone, both directions at once on two streams, 1D chunks vs 2D packet rows
// (width = the packet, pitch = the slot), hipHostMalloc'd vs hipHostRegister'ed
// host buffers.  Prints one JSON line per case.
//   hipcc -O2 --offload-arch=gfx950 tools/microbench_dma.cpp -o build/proto/microbench_dma
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// a blit kernel: float4 per lane, grid-stride (zero-copy reads / writes of pinned host memory)
__global__ void blit_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

struct Case {
  const char *name;
  bool h2d, d2h, two_d, registered;
};

int main(int argc, char **argv) {
  const size_t total = (size_t)262144 * 1408;  // the Tunn bench's batch: 262,144 slots of 1408 B
  const size_t chunk = (size_t)16 << 20;
  const uint32_t W = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1350, pitch = 1408;
  uint8_t *h_alloc[2], *h_reg[2], *d[2];
  for (int i = 0; i < 2; ++i) {
    CK(hipHostMalloc(&h_alloc[i], total, hipHostMallocDefault));
    h_reg[i] = (uint8_t *)std::aligned_alloc(4096, total);
    std::memset(h_reg[i], i, total);
    std::memset(h_alloc[i], i, total);
    CK(hipHostRegister(h_reg[i], total, hipHostRegisterMapped));
    CK(hipMalloc(&d[i], total));
  }
  hipStream_t s[2];
  for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  const Case cases[] = {
      {"h2d_1d_hostmalloc", true, false, false, false}, {"d2h_1d_hostmalloc", false, true, false, false},
      {"both_1d_hostmalloc", true, true, false, false}, {"h2d_2d_hostmalloc", true, false, true, false},
      {"d2h_2d_hostmalloc", false, true, true, false},  {"both_2d_hostmalloc", true, true, true, false},
      {"h2d_1d_registered", true, false, false, true},  {"d2h_1d_registered", false, true, false, true},
      {"both_1d_registered", true, true, false, true},  {"h2d_2d_registered", true, false, true, true},
      {"d2h_2d_registered", false, true, true, true},   {"both_2d_registered", true, true, true, true},
  };
  for (const Case &c : cases) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      size_t bytes = 0;
      for (size_t off = 0; off < total; off += chunk) {
        const size_t n = std::min(chunk, total - off);
        const size_t rows = n / pitch;
        uint8_t *hin = (c.registered ? h_reg[0] : h_alloc[0]) + off;
        uint8_t *hout = (c.registered ? h_reg[1] : h_alloc[1]) + off;
        if (c.h2d) {
          if (c.two_d) CK(hipMemcpy2DAsync(d[0] + off, pitch, hin, pitch, W, rows, hipMemcpyHostToDevice, s[0]));
          else CK(hipMemcpyAsync(d[0] + off, hin, n, hipMemcpyHostToDevice, s[0]));
          bytes += c.two_d ? rows * W : n;
        }
        if (c.d2h) {
          if (c.two_d) CK(hipMemcpy2DAsync(hout, pitch, d[1] + off, pitch, W, rows, hipMemcpyDeviceToHost, s[1]));
          else CK(hipMemcpyAsync(hout, d[1] + off, n, hipMemcpyDeviceToHost, s[1]));
          bytes += c.two_d ? rows * W : n;
        }
      }
      CK(hipDeviceSynchronize());
      const double dt = now() - t0;
      if (rep == 2)
        std::printf("{\"case\": \"%s\", \"width\": %u, \"pitch\": %u, \"bytes\": %zu, \"ms\": %.3f, \"GBps\": %.2f}\n",
                    c.name, W, pitch, bytes, dt * 1e3, bytes / dt / 1e9);
    }
  }
  // kernel copies over PCIe (zero-copy): device -> host writes, host -> device reads, both at once
  const char *kn[] = {"kernel_d2h", "kernel_h2d", "kernel_both", "kernel_d2h_registered",
                      "sdma_h2d_plus_kernel_d2h"};
  for (int kc = 0; kc < 5; ++kc) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      size_t bytes = 0;
      for (size_t off = 0; off < total; off += chunk) {
        const size_t n = std::min(chunk, total - off);
        uint8_t *hh = (kc == 3 ? h_reg[1] : h_alloc[1]) + off;
        if (kc == 4) {
          CK(hipMemcpyAsync(d[0] + off, h_alloc[0] + off, n, hipMemcpyHostToDevice, s[0]));
          bytes += n;
        }
        if (kc == 0 || kc == 2 || kc == 3 || kc == 4) {
          hipLaunchKernelGGL(blit_kernel, dim3(1024), dim3(256), 0, s[1], (const uint4 *)(d[1] + off), (uint4 *)hh, n / 16);
          bytes += n;
        }
        if (kc == 1 || kc == 2) {
          hipLaunchKernelGGL(blit_kernel, dim3(1024), dim3(256), 0, s[0], (const uint4 *)(h_alloc[0] + off),
                             (uint4 *)(d[0] + off), n / 16);
          bytes += n;
        }
      }
      CK(hipDeviceSynchronize());
      const double dt = now() - t0;
      if (rep == 2)
        std::printf("{\"case\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"GBps\": %.2f}\n", kn[kc], bytes,
                    dt * 1e3, bytes / dt / 1e9);
    }
  }
  return 0;
}
