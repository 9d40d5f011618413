// wg_pipe.cpp -- host-resident batches: chunked H2D -> AEAD kernel -> D2H over
// several HIP streams (include/neptun_gpu.h, wg_gpu_pipe_*).
//
// This is the end-to-end shape of NepTUN's data path on a GPU: packets start
// in host memory (TUN reads, device/mod.rs:1295-1326, or UDP receives,
// device/mod.rs:1115-1218) and end there (UDP sends / TUN writes).  On the
// device every chunk uses NepTUN's slot layout (datagram at slot+0, plaintext
// at slot+16) so the kernels run their aligned fast path whatever the host
// layout is; the 2-D copies move only packet bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <new>
#include <string>
#include <vector>

#include "neptun_gpu.h"

int wg_pipe_fail(int rc, const char *what, hipError_t e);  // wg_gpu.cpp
int wg_ctx_device(const wg_gpu_ctx *ctx);                   // wg_gpu.cpp

struct wg_gpu_pipe {
  wg_gpu_ctx *ctx = nullptr;
  int device = 0;
  uint64_t chunk_bytes = 0;
  std::vector<hipStream_t> streams;
  std::vector<uint8_t *> d_in, d_out;
  std::vector<int32_t *> d_status;
  uint32_t max_status = 0;
};

namespace {

#define PIPE_HIP(call, what)                                              \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) return wg_pipe_fail(WG_RC_HIP_ERROR, what, e_); \
  } while (0)

void release(wg_gpu_pipe *p) {
  for (auto s : p->streams) (void)hipStreamDestroy(s);
  for (auto b : p->d_in) (void)hipFree(b);
  for (auto b : p->d_out) (void)hipFree(b);
  for (auto b : p->d_status) (void)hipFree(b);
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// One direction over the whole batch.  Device slot stride S holds the larger
// side (datagram = len_wire bytes); device layout: wire at slot, text at slot+16.
int run_pipe(wg_gpu_pipe *p, bool seal, uint32_t n, uint32_t len, uint32_t key_slot,
             uint64_t counter_base, const uint8_t *h_src, uint64_t src_stride, uint8_t *h_dst,
             uint64_t dst_stride, int32_t *h_status) {
  if (!p || (n && (!h_src || !h_dst))) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "pipe: null argument", hipSuccess);
  if (n == 0) return WG_RC_OK;
  if (!seal && len < WG_DATA_OVERHEAD_SZ)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "pipe: open needs len >= 32", hipSuccess);
  const uint64_t text = seal ? len : len - WG_DATA_OVERHEAD_SZ;  // plaintext bytes
  const uint64_t wire = text + WG_DATA_OVERHEAD_SZ;
  const uint64_t S = (wire + 127) / 128 * 128;
  const uint64_t in_w = seal ? text : wire, out_w = seal ? wire : text;
  if (src_stride < in_w || dst_stride < out_w)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "pipe: stride smaller than the packet", hipSuccess);
  const uint64_t per_chunk = std::min<uint64_t>(p->chunk_bytes / S, p->max_status);
  if (per_chunk == 0) return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "pipe: chunk too small", hipSuccess);
  DevGuard g(p->device);
  const uint32_t depth = (uint32_t)p->streams.size();
  const uint64_t in_off = seal ? 16 : 0, out_off = seal ? 0 : 16;  // device slot offsets
  for (uint64_t c0 = 0, k = 0; c0 < n; c0 += per_chunk, ++k) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(per_chunk, n - c0);
    const uint32_t s = (uint32_t)(k % depth);
    hipStream_t st = p->streams[s];
    PIPE_HIP(hipMemcpy2DAsync(p->d_in[s] + in_off, S, h_src + c0 * src_stride, src_stride, in_w, m,
                              hipMemcpyHostToDevice, st),
             "pipe: H2D");
    int rc = seal ? wg_gpu_seal_strided(p->ctx, m, len, key_slot, counter_base + c0,
                                        p->d_in[s] + in_off, S, p->d_out[s] + out_off, S,
                                        p->d_status[s], st)
                  : wg_gpu_open_strided(p->ctx, m, len, key_slot, p->d_in[s] + in_off, S,
                                        p->d_out[s] + out_off, S, p->d_status[s], st);
    if (rc) return rc;
    PIPE_HIP(hipMemcpy2DAsync(h_dst + c0 * dst_stride, dst_stride, p->d_out[s] + out_off, S, out_w,
                              m, hipMemcpyDeviceToHost, st),
             "pipe: D2H");
    if (h_status)
      PIPE_HIP(hipMemcpyAsync(h_status + c0, p->d_status[s], (size_t)m * 4, hipMemcpyDeviceToHost,
                              st),
               "pipe: status D2H");
  }
  for (auto st : p->streams) PIPE_HIP(hipStreamSynchronize(st), "pipe: sync");
  return WG_RC_OK;
}

}  // namespace

extern "C" {

int wg_gpu_pipe_create(wg_gpu_ctx *ctx, uint64_t chunk_bytes, uint32_t depth, wg_gpu_pipe **out) {
  if (!ctx || !out || depth == 0 || chunk_bytes < 4096)
    return wg_pipe_fail(WG_RC_INVALID_ARGUMENT, "pipe_create: bad argument", hipSuccess);
  *out = nullptr;
  wg_gpu_pipe *p = new (std::nothrow) wg_gpu_pipe;
  if (!p) return wg_pipe_fail(WG_RC_OUT_OF_MEMORY, "pipe_create: host alloc", hipSuccess);
  p->ctx = ctx;
  p->device = wg_ctx_device(ctx);
  p->chunk_bytes = chunk_bytes;
  p->max_status = (uint32_t)std::min<uint64_t>(chunk_bytes / 64, 1u << 24);
  DevGuard g(p->device);
  hipError_t e = hipSuccess;
  for (uint32_t i = 0; i < depth && e == hipSuccess; ++i) {
    hipStream_t s = nullptr;
    uint8_t *a = nullptr, *b = nullptr;
    int32_t *st = nullptr;
    e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) p->streams.push_back(s);
    if (e == hipSuccess) e = hipMalloc(&a, chunk_bytes);
    if (e == hipSuccess) p->d_in.push_back(a);
    if (e == hipSuccess) e = hipMalloc(&b, chunk_bytes);
    if (e == hipSuccess) p->d_out.push_back(b);
    if (e == hipSuccess) e = hipMalloc(&st, (size_t)p->max_status * 4);
    if (e == hipSuccess) p->d_status.push_back(st);
  }
  if (e != hipSuccess) {
    release(p);
    delete p;
    return wg_pipe_fail(WG_RC_HIP_ERROR, "pipe_create: device resources", e);
  }
  *out = p;
  return WG_RC_OK;
}

int wg_gpu_pipe_destroy(wg_gpu_pipe *p) {
  if (!p) return WG_RC_OK;
  DevGuard g(p->device);
  for (auto s : p->streams) (void)hipStreamSynchronize(s);
  release(p);
  delete p;
  return WG_RC_OK;
}

int wg_gpu_pipe_seal_strided(wg_gpu_pipe *pipe, uint32_t n, uint32_t len, uint32_t key_slot,
                             uint64_t counter_base, const uint8_t *h_src, uint64_t src_stride,
                             uint8_t *h_dst, uint64_t dst_stride, int32_t *h_status) {
  return run_pipe(pipe, true, n, len, key_slot, counter_base, h_src, src_stride, h_dst, dst_stride,
                  h_status);
}

int wg_gpu_pipe_open_strided(wg_gpu_pipe *pipe, uint32_t n, uint32_t len, uint32_t key_slot,
                             const uint8_t *h_src, uint64_t src_stride, uint8_t *h_dst,
                             uint64_t dst_stride, int32_t *h_status) {
  return run_pipe(pipe, false, n, len, key_slot, 0, h_src, src_stride, h_dst, dst_stride,
                  h_status);
}

}  // extern "C"
