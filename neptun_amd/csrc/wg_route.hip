// wg_route.hip -- inbound routing of raw datagram batches on the device.
//
// NepTUN routes a DATA datagram by its receiver index (device/mod.rs:1022-1024
// picks the peer by receiver_idx >> 8, noise/mod.rs:550-556 the session by
// receiver_idx % 8).  Here a linear-probing hash table in HBM maps each live
// receiving index to the key slot of that session's receiving key; one lane
// per descriptor reads the datagram header and fills in descs[i].key_slot.
// Memory-bound and tiny next to the AEAD: 16 header bytes + one probe (usually
// one 8-byte L2-resident entry) + a 4-byte store per packet.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "neptun_gpu.h"
#include "wg_aead_kernels.h"

namespace wg {

__global__ __launch_bounds__(256) void route_kernel(wg_packet_desc *descs, uint32_t n,
                                                    const uint8_t *src, const uint2 *table,
                                                    uint32_t bits) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = descs[i].src_off;
  const uint32_t len = descs[i].len;
  uint32_t slot = WG_KEY_SLOT_INVALID_PACKET;
  if (len >= WG_DATA_OVERHEAD_SZ) {  // parse_incoming_packet: DATA needs >= 32 bytes
    const uint8_t *h = src + off;
    uint32_t type, ridx;
    if ((off & 3u) == 0) {
      type = reinterpret_cast<const uint32_t *>(h)[0];
      ridx = reinterpret_cast<const uint32_t *>(h)[1];
    } else {  // any byte alignment is legal input here; the AEAD kernel reports it
      type = h[0] | (uint32_t)h[1] << 8 | (uint32_t)h[2] << 16 | (uint32_t)h[3] << 24;
      ridx = h[4] | (uint32_t)h[5] << 8 | (uint32_t)h[6] << 16 | (uint32_t)h[7] << 24;
    }
    if (type == WG_MSG_DATA) {
      slot = WG_KEY_SLOT_NO_SESSION;
      if (table) {
        const uint32_t mask = (1u << bits) - 1u;
        uint32_t pos = route_hash(ridx, bits);
        for (uint32_t probe = 0; probe <= mask; ++probe) {  // bounded: the table is never full
          const uint2 e = table[pos];
          if (e.y == WG_KEY_SLOT_NO_SESSION) break;  // empty entry ends the chain
          if (e.x == ridx) {
            slot = e.y;
            break;
          }
          pos = (pos + 1u) & mask;
        }
      }
    }
  }
  descs[i].key_slot = slot;
}

}  // namespace wg
