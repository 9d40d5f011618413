// Test harness (not the product): runs the product header wg_x25519.h on the host
// for tests/test_handshake_cpu.py.  stdin: "scalar_hex point_hex" lines.
#include "wg_x25519.h"
#include <cstdio>
#include <cstring>
int main() {
  char hk[65], hu[65];
  while (scanf("%64s %64s", hk, hu) == 2) {
    uint8_t k[32], u[32];
    for (int i = 0; i < 32; ++i) { sscanf(hk + 2*i, "%2hhx", &k[i]); sscanf(hu + 2*i, "%2hhx", &u[i]); }
    uint32_t kw[8], uw[8], ow[8];
    memcpy(kw, k, 32); memcpy(uw, u, 32);
    wg::x25519::scalarmult(ow, kw, uw);
    const uint8_t *o = (const uint8_t*)ow;
    for (int i = 0; i < 32; ++i) printf("%02x", o[i]);
    printf("\n");
  }
}
