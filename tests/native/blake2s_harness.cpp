// Test harness (not the product): runs the product header wg_blake2s.h on the host
// for tests/test_handshake_cpu.py.
#include "wg_blake2s.h"
#include <cstdio>
#include <cstring>
// stdin lines: op hexkey hexdata ; op in {hash, hmac, mac}
static void hexin(const char *s, uint8_t *b, int n) { for (int i = 0; i < n; ++i) sscanf(s + 2*i, "%2hhx", &b[i]); }
int main() {
  char op[8], hk[200], hd[400];
  while (scanf("%7s %199s %399s", op, hk, hd) == 3) {
    uint8_t key[32] = {0}, data[128] = {0};
    int nd = strlen(hd) / 2; if (hd[0] == '-') nd = 0;
    hexin(hk, key, 32); if (nd) hexin(hd, data, nd);
    uint32_t kw[8], dw[32] = {0}, out[8];
    memcpy(kw, key, 32); memcpy(dw, data, nd);
    int outn = 32;
    if (!strcmp(op, "hash")) {  // key||data as a 64-byte hash input when nd == 32, else block hash
      if (nd == 32) wg::b2s::hash64(out, kw, dw); else wg::b2s::hash_block(out, dw, nd);
    } else if (!strcmp(op, "hmac")) wg::b2s::hmac(out, kw, dw, nd);
    else { wg::b2s::mac16_116(out, kw, dw); outn = 16; }
    const uint8_t *o = (const uint8_t *)out;
    for (int i = 0; i < outn; ++i) printf("%02x", o[i]);
    printf("\n");
  }
}
