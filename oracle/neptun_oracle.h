/*
 * neptun_oracle.h -- CPU restatement of NepTUN's data-path AEAD (TEST
 * INFRASTRUCTURE ONLY; see neptun_oracle.c header).  Status codes are
 * WireGuardError's variant index + 1 (neptun/src/noise/errors.rs:4-28), 0 = Ok.
 */
#ifndef NEPTUN_ORACLE_H
#define NEPTUN_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  NEPTUN_OK = 0,
  NEPTUN_ERR_DESTINATION_BUFFER_TOO_SMALL = 1,
  NEPTUN_ERR_INCORRECT_PACKET_LENGTH = 2,
  NEPTUN_ERR_WRONG_INDEX = 5,
  NEPTUN_ERR_INVALID_AEAD_TAG = 10,
  NEPTUN_ERR_INVALID_COUNTER = 11,
  NEPTUN_ERR_DUPLICATE_COUNTER = 12,
  NEPTUN_ERR_INVALID_PACKET = 13,
};

#define NEPTUN_MSG_DATA 4u            /* noise/mod.rs:86 */
#define NEPTUN_DATA_OFFSET 16u        /* session.rs:31 */
#define NEPTUN_AEAD_SIZE 16u          /* session.rs:33 */
#define NEPTUN_DATA_OVERHEAD_SZ 32u   /* noise/mod.rs:91 */

/* Same field meaning as wg_packet_desc in include/neptun_gpu.h. */
typedef struct {
  uint64_t src_off;
  uint64_t dst_off;
  uint64_t counter;
  uint32_t len;
  uint32_t key_slot;
} neptun_oracle_desc;

void neptun_oracle_chacha20_block(const uint8_t key[32], uint32_t block_counter,
                                  const uint8_t nonce[12], uint8_t out[64]);
void neptun_oracle_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]);
void neptun_oracle_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                             size_t aad_len, const uint8_t *pt, size_t len, uint8_t *ct,
                             uint8_t tag[16]);
int neptun_oracle_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t aad_len, const uint8_t *ct, size_t len, const uint8_t tag[16],
                            uint8_t *pt);
int neptun_oracle_format_packet_data(const uint8_t key[32], uint32_t sending_index,
                                     uint64_t counter, const uint8_t *payload, size_t payload_len,
                                     uint8_t *out, size_t out_cap);
int neptun_oracle_parse_data_header(const uint8_t *datagram, size_t len, uint32_t *receiver_idx,
                                    uint64_t *counter);
int neptun_oracle_receive_packet_data(const uint8_t key[32], uint32_t receiving_index,
                                      const uint8_t *datagram, size_t len, uint8_t *out,
                                      size_t out_cap, size_t *out_len);
void neptun_oracle_seal_batch(const neptun_oracle_desc *descs, size_t n, const uint8_t *keys,
                              const uint32_t *key_index, const uint8_t *src, uint8_t *dst,
                              int32_t *status);
void neptun_oracle_open_batch(const neptun_oracle_desc *descs, size_t n, const uint8_t *keys,
                              const uint32_t *key_index, const uint8_t *src, uint8_t *dst,
                              int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
