/*
 * neptun_gpu.h -- C ABI of the MI355X (gfx950) WireGuard transport-data AEAD.
 *
 * Drop-in boundary for NepTUN's per-packet ChaCha20-Poly1305 seal/open, i.e.
 * the bytes-hot part of Tunn::encapsulate / Tunn::decapsulate
 * (/root/reference/neptun/src/noise/mod.rs:295-380).  NepTUN exposes no C ABI
 * of its own; these entry points are what its Rust side binds
 * through `extern "C"` (INTEGRATION.md shows the binding).  Plain pointers and
 * sizes only: no HIP or torch types, the stream is an opaque `void *`
 * (a hipStream_t, NULL = the default stream).
 *
 * Semantics per packet are those of
 *   seal: Session::format_packet_data   session.rs:205-259
 *         header LE32 4 | LE32 sending_index | LE64 counter, nonce 0^4|LE64
 *         counter, empty AAD, ciphertext = plaintext length (no padding),
 *         16-byte tag right after it; wire length = len + 32.
 *   open: Tunn::parse_incoming_packet (DATA arm, noise/mod.rs:139-199) +
 *         Session::receive_packet_data session.rs:265-302 without the replay
 *         window (host-side, wg_replay_* in neptun_tunn.h): header checked (type 4,
 *         len >= 32, receiver_idx == the slot's receiving index), tag verified
 *         (ring open_in_place), plaintext written.  On a tag mismatch the
 *         plaintext bytes are zeroed (ring 0.17 open_within) and the status is
 *         InvalidAeadTag.
 *
 * Per-packet status codes are WireGuardError variant index + 1
 * (neptun/src/noise/errors.rs:4-28), 0 = Ok; ABI-level codes start at 100.
 *
 * Device-resident entry points take DEVICE pointers (src, dst, descs, status)
 * and are asynchronous on `stream`.  Layout requirement of the GPU path:
 * 16-byte alignment of every packet's plaintext and ciphertext start (seal:
 * src_off % 16 == 0 and dst_off % 16 == 0; open: src_off % 16 == 0 and
 * dst_off % 16 == 0).  A misaligned descriptor gets WG_STATUS_MISALIGNED.
 *
 * Thread safety: a context may be used from several host threads; key-table
 * updates are serialised internally and are stream-ordered against launches
 * issued on the same stream.
 */
#ifndef NEPTUN_GPU_H
#define NEPTUN_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WG_GPU_ABI_VERSION 1

/* ---- per-packet status: WireGuardError (errors.rs:4-28) index + 1 ------- */
enum wg_status {
  WG_STATUS_OK = 0,
  WG_STATUS_DESTINATION_BUFFER_TOO_SMALL = 1,
  WG_STATUS_INCORRECT_PACKET_LENGTH = 2,
  WG_STATUS_UNEXPECTED_PACKET = 3,
  WG_STATUS_WRONG_PACKET_TYPE = 4,
  WG_STATUS_WRONG_INDEX = 5,
  WG_STATUS_WRONG_KEY = 6,
  WG_STATUS_INVALID_TAI64N_TIMESTAMP = 7,
  WG_STATUS_WRONG_TAI64N_TIMESTAMP = 8,
  WG_STATUS_INVALID_MAC = 9,
  WG_STATUS_INVALID_AEAD_TAG = 10,
  WG_STATUS_INVALID_COUNTER = 11,
  WG_STATUS_DUPLICATE_COUNTER = 12,
  WG_STATUS_INVALID_PACKET = 13,
  WG_STATUS_NO_CURRENT_SESSION = 14,
  WG_STATUS_LOCK_FAILED = 15,
  WG_STATUS_CONNECTION_EXPIRED = 16,
  WG_STATUS_UNDER_LOAD = 17,
  WG_STATUS_CRYPTO_FAILED = 18,
  WG_STATUS_INVALID_LENGTH = 19,
  WG_STATUS_INVALID_INDEX = 20,
  WG_STATUS_RING_UNSPECIFIED_ERROR = 21,
  WG_STATUS_SYSTEM_TIME_ERROR = 22,
  /* ABI-level (not WireGuardError) */
  WG_STATUS_MISALIGNED = 100,   /* packet start not 16-byte aligned */
  WG_STATUS_BAD_KEY_SLOT = 101, /* key_slot >= context key slots */
};

/* ---- call-level return codes ------------------------------------------- */
enum wg_rc {
  WG_RC_OK = 0,
  WG_RC_INVALID_ARGUMENT = -1,
  WG_RC_HIP_ERROR = -2,
  WG_RC_OUT_OF_MEMORY = -3,
  WG_RC_NO_DEVICE = -4,
};

/* NepTUN wire constants */
#define WG_MSG_DATA 4u              /* noise/mod.rs:86  DATA */
#define WG_DATA_OFFSET 16u          /* session.rs:31    DATA_OFFSET */
#define WG_AEAD_SIZE 16u            /* session.rs:33    AEAD_SIZE */
#define WG_DATA_OVERHEAD_SZ 32u     /* noise/mod.rs:91  DATA_OVERHEAD_SZ */

/*
 * One packet of a batch (32 bytes, device memory for the *_batch calls).
 *   seal: plaintext at src + src_off (len bytes); wire packet (len + 32 bytes)
 *         written at dst + dst_off; counter = the sending counter the host
 *         reserved (Session::sending_key_counter.fetch_add, session.rs:219).
 *   open: datagram (header | ciphertext | tag, len bytes, len >= 32) at
 *         src + src_off; plaintext (len - 32 bytes) written at dst + dst_off;
 *         counter is ignored (parsed from the header on the device).
 *   key_slot: index into the context key table (seal: the session's sending
 *         key; open: its receiving key).
 */
typedef struct wg_packet_desc {
  uint64_t src_off;
  uint64_t dst_off;
  uint64_t counter;
  uint32_t len;
  uint32_t key_slot;
} wg_packet_desc;

typedef struct wg_gpu_ctx wg_gpu_ctx;

/* ABI version (WG_GPU_ABI_VERSION). */
int wg_gpu_abi_version(void);

/* Build id: the first 16 hex digits of the SHA-256 of the sources the library was
 * built from (neptun_amd/csrc/Makefile SRC_FILES); loaders compare it with the tree. */
const char *wg_gpu_build_id(void);

/* Last error message of the calling thread ("" if none). */
const char *wg_gpu_last_error(void);

/*
 * Context = one GPU + a device-resident key table of `key_slots` entries
 * (32-byte ChaCha20 key + the session index that goes with it).  Replaces
 * Session::new's UnboundKey/LessSafeKey setup (session.rs:160-180): the keys a
 * handshake derives (handshake.rs:694, :948) are uploaded with wg_gpu_set_keys.
 */
int wg_gpu_ctx_create(int device, uint32_t key_slots, wg_gpu_ctx **out);
/* Destroy the Tunns, engines and pipes made on a context before the context
 * (they refer to it); the Python mirror's GpuContext.close() does so itself. */
int wg_gpu_ctx_destroy(wg_gpu_ctx *ctx);
uint32_t wg_gpu_ctx_key_slots(const wg_gpu_ctx *ctx);

/*
 * Upload keys[n][32] and indices[n] (HOST memory) into slots
 * [first_slot, first_slot + n).  indices[i] is the session index checked or
 * written with that key: for a sending-key slot the peer's index written into
 * the header (Session::sending_index, session.rs:226); for a receiving-key
 * slot our local index every datagram must carry (Session::receiving_index,
 * session.rs:275-277).  Stream-ordered on `stream`; returns after the copy is
 * enqueued (host buffers may be reused on return).
 */
int wg_gpu_set_keys(wg_gpu_ctx *ctx, uint32_t first_slot, uint32_t n, const uint8_t *keys,
                    const uint32_t *indices, void *stream);

/* Batch seal / open over device-resident descriptors (see wg_packet_desc).
 * src / dst may be NULL: the descriptor offsets are then absolute device
 * addresses (e.g. of mapped, registered host memory). */
int wg_gpu_seal_batch(wg_gpu_ctx *ctx, const wg_packet_desc *descs, uint32_t n,
                      const uint8_t *src, uint8_t *dst, int32_t *status, void *stream);
int wg_gpu_open_batch(wg_gpu_ctx *ctx, const wg_packet_desc *descs, uint32_t n,
                      const uint8_t *src, uint8_t *dst, int32_t *status, void *stream);

/*
 * Mixed-length batches.  The kernels run one packet per wavefront lane, so a
 * wave costs as much as its longest packet; wg_gpu_plan_batch writes a
 * permutation `order` (n device uint32) grouping packets by length, longest
 * first (a device counting sort; `scratch` = WG_PLAN_SCRATCH_BYTES of device
 * memory, private to the call until it completes on `stream`).  The _ordered
 * calls process descs[order[i]] and write status[order[i]] -- the results are
 * identical to the unordered calls, only the scheduling differs.  `seal` != 0
 * plans for a seal (datagram = len + 32), 0 for an open.
 */
#define WG_PLAN_SCRATCH_BYTES 262144u
int wg_gpu_plan_batch(wg_gpu_ctx *ctx, int seal, const wg_packet_desc *descs, uint32_t n,
                      uint32_t *order, uint32_t *scratch, void *stream);
int wg_gpu_seal_batch_ordered(wg_gpu_ctx *ctx, const wg_packet_desc *descs,
                              const uint32_t *order, uint32_t n, const uint8_t *src,
                              uint8_t *dst, int32_t *status, void *stream);
int wg_gpu_open_batch_ordered(wg_gpu_ctx *ctx, const wg_packet_desc *descs,
                              const uint32_t *order, uint32_t n, const uint8_t *src,
                              uint8_t *dst, int32_t *status, void *stream);

/*
 * Uniform batch: n packets of one session, all `len` bytes, packet i at
 * src + i*src_stride / dst + i*dst_stride.  Seal uses counter
 * counter_base + i (one fetch_add(n) per batch instead of per packet,
 * session.rs:219) -- the nonce is derived from the lane index.  Open parses
 * each header.  Strides and base pointers must be multiples of 16.
 * `status` may be NULL (no per-packet status written).
 */
int wg_gpu_seal_strided(wg_gpu_ctx *ctx, uint32_t n, uint32_t len, uint32_t key_slot,
                        uint64_t counter_base, const uint8_t *src, uint64_t src_stride,
                        uint8_t *dst, uint64_t dst_stride, int32_t *status, void *stream);
int wg_gpu_open_strided(wg_gpu_ctx *ctx, uint32_t n, uint32_t len, uint32_t key_slot,
                        const uint8_t *src, uint64_t src_stride, uint8_t *dst,
                        uint64_t dst_stride, int32_t *status, void *stream);

/*
 * Slot padding (strided calls; new, no reference counterpart).  Default 0: no
 * byte outside a packet's output is written.  With writable != 0 the caller
 * declares the rest of every output slot scratch: when the output slots start
 * on 128-byte boundaries (seal: dst; open: the 128-byte run grid's origin) and
 * the stride is a multiple of 128, the kernels zero-fill each output from its
 * end to the next 128-byte boundary -- never past the slot -- and an open whose
 * plaintext sits 16 bytes into its slot also zero-fills those 16 bytes, so every
 * HBM line they write is written whole (no partial-line merge).
 * Results are otherwise identical.  Applies to later calls on the context.
 */
int wg_gpu_ctx_set_slot_padding(wg_gpu_ctx *ctx, int writable);

/*
 * Latency form of the descriptor batches (new, no reference counterpart; NepTUN's
 * inter-thread batches hold at most 50 packets, packet_workers.rs:27).  A batch of
 * n packets with n * G <= `lanes` runs G lanes per packet -- the largest G of 64,
 * 32, ..., 2 that fits -- instead of one packet per lane: the keystream blocks are
 * spread over the group and the Poly1305 partial sums combined with powers of r,
 * so a small batch takes about as long as one packet's share of blocks.  lanes = 0
 * turns it off; lanes < 0 restores the default (WG_XLANE_LANES from the
 * environment, else 256 per compute unit).  Results are identical either way.
 * Applies to later wg_gpu_seal_batch / wg_gpu_open_batch (and _ordered) calls.
 */
int wg_gpu_ctx_set_xlane_lanes(wg_gpu_ctx *ctx, int64_t lanes);

/*
 * Split waves of the uniform strided batches (new; BASELINE's AEAD bench size 8192 B,
 * chacha20poly1305_benching.rs:37-55): a batch whose waves of 64 packets fill only part
 * of the chip runs each wave as `parts` jobs over consecutive rounds of its packets,
 * and a finish kernel combines their Poly1305 sums (tags, checks, statuses).  parts
 * < 0: the library's choice (a fill model, WG_SPLIT_K from the environment overrides);
 * 1: never; 2 .. 8: that many where every part keeps at least 8 of the packets'
 * keystream rounds (else unsplit; part 0 takes the rounds the count does not divide).
 * Results are identical either way.
 */
int wg_gpu_ctx_set_split(wg_gpu_ctx *ctx, int parts);

/*
 * The parts (>= 1; 1 = unsplit) a strided batch of n packets of `len` input bytes
 * would run its full waves in, on the throughput form (batches that take the latency
 * form are never split).  For tools and benches: the kernels a launch makes.
 */
int wg_gpu_strided_split_parts(wg_gpu_ctx *ctx, int seal, uint32_t n, uint32_t len);

/*
 * Handshake-side crypto, batched.  Device pointers,
 * asynchronous on `stream`.
 *   wg_gpu_x25519_batch: out[i] = X25519(scalars[i], points[i]) (RFC 7748;
 *     x25519-dalek's StaticSecret::diffie_hellman / PublicKey::from with the
 *     base point 9), 32 bytes each, no rejection of all-zero results (neither
 *     does the reference).
 *   wg_gpu_handshake_anon_batch: for n handshake initiations (148 bytes each,
 *     `stride` apart, stride % 4 == 0) the responder-side work before the peer
 *     is known: the mac1 check of RateLimiter::verify_packet
 *     (rate_limiter.rs:187-195, when check_mac1 != 0) and parse_handshake_anon
 *     (noise/handshake.rs:367-412).  out[i] gets the sender index and the
 *     initiator's static public key (HalfHandshake) or a status:
 *     WG_STATUS_WRONG_PACKET_TYPE, WG_STATUS_INVALID_MAC, WG_STATUS_INVALID_AEAD_TAG.
 *     static_private (32 bytes) is HOST memory.
 */
typedef struct wg_half_handshake {
  uint32_t peer_index;
  int32_t status;
  uint8_t peer_static_public[32];
} wg_half_handshake;

int wg_gpu_x25519_batch(wg_gpu_ctx *ctx, uint32_t n, const uint8_t *scalars, const uint8_t *points,
                        uint8_t *out, void *stream);
int wg_gpu_handshake_anon_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32], uint32_t n,
                                const uint8_t *msgs, uint64_t stride, int check_mac1,
                                wg_half_handshake *out, void *stream);

/*
 * Responder side, batched.  The reference's
 * receive_handshake_initialization (noise/handshake.rs:527-613) holds two
 * pieces of sequential per-peer state: the last TAI64N timestamp (replay
 * check, :592-596) and next_index (inc_index, :508-513, consumed by
 * format_handshake_response :853-949).  The batch API splits there:
 *   1. wg_gpu_handshake_consume_batch: the crypto of
 *      receive_handshake_initialization for n initiations whose peer the
 *      caller has identified (parse_handshake_anon / its peer table): DH,
 *      HASH/HMAC chain, AEAD-open of the static key (compared with the
 *      peer's: WG_STATUS_WRONG_KEY) and of the timestamp.  out[i] is the
 *      InitReceived state + the decrypted timestamp, or a status
 *      (WRONG_PACKET_TYPE, INVALID_AEAD_TAG, WRONG_KEY).
 *   2. the caller, in packet order: wg_handshake_timestamp_after (else
 *      WrongTai64nTimestamp), last timestamp update, inc_index().
 *   3. wg_gpu_handshake_respond_batch: format_handshake_response +
 *      append_mac1_and_mac2 (:732-765) from the states: the 92-byte response
 *      and the session keys (Session::new(local, peer, temp2, temp3), :948).
 *      Entries whose state status != 0 are skipped (message zeroed).
 * Under load (RateLimiter::verify_packet, rate_limiter.rs:197-218):
 *   wg_gpu_mac2_check_batch: cookie = MAC(secret, LE64(counter) || addr) and the
 *     mac2 check of each handshake message (len 148 or 92); status 0 valid,
 *     1 = answer with a cookie reply; the cookie is returned.  Any other length
 *     is not a handshake message (parse_incoming_packet rejects it): status
 *     WG_STATUS_INVALID_PACKET, cookie zeroed, nothing of the message read.
 *   wg_gpu_cookie_reply_batch: format_cookie_reply (rate_limiter.rs:133-170):
 *     nonce = b2s_mac_24(nonce_key, LE64(nonce_ctr)) (the caller hands out
 *     nonce_ctr in reply order, :112-121), XChaCha20-Poly1305(cookie_key, nonce,
 *     aad = mac1, cookie) -> 64-byte COOKIE_REPLY messages.
 * Device pointers for the arrays, host pointers for the 16/32-byte keys.
 */
typedef struct wg_responder_peer {
  uint8_t peer_static_public[32];  /* NoiseParams::peer_static_public */
  uint8_t static_shared[32];       /* NoiseParams::static_shared = DH(static_private, peer_static_public) */
} wg_responder_peer;

typedef struct wg_init_received {  /* HandshakeState::InitReceived + the timestamp */
  int32_t status;
  uint32_t peer_index;
  uint8_t timestamp[12];           /* TAI64N, big-endian seconds then nanoseconds */
  uint8_t chaining_key[32];
  uint8_t hash[32];
  uint8_t peer_ephemeral[32];
  uint8_t pad[12];
} wg_init_received;                /* 128 bytes */

typedef struct wg_response_job {
  uint8_t ephemeral_private[32];   /* DH_GENERATE() (random, from the caller) */
  uint8_t peer_static_public[32];
  uint8_t preshared_key[32];       /* zeros when the peer has none (handshake.rs:920) */
  uint8_t mac1_key[32];            /* HASH(LABEL_MAC1 || peer_static_public) */
  uint8_t cookie[16];              /* cookies.write_cookie, when has_cookie */
  uint32_t local_index;            /* inc_index() */
  uint32_t has_cookie;
  uint8_t pad[8];
} wg_response_job;                 /* 160 bytes */

typedef struct wg_response_out {
  uint8_t message[92];             /* HANDSHAKE_RESP incl. mac1 / mac2 */
  uint8_t pad[4];
  uint8_t receiving_key[32];       /* temp2 */
  uint8_t sending_key[32];         /* temp3 */
  uint8_t mac1[16];                /* cookies.last_mac1 */
} wg_response_out;                 /* 176 bytes */

typedef struct wg_cookie_reply_job {
  uint8_t cookie[16];
  uint8_t mac1[16];                /* mac1 of the message being answered (the AAD) */
  uint64_t nonce_ctr;
  uint32_t receiver_idx;           /* the message's sender index */
  uint32_t pad;
} wg_cookie_reply_job;             /* 48 bytes */

int wg_gpu_handshake_consume_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32], uint32_t n,
                                   const uint8_t *msgs, uint64_t stride,
                                   const wg_responder_peer *peers, wg_init_received *out,
                                   void *stream);
/* Tai64N::after (handshake.rs:267-269): 1 if ts is strictly later than last */
int wg_handshake_timestamp_after(const uint8_t ts[12], const uint8_t last[12]);
int wg_gpu_handshake_respond_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_init_received *states,
                                   const wg_response_job *jobs, wg_response_out *out, void *stream);
int wg_gpu_mac2_check_batch(wg_gpu_ctx *ctx, const uint8_t secret_key[16], uint64_t cookie_counter,
                            uint32_t n, const uint8_t *msgs, uint64_t stride, const uint32_t *lens,
                            const uint8_t *addrs, uint8_t *cookies, int32_t *status, void *stream);
int wg_gpu_cookie_reply_batch(wg_gpu_ctx *ctx, const uint8_t cookie_key[32],
                              const uint8_t nonce_key[32], uint32_t n,
                              const wg_cookie_reply_job *jobs, uint8_t *out, void *stream);

/*
 * Initiator side, batched.  The reference's sequential
 * per-peer state stays with the caller: inc_index() for each initiation, the
 * InitSent / previous-state match of a response by its receiver index
 * (handshake.rs:619-624, else UnexpectedPacket), and cookies.index /
 * last_mac1 for cookie replies (:701-709, else UnexpectedPacket / WrongIndex).
 *   wg_gpu_handshake_initiate_batch: format_handshake_initiation
 *     (noise/handshake.rs:769-851) + append_mac1_and_mac2 (:732-765) with the
 *     caller's random ephemeral key and TAI64N stamp: the 148-byte message and
 *     the InitSent state (chaining key, hash; the ephemeral key stays with the
 *     caller) and mac1 (cookies.last_mac1).
 *   wg_gpu_handshake_receive_response_batch: receive_handshake_response
 *     (:615-695) for n 92-byte responses (`stride` apart, stride % 4 == 0),
 *     after the mac1 check of RateLimiter::verify_packet (rate_limiter.rs:182-195,
 *     when check_mac1 != 0; the key is derived from static_private).  out[i]:
 *     the session keys -- Session::new(local, peer, temp3, temp2): sending =
 *     temp2, receiving = temp3 -- and the responder's sender index, or a status
 *     (WRONG_PACKET_TYPE, INVALID_MAC, INVALID_AEAD_TAG; keys zeroed).
 *     static_private (32 bytes) is HOST memory.
 *   wg_gpu_cookie_reply_open_batch: the decryption of receive_cookie_reply
 *     (:711-724): XChaCha20-Poly1305 open of the cookie with key
 *     HASH(LABEL_COOKIE || responder static public), aad = last mac1.  out[i]:
 *     the cookie (cookies.write_cookie) or WRONG_PACKET_TYPE / INVALID_AEAD_TAG.
 * Device pointers for the arrays.
 */
typedef struct wg_initiation_job {
  uint8_t ephemeral_private[32];   /* DH_GENERATE() (random, from the caller) */
  uint8_t static_public[32];       /* NoiseParams::static_public */
  uint8_t peer_static_public[32];
  uint8_t static_shared[32];       /* NoiseParams::static_shared = DH(static_private, peer_static_public) */
  uint8_t mac1_key[32];            /* sending_mac1_key = HASH(LABEL_MAC1 || peer_static_public) */
  uint8_t cookie[16];              /* cookies.write_cookie, when has_cookie */
  uint8_t timestamp[12];           /* TAI64N stamp: big-endian seconds then nanoseconds */
  uint32_t local_index;            /* inc_index() */
  uint32_t has_cookie;
  uint8_t pad[12];
} wg_initiation_job;               /* 208 bytes */

typedef struct wg_init_sent {      /* HandshakeState::InitSent (+ the message and last mac1) */
  uint8_t message[148];            /* HANDSHAKE_INIT incl. mac1 / mac2 */
  uint32_t local_index;
  uint8_t chaining_key[32];
  uint8_t hash[32];
  uint8_t mac1[16];                /* cookies.last_mac1 */
} wg_init_sent;                    /* 232 bytes */

typedef struct wg_response_received_job {
  uint8_t chaining_key[32];        /* the matched InitSent state */
  uint8_t hash[32];
  uint8_t ephemeral_private[32];
  uint8_t preshared_key[32];       /* zeros when the peer has none (handshake.rs:657-661) */
} wg_response_received_job;        /* 128 bytes */

typedef struct wg_session_keys {
  int32_t status;
  uint32_t peer_index;             /* the response's sender index */
  uint8_t sending_key[32];         /* temp2 */
  uint8_t receiving_key[32];       /* temp3 */
  uint32_t receiver_idx;           /* the response's receiver index (0 on WrongPacketType): jobs[i]
                                      must be the InitSent state of that local index -- the caller
                                      checks it (receive_handshake_response, handshake.rs:620-630) */
  uint32_t pad;
} wg_session_keys;                 /* 80 bytes */

typedef struct wg_cookie_open_job {
  uint8_t message[64];             /* COOKIE_REPLY */
  uint8_t cookie_key[32];          /* HASH(LABEL_COOKIE || responder static public) */
  uint8_t mac1[16];                /* cookies.last_mac1 */
} wg_cookie_open_job;              /* 112 bytes */

typedef struct wg_cookie_open_out {
  int32_t status;
  uint32_t receiver_idx;           /* the reply's receiver index (the caller compares cookies.index) */
  uint8_t cookie[16];
} wg_cookie_open_out;              /* 24 bytes */

int wg_gpu_handshake_initiate_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_initiation_job *jobs,
                                    wg_init_sent *out, void *stream);
int wg_gpu_handshake_receive_response_batch(wg_gpu_ctx *ctx, const uint8_t static_private[32],
                                            uint32_t n, const uint8_t *msgs, uint64_t stride,
                                            int check_mac1, const wg_response_received_job *jobs,
                                            wg_session_keys *out, void *stream);
int wg_gpu_cookie_reply_open_batch(wg_gpu_ctx *ctx, uint32_t n, const wg_cookie_open_job *jobs,
                                   wg_cookie_open_out *out, void *stream);

/*
 * Host memory registration (hipHostRegister, mapped) for copy-free batches:
 * the kernels can then address the caller's buffers directly (absolute
 * device addresses in descriptors with NULL src / dst bases, or the Tunn
 * direct path in neptun_tunn.h).  Ranges must not overlap; wg_gpu_ctx_destroy
 * releases any left.  wg_gpu_unregister_host waits for the device first.
 */
int wg_gpu_register_host(wg_gpu_ctx *ctx, void *base, uint64_t bytes);
int wg_gpu_unregister_host(wg_gpu_ctx *ctx, void *base);
/* device address of registered host memory [host, host + bytes): 0 on success */
int wg_gpu_host_device_address(wg_gpu_ctx *ctx, const void *host, uint64_t bytes, uint64_t *dev);

/*
 * Inbound routing on the device.  NepTUN routes a DATA
 * datagram by its receiver index: the device picks the peer by
 * receiver_idx >> 8 (device/mod.rs:1022-1024) and the peer's Tunn the session
 * sessions[receiver_idx % 8] (noise/mod.rs:550-556).  Here one HBM table maps
 * every live receiving index straight to the key slot holding that session's
 * receiving key, so a batch of raw datagrams needs no host pre-pass:
 *   wg_gpu_route_set   replaces the table (host arrays; n <= 2^22 entries);
 *   wg_gpu_route_batch reads each descriptor's datagram header on the device
 *                      (src + src_off, descs[i].len bytes) and writes
 *                      descs[i].key_slot: the session's slot, or
 *                      WG_KEY_SLOT_INVALID_PACKET when parse_incoming_packet
 *                      would not yield a DATA packet (len < 32 or type != 4,
 *                      mod.rs:139-199) or WG_KEY_SLOT_NO_SESSION when no
 *                      session has that receiving index.
 * The open kernels turn the two sentinels into WG_STATUS_INVALID_PACKET and
 * WG_STATUS_NO_CURRENT_SESSION (in the reference's check order); the seal
 * kernels treat them like any out-of-table slot.
 */
#define WG_KEY_SLOT_NO_SESSION 0xFFFFFFFFu
#define WG_KEY_SLOT_INVALID_PACKET 0xFFFFFFFEu
int wg_gpu_route_set(wg_gpu_ctx *ctx, uint32_t n, const uint32_t *receiver_idx,
                     const uint32_t *key_slot);
int wg_gpu_route_batch(wg_gpu_ctx *ctx, wg_packet_desc *descs, uint32_t n, const uint8_t *src,
                       void *stream);

/*
 * Host-resident batches (the real data path: TUN read buffers in, UDP send
 * buffers out and vice versa).  A pipe owns `depth` streams and device staging
 * buffers of `chunk_bytes` each; a call splits the batch into chunks and runs
 * H2D copy -> kernel -> D2H copy per chunk, chunks round-robin over the
 * streams so copies in both directions overlap the kernels.  Host buffers
 * should be pinned (hipHostMalloc / cudaHostRegister-equivalent) for the copies
 * to overlap.  Only the packet bytes are copied back (2-D copies of `len` or
 * `len + 32` bytes at `dst_stride`); the calls return when every chunk is done.
 * Semantics are those of wg_gpu_seal_strided / wg_gpu_open_strided; packet i is
 * at h_src + i*src_stride / h_dst + i*dst_stride, status (may be NULL) in host
 * memory.  A pipe is not thread-safe: one pipe per calling thread.
 */
typedef struct wg_gpu_pipe wg_gpu_pipe;
int wg_gpu_pipe_create(wg_gpu_ctx *ctx, uint64_t chunk_bytes, uint32_t depth, wg_gpu_pipe **out);
int wg_gpu_pipe_destroy(wg_gpu_pipe *pipe);
int wg_gpu_pipe_seal_strided(wg_gpu_pipe *pipe, uint32_t n, uint32_t len, uint32_t key_slot,
                             uint64_t counter_base, const uint8_t *h_src, uint64_t src_stride,
                             uint8_t *h_dst, uint64_t dst_stride, int32_t *h_status);
int wg_gpu_pipe_open_strided(wg_gpu_pipe *pipe, uint32_t n, uint32_t len, uint32_t key_slot,
                             const uint8_t *h_src, uint64_t src_stride, uint8_t *h_dst,
                             uint64_t dst_stride, int32_t *h_status);

#ifdef __cplusplus
}
#endif
#endif /* NEPTUN_GPU_H */
