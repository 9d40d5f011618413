/*
 * neptun_tunn.h -- batched Tunn data plane over the GPU AEAD (C ABI).
 *
 * Mirrors the data-packet part of neptun::noise::Tunn so that one batch call
 * returns exactly what N sequential Tunn::encapsulate / Tunn::decapsulate
 * calls would (/root/reference/neptun/src/noise/mod.rs:295-380, 545-569,
 * 606-670; session.rs:40-302):
 *   encapsulate: sessions[current % 8] (mod.rs:310), dst capacity check
 *     (session.rs:210-217: IncorrectPacketLength, no counter consumed), one
 *     sending-counter reservation per batch (session.rs:219 fetch_add),
 *     tx_bytes += P + 32 (mod.rs:321) -> WriteToNetwork(P + 32).
 *   decapsulate: parse_incoming_packet (mod.rs:139-199), session
 *     sessions[receiver_idx % 8] (mod.rs:550-556, NoCurrentSession),
 *     receive_packet_data checks in the reference order -- dst capacity
 *     (DestinationBufferTooSmall), receiver index (WrongIndex), replay quick
 *     check (InvalidCounter / DuplicateCounter), tag (InvalidAeadTag), replay
 *     mark -- then validate_decapsulated_packet (mod.rs:606-670: keepalive ->
 *     Done, IPv4/IPv6 length truncation, InvalidPacket) and rx_bytes.
 * Handshake / cookie messages are not the data path: such datagrams come back
 * as WG_TUNN_NOT_DATA for the caller's CPU Tunn.  Of the timers (timers.rs)
 * only what the data plane reads is mirrored: timers[TimeCurrent] (set by the
 * caller, wg_tunn_set_time) and the per-ring-slot session_timers that
 * set_current_session compares (mod.rs:528-542); rekey / keepalive / expiry
 * stay with the caller's CPU Tunn.
 *
 * The replay window (session.rs:40-157) is exposed on its own (wg_replay_*)
 * for tests and for embedders that keep their own sessions.
 */
#ifndef NEPTUN_TUNN_H
#define NEPTUN_TUNN_H

#include <stddef.h>
#include <stdint.h>

#include "neptun_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define WG_N_SESSIONS 8          /* noise/mod.rs:47 */
#define WG_REPLAY_WORDS 16       /* session.rs:37 N_WORDS (1024-bit window) */

/* ReceivingKeyCounterValidator (session.rs:40-48) */
typedef struct wg_replay {
  uint64_t next;
  uint64_t receive_cnt;
  uint64_t bitmap[WG_REPLAY_WORDS];
} wg_replay;

void wg_replay_init(wg_replay *w);
/* will_accept (session.rs:90-104): 0, WG_STATUS_INVALID_COUNTER or WG_STATUS_DUPLICATE_COUNTER */
int wg_replay_will_accept(const wg_replay *w, uint64_t counter);
/* mark_did_receive (session.rs:109-156): 0 or WG_STATUS_INVALID_COUNTER; does not touch receive_cnt */
int wg_replay_mark_did_receive(wg_replay *w, uint64_t counter);

enum wg_tunn_kind {
  WG_TUNN_DONE = 0,              /* TunnResult::Done (keepalive) */
  WG_TUNN_ERR = 1,               /* TunnResult::Err(status) */
  WG_TUNN_WRITE_TO_NETWORK = 2,  /* datagram of `len` bytes at dst */
  WG_TUNN_WRITE_TO_TUNNEL = 3,   /* IP packet of `len` bytes at dst, source address src_ip */
  WG_TUNN_NOT_DATA = 4,          /* handshake / cookie message: hand it to the CPU Tunn */
};

typedef struct wg_tunn_result {
  int32_t kind;        /* wg_tunn_kind */
  int32_t status;      /* wg_status when kind == WG_TUNN_ERR, else 0 */
  uint32_t len;
  uint8_t ip_version;  /* 4 or 6 for WG_TUNN_WRITE_TO_TUNNEL */
  uint8_t src_ip[16];  /* IPv4 in the first 4 bytes */
  uint8_t pad[3];
} wg_tunn_result;

typedef struct wg_tunn wg_tunn;

/* Engine: the device side the Tunns of one GPU share -- the host copy pool, the
 * HIP streams and the pinned / device staging their batches run on.  NepTUN
 * keeps one Tunn per peer (device/peer.rs:29, Mutex<Tunn>) and its PacketWorkers
 * serve all peers from one set of worker threads (device/packet_workers.rs:99-287);
 * so here any number of Tunns attach to one engine without adding a thread or a
 * stream.  A batch call borrows one of the engine's lanes (a staging pipeline:
 * streams + staging sets; created on first need, at most WG_ENGINE_LANES,
 * default 8) for its duration; calls on different Tunns run concurrently up to
 * that many, then wait for a lane.  The pool's threads (WG_TUNN_THREADS, default
 * the CPUs this process may use, at most 16) are the engine's, shared by its
 * lanes: a call that finds the pool busy runs its host steps on its own thread.
 *   wg_engine_create / wg_engine_destroy: an engine on ctx (destroy fails while
 *     Tunns are attached);
 *   wg_tunn_create_on: a Tunn attached to engine e.
 * wg_tunn_create(ctx, ...) attaches to the context's default engine (made with
 * the context's first such Tunn, destroyed with its last). */
typedef struct wg_engine wg_engine;
int wg_engine_create(wg_gpu_ctx *ctx, wg_engine **out);
int wg_engine_destroy(wg_engine *e);
int wg_tunn_create_on(wg_engine *e, uint32_t first_slot, wg_tunn **out);
/* what an engine holds: attached Tunns, lanes made so far, pool threads (incl. the
 * calling thread's share: workers + 1), HIP streams made so far (lanes' only), and
 * how many small calls' chunks went out in a launch shared with another concurrent
 * call (WG_COMBINE=1, off by default: one latency-form launch for the engine's
 * concurrent small calls of one direction, at most WG_COMBINE_DEPTH such launches in
 * flight, default 2); how many small calls' chunks were served by the engine's
 * resident kernel instead of a launch of their own (WG_TUNN_SRV=1, off by default:
 * chunks of up to 64 packets whose completion is the kernel's word; while it runs,
 * hipDeviceSynchronize and hipFree in the process wait for it to go idle) and how
 * many times that kernel was launched (a lease of 1 s, renewed by the next call; a
 * new launch after a key-table update or an idle stop) */
typedef struct wg_engine_info {
  uint32_t tunns, lanes, max_lanes, pool_threads, streams;
  uint32_t combined;
  uint64_t served, service_launches;
} wg_engine_info;
int wg_engine_get_info(const wg_engine *e, wg_engine_info *out);
/* the engine a Tunn is attached to (NULL: a multi-GPU Tunn with private engines) */
wg_engine *wg_tunn_engine(const wg_tunn *t);

/* A Tunn bound to a GPU context's default engine; it uses key slots
 * [first_slot, first_slot + 16). */
int wg_tunn_create(wg_gpu_ctx *ctx, uint32_t first_slot, wg_tunn **out);
int wg_tunn_destroy(wg_tunn *t);

/* A Tunn whose batches are spread over several GPU contexts (normally one per
 * GPU; several on one GPU are allowed, e.g. for tests).  Session keys are
 * installed on every context (same key slots).  A batch reserves its sending
 * counters once (session.rs:219) and is then split into contiguous,
 * byte-balanced shares, one per context, that run concurrently -- each on its
 * own host driver thread, copy threads, streams and pinned staging, bound to
 * the GPU's NUMA node; no data is exchanged between GPUs.  Decapsulate
 * decisions (replay window, validation, stats) are still taken in packet
 * order, after the shares are back.  Results equal the single-context Tunn's. */
#define WG_TUNN_MAX_ENGINES 64
int wg_tunn_create_multi(wg_gpu_ctx *const *ctxs, uint32_t nctx, uint32_t first_slot,
                         wg_tunn **out);
uint32_t wg_tunn_engines(const wg_tunn *t);
/* the HIP device and NUMA node (-1: unknown / not bound) of engine e */
int wg_tunn_engine_info(const wg_tunn *t, uint32_t engine, int *device, int *numa_node);

/* Session::new(local_index, peer_index, receiving_key, sending_key) stored at
 * sessions[local_index % 8] (mod.rs:449-452, 477-481) with session timer =
 * the Tunn's current time; make_current != 0 then runs set_current_session
 * (mod.rs:528-542). */
int wg_tunn_install_session(wg_tunn *t, uint32_t local_index, uint32_t peer_index,
                            const uint8_t receiving_key[32], const uint8_t sending_key[32],
                            int make_current);
int wg_tunn_stats(const wg_tunn *t, uint64_t *tx_bytes, uint64_t *rx_bytes);
/* timers[TimeCurrent] = now (update_timers, timers.rs:228-233; any monotonic
 * unit, e.g. ns since the Tunn was created).  wg_tunn_install_session records
 * it as the ring slot's session timer (timer_tick_session_established,
 * timers.rs:173-185); set_current_session switches to a session only if the
 * current slot is empty or its timer is not newer (mod.rs:528-542).  Default 0. */
int wg_tunn_set_time(wg_tunn *t, uint64_t now);

/* Registered (copy-free) batches: when the caller's buffers are registered with
 * wg_gpu_register_host (include/neptun_gpu.h), no host thread copies packet bytes:
 * see "Data movement" below.  Results are identical either way.
 *
 * Data movement.  A batch flows in chunks (WG_TUNN_CHUNK_KB, default 16 MiB) through
 * WG_TUNN_SETS staging sets (default 2; a registered batch whose first chunk takes the
 * scatter below uses 4).  Registered buffers (one engine): the inputs
 * go to HBM as 2D copy-engine runs straight from the caller's memory (on their own
 * stream, under the previous chunk's kernel; WG_TUNN_DMA_STREAMS=0: one stream), the
 * AEAD kernel reads them in HBM and its descriptors / statuses in pinned memory, and
 * the outputs reach the caller's registered destinations either from the AEAD kernel
 * itself (decapsulate: on per-chunk speculated replay decisions, repaired after the
 * real in-order pass) or through a scatter kernel: by default the kernel where its
 * 128-byte output runs sit on whole lines of host memory -- encapsulate's datagram at a
 * 128-byte boundary, decapsulate's plaintext 16 bytes past one -- and the scatter
 * elsewhere; WG_TUNN_DMA_OUT=direct|scatter forces either (direct needs 16-byte-aligned
 * destinations).  A decapsulate batch of 16,384 packets or more starts its first chunk after
 * pass 1 of its first sixteenth.  WG_TUNN_DMA=0 instead has the AEAD kernels
 * read -- and, for encapsulate with 16-byte-aligned buffers, write -- the caller's
 * registered memory directly over PCIe.  Other buffers: the host copies packets into pinned
 * staging (streaming stores, WG_TUNN_NT=0 for memcpy) on a pool of WG_TUNN_THREADS
 * threads (default: the CPUs this process may use, at most 16; they spin
 * WG_TUNN_SPIN_US, default 20, before blocking between steps), the kernels read and
 * write that staging over PCIe (WG_TUNN_ZEROCOPY=0: explicit copies to and from
 * HBM instead), and the pool copies the results out.
 * A batch call that returns an error leaves every selected packet's result at
 * ERR CryptoFailed unless its chunk completed; the destination bytes of such
 * packets are unspecified (a registered decapsulate may already have written a
 * plaintext there on a speculated replay decision). */
/* sending counter of the current session / replay state of a ring slot (for tests) */
int wg_tunn_session_counters(const wg_tunn *t, uint32_t ring_slot, uint64_t *sending_counter,
                             wg_replay *window);

/* n x Tunn::encapsulate(src[i][..src_len[i]], dst[i][..dst_cap[i]]) with host buffers */
int wg_tunn_encapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *src,
                              const uint32_t *src_len, uint8_t *const *dst,
                              const uint32_t *dst_cap, wg_tunn_result *res);
/* n x Tunn::decapsulate(None, datagram[i][..len[i]], dst[i][..dst_cap[i]]) */
int wg_tunn_decapsulate_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                              const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                              wg_tunn_result *res);
/* Multi-peer batches: packet i belongs to tunn[i] (any mix of the engine's
 * Tunns, in any order) -- the inter-thread batch of NepTUN's PacketWorkers, whose
 * entries each carry their own peer (packet_workers.rs:178-205) and are then
 * encapsulated one by one under that peer's Tunn lock (:207-233, device/mod.rs:
 * 1328-1337).  The results equal the sequential calls tunn[i]->encapsulate /
 * decapsulate in packet order: each Tunn's sending counters are handed out in
 * the order of its packets, its replay window and set_current_session see its
 * packets in order, tx_bytes / rx_bytes go to the packet's Tunn.  Every tunn[i]
 * must be attached to `e` (else WG_RC_INVALID_ARGUMENT, nothing done).  The call
 * takes each distinct Tunn's lock (in address order) for its duration, as the
 * single-Tunn calls take their Tunn's.
 * e == NULL: the Tunns may be attached to any engines (normally one engine per
 * GPU, NepTUN's workers serving every peer, packet_workers.rs:113-131): the batch is
 * split by engine, each engine's packets kept in batch order, the shares run
 * concurrently (each on its engine's driver thread, one on the caller) and the
 * results come back in packet order -- still equal to the sequential calls.  A Tunn
 * of wg_tunn_create_multi (private engines) is refused. */
int wg_tunn_encapsulate_multi(wg_engine *e, uint32_t n, wg_tunn *const *tunn,
                              const uint8_t *const *src, const uint32_t *src_len,
                              uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res);
int wg_tunn_decapsulate_multi(wg_engine *e, uint32_t n, wg_tunn *const *tunn,
                              const uint8_t *const *datagram, const uint32_t *len,
                              uint8_t *const *dst, const uint32_t *dst_cap, wg_tunn_result *res);
/* n x Tunn::decrypt(datagram[i], dst[i]) (feature "xray", mod.rs:383-417 ->
 * Session::decrypt_data_packet session.rs:316-353): the first session whose
 * receiving OR sending index equals the header's receiver_idx, opened with the
 * matching direction's key, no replay window, no set_current_session; then
 * validate_decapsulated_packet (rx_bytes as the reference).  Ok(p) comes back
 * as WG_TUNN_WRITE_TO_TUNNEL; a keepalive is ERR UnexpectedPacket and a
 * handshake / cookie message ERR WrongPacketType, like the reference. */
int wg_tunn_decrypt_batch(wg_tunn *t, uint32_t n, const uint8_t *const *datagram,
                          const uint32_t *len, uint8_t *const *dst, const uint32_t *dst_cap,
                          wg_tunn_result *res);

/* Where a Tunn's batch time goes (diagnostics; cumulative since creation or the
 * last reset, summed over engines).  Host phases are wall time on the thread
 * that runs them; the pool phases count the wall time of the whole parallel
 * step.  The device times come from timing events on the chunk streams and are
 * only collected after wg_tunn_set_phase_timing(t, 1). */
typedef struct wg_tunn_phases {
  uint64_t calls, chunks, packets;
  double total_us;        /* inside the batch calls */
  double checks_us;       /* pass 1: parse / session / index checks (pool), counter reservation */
  double pack_us;         /* packets into pinned staging + descriptors (pool) */
  double submit_us;       /* enqueueing copies and kernels */
  double wait_us;         /* the calling / driver thread blocked on a chunk's completion */
  double decide_us;       /* in-order replay window pass (decapsulate; one thread) */
  double copy_out_us;     /* validation + results out of staging into dst (pool) */
  double dev_h2d_us, dev_kernel_us, dev_d2h_us;  /* device time per stage, summed over chunks */
  double pack_spec_us;    /* of pack_us: speculated decisions + output jobs (registered decapsulate) */
  double prep_us;         /* registered (DMA) batches: device addresses, chunks and input runs,
                             before the first chunk is enqueued */
} wg_tunn_phases;
int wg_tunn_get_phases(const wg_tunn *t, wg_tunn_phases *out);
int wg_tunn_reset_phases(wg_tunn *t);
int wg_tunn_set_phase_timing(wg_tunn *t, int on);

#ifdef __cplusplus
}
#endif
#endif /* NEPTUN_TUNN_H */
