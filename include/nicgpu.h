/*
 * nicgpu.h — C-ABI of the MI355X (gfx950) RX offload layer.
 *
 * This is the drop-in boundary under the nic:: C++20 API (include/nic/).
 * Plain C: no HIP, torch or C++ types; device pointers are caller-owned; every
 * launch takes an explicit stream (a hipStream_t passed as void*, NULL = the
 * null stream) and is asynchronous; every entry point returns an int status
 * (0 = ok, < 0 = error, see nicgpu_strerror).  Nothing here falls back to the
 * CPU: a missing GPU or a HIP failure is an error.
 *
 * Reference interfaces replaced (file:line in rosslwheeler/smart_nic):
 *   nicgpu_checksum_batch   <- nic::compute_checksum, include/nic/checksum.h:9,
 *                              src/checksum.cpp:10-34 (one call per packet today)
 *   nicgpu_rx_offload       <- the RX verify in QueuePair::handle_rx_segment,
 *                              src/queue_pair.cpp:434-447, fused with
 *                              nic::RssEngine::select_queue, include/nic/rss.h:35,
 *                              src/rss.cpp:49-61 (+ RssStats, rss.h:18-21)
 *   nicgpu_rss_set_key      <- nic::RssEngine::set_key, rss.h:29, rss.cpp:27-33
 *   nicgpu_rss_set_table    <- nic::RssEngine::set_table, rss.h:30, rss.cpp:35-41
 *   nicgpu_tso_checksum     <- QueuePair::build_segments + per-segment RX verify,
 *                              src/queue_pair.cpp:212-278, 434-447
 *
 * Batch layout in HBM:
 *   frames : byte buffer, 16-B aligned base.  Reads are 16-B granular: the
 *            allocation must cover every 16-B chunk that holds a packet byte.
 *   desc   : one uint64 per packet = offset (bits 0..39, any byte alignment)
 *            | length (bits 40..63, must be <= NICGPU_MAX_PACKET; longer
 *            descriptors give unspecified results).  NICGPU_DESC(off,len).
 *   outputs: structure-of-arrays, any of them may be NULL.
 */
#ifndef NICGPU_H
#define NICGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: nicgpu_qp_view gained piece_cs4 (split piece sums: piece_csum covers each
 *    piece past its first 4 bytes) and the plans of nicgpu_qp_plan* are split
 *    (one piece per plain packet); host-image staging (nicgpu_host_register,
 *    nicgpu_image_*, nicgpu_qp_writeback) added.  A caller built against 1
 *    must not use this library: check nicgpu_abi_version() first. */
#define NICGPU_ABI_VERSION 2

#define NICGPU_OK 0
#define NICGPU_ERR_INVALID (-1)    /* bad argument (null ctx, bad mode, size limits) */
#define NICGPU_ERR_HIP (-2)        /* a HIP runtime call failed */
#define NICGPU_ERR_NO_DEVICE (-3)  /* no gfx950 device visible */
#define NICGPU_ERR_NOMEM (-4)
#define NICGPU_ERR_RANGE (-5)    /* a batch too large for 32-bit piece indices: split it */
#define NICGPU_ERR_AGAIN (-6)    /* an asynchronous plan outgrew its buffers: redo the batch (the next plan fits) */
#define NICGPU_ERR_UNSETTLED (-7) /* segmented resolve: positions did not settle; nothing written, resolve per queue pair */

#define NICGPU_DESC_OFFSET_BITS 40
/* Longest packet the kernels accept: 64 KiB - 1 (the TSO super-frame limit of
 * an IPv4 total length).  Per-packet 32-bit partial sums stay exact below it. */
#define NICGPU_MAX_PACKET 65535u
#define NICGPU_DESC(off, len) \
  ((uint64_t) (off) | ((uint64_t) (len) << NICGPU_DESC_OFFSET_BITS))

/* Hash-input (tuple) selection — the reference has no parser; callers handed
 * select_queue a 12-B src_ip|dst_ip|sport|dport string
 * (tests/tutorial_lesson8_test.cpp:20-35).  AUTO parses Ethernet (+ up to two
 * 0x8100/0x88A8 tags) -> IPv4 TCP/UDP 12 B, other IPv4 or fragments 8 B,
 * IPv6 TCP/UDP 36 B, other IPv6 32 B, anything else 0 B (hash 0).
 * RAW hashes frame bytes [raw_off, raw_off + raw_len) clipped to the frame,
 * raw_off + raw_len <= NICGPU_RAW_MAX_END. */
#define NICGPU_TUPLE_NONE 0
#define NICGPU_TUPLE_AUTO 1
#define NICGPU_TUPLE_RAW 2
#define NICGPU_RAW_MAX_END 64
#define NICGPU_MAX_TUPLE 64
/* Key bytes an RSS context holds.  Longer keys are never needed: tuples are at
 * most NICGPU_MAX_TUPLE bytes, so key bits past 8 * 64 + 31 are never read and
 * a longer key hashes exactly like its first NICGPU_MAX_KEY bytes (no wrap
 * either way, src/rss.cpp:83-89).  nic::RssEngine truncates for the GPU. */
#define NICGPU_MAX_KEY 256
/* Indirection-table entries an RSS context holds (tables above 1024 entries are
 * read from global memory and their hits counted with global atomics). */
#define NICGPU_MAX_TABLE (1u << 24)

/* Library identity / device probe. */
int nicgpu_abi_version(void);
const char* nicgpu_strerror(int status);
/* Number of visible gfx950 devices (>= 0) or a negative status. */
int nicgpu_device_count(void);

/* Minimal device-memory plumbing for host layers that must not include HIP
 * headers (libnic_host.so).  Operate on the current HIP device. */
int nicgpu_get_device(int* device);
int nicgpu_set_device(int device);
int nicgpu_malloc(void** dev_ptr, size_t bytes);
int nicgpu_free(void* dev_ptr);
/* Page-locked host memory (hipHostMalloc), for staging descriptor and result
 * arrays at full PCIe rate. */
int nicgpu_host_alloc(void** host_ptr, size_t bytes);
int nicgpu_host_free(void* host_ptr);
int nicgpu_memset_async(void* dev_ptr, int value, size_t bytes, void* stream);
/* Copies in any direction (hipMemcpyDefault), enqueued on `stream`. */
int nicgpu_memcpy_async(void* dst, const void* src, size_t bytes, void* stream);
int nicgpu_stream_synchronize(void* stream);
/* A non-blocking stream on the current device (hipStreamNonBlocking: no
 * implicit ordering with the null stream), and completion events for ordering
 * one stream after another (copies beside compute). */
int nicgpu_stream_create(void** stream);
/* A stream at the device's least (low != 0) or greatest (low == 0) priority
 * (hipDeviceGetStreamPriorityRange): the batched stage plans the next batch on
 * a least-priority stream so that its kernels yield wave slots to the
 * delivery running beside them. */
int nicgpu_stream_create_priority(void** stream, int low);
int nicgpu_stream_destroy(void* stream);
int nicgpu_event_create(void** event);
int nicgpu_event_destroy(void* event);
int nicgpu_event_record(void* event, void* stream);
int nicgpu_stream_wait_event(void* stream, void* event);

/* RSS context: the uploaded Toeplitz key (as a nibble lookup table of 32-bit
 * key windows, built on the device) and indirection table, on one device.
 * One context per stream/thread; contexts are not internally locked. */
typedef struct nicgpu_rss_ctx nicgpu_rss_ctx;

int nicgpu_rss_create(nicgpu_rss_ctx** out, int device);
int nicgpu_rss_destroy(nicgpu_rss_ctx* ctx);

/* Key bytes from host memory; len 0 selects the reference's 20-byte default
 * key (src/rss.cpp:10-13, 27-33).  Enqueued on `stream`. */
int nicgpu_rss_set_key(nicgpu_rss_ctx* ctx, const uint8_t* key, size_t len, void* stream);
/* Key bytes already in device memory (e.g. after an RCCL broadcast). */
int nicgpu_rss_set_key_device(nicgpu_rss_ctx* ctx, const uint8_t* key_dev, size_t len,
                              void* stream);
/* Indirection table; n 0 selects 128 zeros (src/rss.cpp:35-41). */
int nicgpu_rss_set_table(nicgpu_rss_ctx* ctx, const uint16_t* table, size_t n, void* stream);
int nicgpu_rss_set_table_device(nicgpu_rss_ctx* ctx, const uint16_t* table_dev, size_t n,
                                void* stream);
/* Current sizes (host-side mirror, no device sync). */
int nicgpu_rss_info(const nicgpu_rss_ctx* ctx, size_t* key_len, size_t* table_n);

/* Fused RX offload over a batch:
 *   out_csum[i]  = compute_checksum(frame i)                 (u16)
 *   out_hash[i]  = toeplitz(key, tuple(frame i))             (u32)
 *   out_queue[i] = table[out_hash[i] % table_n]              (u16)
 *   out_hits[j] += #packets with out_hash % table_n == j     (u64[table_n], accumulated)
 * With tuple_mode NONE only out_csum is produced (ctx may be NULL).  With
 * out_csum NULL (and no L3/L4 flags) only each packet's headers are read.
 * RX status per queue_pair.cpp:437-438 is (out_csum[i] == 0). */
int nicgpu_rx_offload(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc,
                      size_t n, int tuple_mode, uint32_t raw_off, uint32_t raw_len,
                      uint16_t* out_csum, uint32_t* out_hash, uint16_t* out_queue,
                      uint64_t* out_hits, void* stream);

/* nicgpu_rx_offload over the first min(n_max, *n_dev) packets, the count read
 * on the device when the launch runs (n_dev: a device uint64 another kernel of
 * the same stream wrote), so a pipeline need not wait for it.  The launch is
 * sized for n_max; outputs past the count are left alone. */
int nicgpu_rx_offload_count(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n_max,
                            const uint64_t* n_dev, int tuple_mode, uint32_t raw_off, uint32_t raw_len,
                            uint16_t* out_csum, uint32_t* out_hash, uint16_t* out_queue, uint64_t* out_hits,
                            void* stream);

/* nicgpu_rx_offload plus L3/L4 checksum verification in the same pass
 * (out_l34[i] = NICGPU_L34_* flags; may be NULL).  The IPv4 header checksum and
 * the TCP/UDP checksum over pseudo-header || segment are those of the
 * reference's PacketGenerator::ipv4_checksum / tcp_checksum / udp_checksum
 * (src/packet_generator.cpp:200-305): a field verifies when the checksum over
 * the covered bytes, field included, is 0.  Semantics: oracle/oracle.h
 * (oracle_l34_verify).  tuple_mode NONE with only out_csum/out_l34 is allowed. */
#define NICGPU_L34_IPV4 0x01u       /* IPv4 header parsed (Eth + <= 2 tags) */
#define NICGPU_L34_IPV4_OK 0x02u    /* its header checksum verifies */
#define NICGPU_L34_L4 0x04u         /* TCP/UDP, unfragmented, datagram within the frame */
#define NICGPU_L34_L4_OK 0x08u      /* L4 checksum verifies (or UDP carries none) */
#define NICGPU_L34_UDP_NOCSUM 0x10u /* UDP checksum field 0: not verified */
int nicgpu_rx_offload_ex(const nicgpu_rss_ctx* ctx, const uint8_t* frames, const uint64_t* desc, size_t n,
                         int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint16_t* out_csum, uint32_t* out_hash,
                         uint16_t* out_queue, uint64_t* out_hits, uint8_t* out_l34, void* stream);

/* Checksum only (== rx_offload with NICGPU_TUPLE_NONE). */
int nicgpu_checksum_batch(const uint8_t* frames, const uint64_t* desc, size_t n,
                          uint16_t* out_csum, void* stream);

/* Split sums (the batched QueuePair stage's piece pass, one piece per plain
 * packet): out_head4[i] = compute_checksum(first min(4, len_i) bytes of frame
 * i), out_rest[i] = compute_checksum(its bytes past the first 4) — the two
 * sums queue_pair.cpp:392-395 / :434-447 take of a segment with and without
 * its VLAN tag, from one pass over the frame. */
int nicgpu_checksum_batch_split(const uint8_t* frames, const uint64_t* desc, size_t n, uint16_t* out_rest,
                                uint16_t* out_head4, void* stream);

/* Per-segment checksums of TSO/GSO segmentation without materialising the
 * segments: for frame i (desc[i]) with header length hdr_len[i] and mss[i],
 * segment k = frame[0:H] || frame[H + k*mss : min(L, H + (k+1)*mss)], and
 * out_csum[seg_base[i] + k] = compute_checksum(segment k).  Frames that the
 * reference would not segment (H >= L, or L <= mss) yield one checksum of the
 * whole frame.  The caller validates MSS/segment-count limits
 * (queue_pair.cpp:225-270) and sizes seg_base (exclusive prefix of segment
 * counts).  mss must be >= 1 for segmented frames. */
int nicgpu_tso_checksum(const uint8_t* frames, const uint64_t* desc, const uint16_t* hdr_len,
                        const uint16_t* mss, const uint32_t* seg_base, size_t n,
                        uint16_t* out_csum, void* stream);

/* RoCEv2 ICRC over a batch: nic::rocev2::IcrcCalculator
 * (include/nic/rocev2/packet.h:195-214, src/rocev2/packet.cpp:14-75), one
 * call per packet today.  Each descriptor's bytes are the span the reference
 * is handed (BTH through payload; the reference masks no fields).
 *   NICGPU_ICRC_CALCULATE: out_crc[i] = calculate(span)   (out_ok must be NULL)
 *   NICGPU_ICRC_VERIFY:    out_ok[i]  = verify(span): span >= 4 B and the
 *                          CRC-32C of all but its last 4 bytes equals those
 *                          bytes read big-endian; out_crc[i] (optional) = that
 *                          CRC, or 0 for spans shorter than 4 B. */
#define NICGPU_ICRC_CALCULATE 0
#define NICGPU_ICRC_VERIFY 1
int nicgpu_icrc_batch(const uint8_t* frames, const uint64_t* desc, size_t n, int mode, uint32_t* out_crc,
                      uint8_t* out_ok, void* stream);

/* TSO/GSO segmentation with VLAN insert/strip, materialised:
 * QueuePair::build_segments (src/queue_pair.cpp:212-278), the TX VLAN insert
 * (:324-331) and the RX VLAN strip (:389-395) applied to every frame.
 * flags[i] (NULL = NICGPU_SEG_TSO for every frame): NICGPU_SEG_* bits plus the
 * VLAN tag in the low 16 bits.  Segmentation happens when NICGPU_SEG_TSO is set,
 * mss > 0 and L > mss; mss > 9000 or hdr_len > L then produces no segment
 * (InvalidMss), as do more than 64 segments (TooManySegments); hdr_len >= L
 * gives one copy of the frame.  Segment k of frame i is written to
 * out[(seg_base[i] + k) * stride ..] (skipped if it does not fit the slot) with
 * out_len = its size and out_csum = compute_checksum(segment bytes), the value
 * the RX verify tests against 0 (:434-447).  seg_base: exclusive prefix sum of
 * the segment counts under these rules (smart_nic_amd.tso_segment_counts). */
#define NICGPU_SEG_TSO 0x10000u          /* tso_enabled || gso_enabled */
#define NICGPU_SEG_VLAN_INSERT 0x20000u  /* TX: prepend 81 00 tag */
#define NICGPU_SEG_VLAN_STRIP 0x40000u   /* RX: strip 4 bytes when the segment has a VLAN */
#define NICGPU_SEG_VLAN_PRESENT 0x80000u /* RX descriptor says a VLAN is present */
int nicgpu_tso_segment(const uint8_t* frames, const uint64_t* desc, const uint16_t* hdr_len, const uint16_t* mss,
                       const uint32_t* seg_base, const uint32_t* flags, size_t n, uint8_t* out, uint64_t out_size,
                       uint32_t stride, uint32_t* out_len, uint16_t* out_csum, void* stream);

/* One DMA write of the batched QueuePair stage (nic/rx_stage.h):
 *   mem[dst ..] <- prefix bytes (prefix_len 0 or 4; little-endian word, i.e.
 *                  memory order) || mem[src_a, +len_a) || mem[src_b, +len_b).
 * Replaces the per-segment DMAEngine::write of QueuePair::handle_rx_segment
 * (src/queue_pair.cpp:416-426) after build_segments / VLAN insert-strip
 * (:212-278, :324-331, :389-395).  40 bytes, naturally aligned. */
typedef struct nicgpu_segment_write {
  uint64_t dst;
  uint64_t src_a;
  uint64_t src_b;
  uint32_t len_a;
  uint32_t len_b;
  uint32_t prefix;
  uint32_t prefix_len;
} nicgpu_segment_write;

/* Perform n writes (device array) inside the memory image mem[0, mem_size).
 * The writes run in parallel: destinations must not overlap each other or any
 * source (nic::BatchedQueuePair orders overlapping writes into successive
 * launches).  Entries reaching outside the image are skipped. */
int nicgpu_segment_gather(uint8_t* mem, uint64_t mem_size, const nicgpu_segment_write* writes, size_t n,
                          void* stream);
/* The same with every source read from src[0, mem_size) (a copy of the image
 * taken earlier, e.g. before a batch whose writes overwrite its own sources);
 * destinations are in mem and must not overlap each other. */
int nicgpu_segment_gather_from(uint8_t* mem, const uint8_t* src, uint64_t mem_size,
                               const nicgpu_segment_write* writes, size_t n, void* stream);

/* ------------------------------------------------------------------------
 * Batched QueuePair on the device: the per-packet decisions of
 * QueuePair::process_once (src/queue_pair.cpp:67-460) for a whole batch, run
 * by nic::BatchedQueuePair (include/nic/rx_stage.h) when the batch's buffers
 * do not overlap and no interrupt callback is set.  The decision logic is
 * smart_nic_amd/csrc/qp_logic.h, the same source the host resolve uses.
 *
 * C mirrors of the reference PODs, same layouts (include/nic/tx_rx.h:37-62,
 * include/nic/completion_queue.h:13-26, include/nic/queue_pair.h:36-53). */
typedef struct nicgpu_tx_descriptor {
  uint64_t buffer_address;
  uint32_t length;
  uint8_t checksum; /* ChecksumMode: 0 None, 1 Layer3, 2 Layer4 */
  uint8_t pad0;
  uint16_t descriptor_index;
  uint16_t checksum_value;
  uint8_t checksum_offload;
  uint8_t tso_enabled;
  uint8_t gso_enabled;
  uint8_t pad1;
  uint16_t mss;
  uint16_t header_length;
  uint8_t vlan_insert;
  uint8_t pad2;
  uint16_t vlan_tag;
  uint16_t pad3;
} nicgpu_tx_descriptor; /* 32 B */

typedef struct nicgpu_rx_descriptor {
  uint64_t buffer_address;
  uint32_t buffer_length;
  uint8_t checksum;
  uint8_t pad0;
  uint16_t descriptor_index;
  uint8_t checksum_offload;
  uint8_t vlan_strip;
  uint8_t vlan_present;
  uint8_t pad1;
  uint16_t vlan_tag;
  uint8_t gro_enabled;
  uint8_t pad2;
} nicgpu_rx_descriptor; /* 24 B */

typedef struct nicgpu_completion {
  uint16_t queue_id;
  uint16_t descriptor_index;
  uint32_t status; /* CompletionCode */
  uint8_t checksum_offloaded;
  uint8_t checksum_verified;
  uint8_t tso_performed;
  uint8_t gso_performed;
  uint8_t vlan_inserted;
  uint8_t vlan_stripped;
  uint8_t gro_aggregated;
  uint8_t pad0;
  uint16_t segments_produced;
  uint16_t vlan_tag;
} nicgpu_completion; /* 20 B */

typedef struct nicgpu_qp_stats {
  uint64_t tx_packets, rx_packets, tx_bytes, rx_bytes, drops_checksum, drops_no_rx_desc, drops_buffer_small,
      drops_mtu_exceeded, drops_invalid_mss, drops_too_many_segments, tx_tso_segments, tx_gso_segments,
      tx_vlan_insertions, rx_vlan_strips, rx_checksum_verified, rx_gro_aggregated;
} nicgpu_qp_stats;

/* Device buffers of a QueuePair context (valid until the next
 * nicgpu_qp_reserve / nicgpu_qp_plan that grows them). */
typedef struct nicgpu_qp_view {
  nicgpu_tx_descriptor* tx;     /* [ntx]  the caller uploads the TX descriptors here */
  nicgpu_rx_descriptor* rx;     /* [nrx]  and the RX descriptors (the ring, rx[0] first) */
  uint32_t* piece_base;         /* [ntx + 1] first piece of each TX descriptor */
  uint16_t* piece_csum;         /* [npieces] split sums (nicgpu_checksum_batch_split): each piece past its first 4 bytes */
  nicgpu_completion* txc;       /* [ntx]  TX completions, in posting order */
  nicgpu_completion* rxc;       /* [nrx]  RX completions, in posting order */
  nicgpu_segment_write* writes; /* [nrx]  DMA write of RX completion j (all lengths 0: none) */
  uint64_t* rss_desc;           /* [nrx]  frames delivered with Success (NICGPU_DESC) */
  uint32_t* rss_hash;           /* [nrx]  their hashes / queues, as RSS leaves them */
  uint16_t* rss_queue;
  uint32_t* rx_hash;            /* [nrx]  per RX completion: hash (0 unless Success) */
  uint16_t* rx_queue;           /* [nrx]  per RX completion: queue (0xFFFF unless Success) */
  uint32_t* queue_which;        /* [nrx]  Success completions grouped by queue (nicgpu_qp_group) */
  uint32_t* queue_start;        /* [65536] queue q = queue_which[queue_start[q], queue_end[q]) */
  uint32_t* queue_end;
  uint64_t* rss_count;          /* [1]    frames listed by nicgpu_qp_rss_list (device scalar) */
  uint16_t* piece_cs4;          /* [npieces] and of each piece's first min(4, len) bytes */
} nicgpu_qp_view;

typedef struct nicgpu_qp nicgpu_qp;
/* Largest batch nicgpu_qp_reserve accepts: piece indices are 32-bit and a TX
 * descriptor plans at most 256 pieces.  nic::BatchedQueuePair sends larger
 * batches to its host path (include/nic/rx_stage.h). */
#define NICGPU_QP_MAX_TX (0xFFFFFFFFull / 256u)
#define NICGPU_QP_MAX_RX 0x7FFFFFFEull
int nicgpu_qp_create(nicgpu_qp** out, int device);
int nicgpu_qp_destroy(nicgpu_qp* q);
/* Capacity for ntx TX and nrx RX descriptors (ntx <= 2^32 / 256 and
 * nrx < 2^31 - 1); fills *view.  Piece indices are 32-bit: a batch plans at
 * most 256 pieces per TX descriptor unless one of them is a huge plain packet
 * that is verified and then dropped (one piece per 64 KiB); nicgpu_qp_plan
 * then returns NICGPU_ERR_RANGE before anything is sized from the count. */
int nicgpu_qp_reserve(nicgpu_qp* q, size_t ntx, size_t nrx, nicgpu_qp_view* view);
/* Whether the buffers of view.tx[0, ntx) and view.rx[0, nrx) are disjoint, as
 * nic::rx_stage_detail::buffers_disjoint defines it (RX spans: at most
 * buffer_length bytes inside the image; TX spans: the whole buffer; an
 * overlap among RX spans or between an RX and a TX span is one).  *verdict =
 * 1 disjoint, 0 not, -1 undecided: the RX spans, in ring order, are not
 * ascending and apart (the caller then sorts on the host).  Synchronises
 * `stream`. */
int nicgpu_qp_check(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, int* verdict, void* stream);
/* nicgpu_qp_check with flags: NICGPU_QP_CHECK_WHOLE checks a segmented batch
 * as one ring (every RX span against every other and every TX span, across
 * queue pairs too), not queue pair by queue pair. */
#define NICGPU_QP_CHECK_WHOLE 1u
int nicgpu_qp_check_flags(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, unsigned flags, int* verdict,
                          void* stream);
/* nicgpu_qp_check_flags in two halves: _async enqueues the check on `stream`
 * and returns; _wait waits for its verdict (one check pending per nicgpu_qp).
 * The check may then run beside the plan and the speculative resolve. */
int nicgpu_qp_check_async(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, unsigned flags, void* stream);
int nicgpu_qp_check_wait(nicgpu_qp* q, int* verdict);
/* After an unsegmented check: bounds[0..1] = [min start, max end) of the TX
 * spans; when the verdict was 0 or 1 (the RX spans ascend) bounds[2..3] =
 * [least start, max end) of the RX spans, all bytes the batch's DMA writes can
 * touch (undefined for a verdict of -1); [~0, 0) when empty.
 * A pipeline tells with them whether a batch's frames lie where an earlier
 * batch still writes. */
int nicgpu_qp_check_bounds(const nicgpu_qp* q, uint64_t* bounds);
/* The piece sums of q's current plan again (nicgpu_qp_plan_async's sums), on
 * `stream`: for frames an earlier batch's DMA writes changed after the first
 * sums read them, or for a batch that skipped them (deferred RX verify). */
int nicgpu_qp_resum(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, void* stream);
/* The kernels of the next plan/check/resolve read the caller's device arrays
 * tx[0, ntx) and rx[0, nrx) in place of view.tx / view.rx (no copy; view is
 * refreshed to point at them).  They must stay valid and unchanged until the
 * batch is resolved, and lie outside the memory image the batch writes (a
 * write there would change a descriptor the reference pops later).  A later
 * nicgpu_qp_reserve returns the context to its own arrays. */
int nicgpu_qp_bind(nicgpu_qp* q, const nicgpu_tx_descriptor* tx, size_t ntx, const nicgpu_rx_descriptor* rx,
                   size_t nrx, nicgpu_qp_view* view);
/* The plan (qp_logic.h plan_packet, split form: one piece per plain packet below
 * 64 KiB, PacketPlan kPlainSplit) of view.tx[0, ntx) and the split checksums
 * of every piece over the image mem[0, mem_size) — view.piece_csum holds each
 * piece's bytes past its first 4, view.piece_cs4 its first min(4, len) bytes;
 * neither is compute_checksum of the whole piece: *npieces on return
 * (NICGPU_ERR_RANGE, nothing enqueued after the count, when a descriptor plans
 * more than 256 pieces: the total may then not fit 32 bits).  Waits for
 * `stream` once (the piece count sizes the piece buffers); the piece
 * descriptors and checksums are then enqueued on it.  Refreshes *view (the
 * piece buffers may grow). */
int nicgpu_qp_plan(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                   uint64_t* npieces, nicgpu_qp_view* view, void* stream);
/* nicgpu_qp_plan with the plan (which reads only view.tx) on plan_stream,
 * waited for once, and the piece checksums (which read the image) enqueued on
 * sums_stream behind it.  A batched stage plans batch k+1 on a side stream
 * while batch k's DMA writes, which may write bytes batch k+1 sends, still run
 * on the main one. */
int nicgpu_qp_plan_on(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                      uint64_t* npieces, nicgpu_qp_view* view, void* plan_stream, void* sums_stream);
/* nicgpu_qp_plan_on without its wait: nothing is read back.  The piece
 * buffers hold at least ntx + ntx / 4 + 64 pieces (and what the last resolve
 * reported); the fill and the sums use the piece count the scan leaves on the
 * device, bounded by that capacity.  When the plan does not fit, the next
 * nicgpu_qp_resolve_start settles nothing and nicgpu_qp_resolve_finish returns
 * NICGPU_ERR_AGAIN: the caller redoes the batch (the next plan is sized from
 * this one's count); NICGPU_ERR_RANGE likewise when a descriptor plans more
 * than 256 pieces (as nicgpu_qp_plan).  Refreshes *view. */
int nicgpu_qp_plan_async(nicgpu_qp* q, const uint8_t* mem, uint64_t mem_size, size_t ntx, uint64_t max_mtu,
                         nicgpu_qp_view* view, void* plan_stream, void* sums_stream);
/* The piece count of the plan the last nicgpu_qp_resolve_finish resolved. */
int nicgpu_qp_piece_count(const nicgpu_qp* q, uint64_t* npieces);
/* The reference's control flow over view.tx[0, ntx) against view.rx[0, nrx)
 * from the piece sums: TX descriptors [0, *done) are resolved, with
 * completions in view.txc[0, *done) and view.rxc[0, *rx_used), their writes in
 * view.writes and their statistics in *stats.  Ring positions are found by
 * relaxation: each packet is resolved at the exclusive scan of the previous
 * step's pops (first guess: what it needs), which is exact for at least one
 * more packet per step and, when a packet's pops do not depend on where in the
 * ring it lands (a ring that runs short, failed segment checksums on uniform
 * RX descriptors), for all of them after two.  When 8 steps have not settled
 * every packet (a long chain of TSO/GSO packets each ending early on the RX
 * side), the positions are walked instead: only a packet needing more than one
 * RX descriptor can pop other than its need while the ring lasts, so one
 * thread per queue pair resolves those in ring order at their exact positions
 * and the ring's end is relaxed once more (nicgpu_qp_walks counts these).
 * Should *done still stop short, it stops at the first packet not yet exact
 * and the caller resolves the rest in order (piece checksums from
 * view.piece_base[*done]).  Synchronises `stream`. */
int nicgpu_qp_resolve(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, uint64_t max_mtu, uint16_t queue_id,
                      uint64_t* done, uint64_t* rx_used, nicgpu_qp_stats* stats, void* stream);
/* nicgpu_qp_resolve in two halves (NICGPU_ERR_AGAIN / _RANGE from _finish:
 * see nicgpu_qp_plan_async).  _start enqueues the speculative pass
 * (every packet at the scan of what it needs) on `stream` and returns without
 * waiting; its settled prefix — the RX completions of the packets before the
 * first one that popped otherwise, all of them when none did — is a device
 * scalar that nicgpu_qp_deliver_range(NICGPU_DELIVER_SETTLED) reads, so the DMA
 * writes can be enqueued before the host has seen the resolve.  _finish waits
 * for the pass only (not for work enqueued after it), relaxes on `stream` when
 * the guess was wrong (those steps then wait behind that work), and returns
 * what nicgpu_qp_resolve does plus *rx_settled (<= *rx_used; may be null).
 * One resolve may be pending per nicgpu_qp. */
int nicgpu_qp_resolve_start(nicgpu_qp* q, uint64_t mem_size, size_t ntx, size_t nrx, uint64_t max_mtu,
                            uint16_t queue_id, void* stream);
int nicgpu_qp_resolve_finish(nicgpu_qp* q, uint64_t* done, uint64_t* rx_used, uint64_t* rx_settled,
                             nicgpu_qp_stats* stats);
/* The resolves of q whose positions the walk made, since q was created. */
int nicgpu_qp_walks(const nicgpu_qp* q, uint64_t* walks);
/* Deferred RX verify (off by default).  With it on, a batch planned by
 * nicgpu_qp_plan_async in which no decision that moves ring positions reads a
 * sum — no TX descriptor needs the TX verify (queue_pair.cpp:94-105) and none
 * makes more than one segment — skips its piece sums: the resolve takes every
 * RX verify (:434-447) to pass, and the delivery (nicgpu_qp_deliver_range)
 * sums the bytes each such completion's write delivers, which are exactly the
 * bytes that verify covers.  A completion whose sum fails gets the
 * reference's ChecksumError completion there (status, no VLAN strip), RSS
 * skips it, and the counts the resolve's statistics took for it as delivered
 * are accumulated on the device for the caller to correct
 * (nicgpu_qp_verify_fixups_async).  Completions and statistics of such a
 * batch are therefore final only after its deliveries; nicgpu_qp_deferred
 * tells, after nicgpu_qp_resolve_finish, whether the last batch deferred.
 * Its host-resolved rest (*done < ntx) needs nicgpu_qp_resum first: the
 * piece sums were skipped.  Segmented batches too (each segment's
 * corrections apart).  The synchronous nicgpu_qp_plan / _plan_on always sum. */
int nicgpu_qp_set_deferred_verify(nicgpu_qp* q, int on);
/* CUs the next deliveries of q leave without a delivery block (< 0: the
 * default, 0 unless NICGPU_DLV_RESERVE_CUS says otherwise): a pipeline whose
 * next batch plans and checks beside this delivery gives those kernels wave
 * slots this way (nic::BatchedQueuePair: 32 while another batch is submitted). */
int nicgpu_qp_set_delivery_reserve(nicgpu_qp* q, int cus);
int nicgpu_qp_deferred(const nicgpu_qp* q, int* deferred);
/* The deferred verifies' corrections of q's last planned batch (the plan's
 * count kernel zeroes them, in stream order, before the batch's deliveries),
 * on `stream` into out[nseg][NICGPU_QP_FIXUPS] (nseg: 1, or the segments of a
 * segmented batch, each its queue pair's): [0] verifies that failed (each a
 * drops_checksum the statistics lack and an rx_packets and tx_packets they
 * hold too many), then what they hold too many of: [1] rx_bytes, [2]
 * rx_vlan_strips, [3] tx_bytes, [4] tx_vlan_insertions; [5..7] 0.  Per batch,
 * so a batch that failed after its deliveries leaves nothing behind for the
 * next one. */
#define NICGPU_QP_FIXUPS 8u
int nicgpu_qp_verify_fixups_async(nicgpu_qp* q, uint64_t* out, size_t nseg, void* stream);
/* The frames of view.rxc[0, nrx) delivered with Success, as RSS descriptors
 * (view.rss_desc[0, m), lengths clipped to NICGPU_MAX_PACKET), m written to
 * the device scalar view.rss_count; view.rx_hash / rx_queue reset to 0 /
 * 0xFFFF.  Enqueued only (no wait): the steps below and
 * nicgpu_rx_offload_count read m on the device. */
int nicgpu_qp_rss_list(nicgpu_qp* q, size_t nrx, void* stream);
/* view.rx_hash / rx_queue of those m frames from view.rss_hash / rss_queue
 * (nrx: the bound the list was made over).  Enqueued only. */
int nicgpu_qp_rss_scatter(nicgpu_qp* q, size_t nrx, void* stream);
/* The RSS dispatch lists: the m listed frames grouped by queue (a stable sort,
 * so each queue lists its completions in posting order) into
 * view.queue_which[0, m), with each queue's range in view.queue_start /
 * queue_end for queues [0, nq) (nq <= 65536, at least the largest queue the
 * indirection table holds + 1; empty queues get start = end = 0).  The sort
 * runs over the nrx bound with the unlisted entries keyed nq, past every
 * queue, on the low bits that hold 0..nq only.  Enqueued only. */
int nicgpu_qp_group(nicgpu_qp* q, size_t nrx, size_t nq, void* stream);
/* The DMA writes view.writes[0, nrx) (as nicgpu_segment_gather) and, unless
 * tuple_mode is NICGPU_TUPLE_NONE, the RSS of every RX completion whose status
 * is Success, hashed from the bytes its write delivers (as nicgpu_rx_offload
 * over those frames with ctx and the tuple mode): view.rx_hash / rx_queue per
 * completion (0 / 0xFFFF for the others), the table-index hits added into
 * hits_dev (ctx's table size, u64), the Success count in *view.rss_count.  One
 * launch, the headers taken from the bytes the writes move (no read-back);
 * nicgpu_qp_group then lists the completions per queue.  Replaces
 * nicgpu_segment_gather + nicgpu_qp_rss_list + an RSS launch + nicgpu_qp_rss_scatter. */
int nicgpu_qp_deliver(nicgpu_qp* q, uint8_t* mem, uint64_t mem_size, size_t nrx, const nicgpu_rss_ctx* ctx,
                      int tuple_mode, uint32_t raw_off, uint32_t raw_len, uint64_t* hits_dev, void* stream);
#define NICGPU_DELIVER_SETTLED 1u /* end at the settled prefix of the pending nicgpu_qp_resolve_start */
#define NICGPU_DELIVER_APPEND 2u  /* add to *view.rss_count instead of resetting it (a later range) */
#define NICGPU_DELIVER_RESET_HITS 4u /* set hits_dev to this range's hits instead of adding (no memset first) */
/* nicgpu_qp_deliver over completions [rx_begin, rx_end) (bounded on the device
 * with NICGPU_DELIVER_SETTLED).  Ranges of one batch may be delivered in any
 * order when the batch's buffers are disjoint (nicgpu_qp_check verdict 1): the
 * settled prefix first, the rest after nicgpu_qp_resolve_finish with APPEND;
 * hits_dev accumulates over the ranges, nicgpu_qp_group runs after the last. */
int nicgpu_qp_deliver_range(nicgpu_qp* q, uint8_t* mem, uint64_t mem_size, size_t rx_begin, size_t rx_end,
                            unsigned flags, const nicgpu_rss_ctx* ctx, int tuple_mode, uint32_t raw_off,
                            uint32_t raw_len, uint64_t* hits_dev, void* stream);

/* ---- Several queue pairs in one batch (nic::BatchedQueueManager) ----
 * QueueManager::process_once (src/queue_manager.cpp:54-78) serves several
 * QueuePairs; when no queue's buffers meet another's, each queue pair's
 * results are independent of the interleaving, so their batches can be
 * resolved together: view.tx holds the queue pairs' TX batches back to back
 * (segment s's are [tx_begin_s, tx_begin_{s+1}), the last ends at ntx) and
 * view.rx their RX rings back to back (segment s's ring is
 * [rx_begin_s, rx_begin_s + nrx_s), rx_begin ascending).  Every kernel of the
 * next plans and resolves then runs segment s's packets with its own queue id
 * and MTU against its own ring: ring positions are the scan of the pops
 * restarted at every segment, a ring's end is its own.  Completions land at
 * their absolute slots: segment s's TX completions at view.txc[tx_begin_s ..],
 * its RX completions at view.rxc[rx_begin_s, + used_s); the ring slots it does
 * not use hold an empty write and status NICGPU_QP_SLOT_UNUSED (no delivery,
 * no RSS).  The resolve settles all of the batch or nothing:
 * nicgpu_qp_resolve_finish returns NICGPU_ERR_UNSETTLED when some position
 * is still unsettled after the relaxation steps (nothing was written; the
 * caller resolves the queue pairs one by one) and otherwise *done = ntx,
 * *rx_used = *rx_settled = the concatenated ring's length when the
 * speculative pass settled everything (0 settled otherwise: deliver it all
 * afterwards). */
typedef struct nicgpu_qp_segment {
  uint64_t tx_begin;
  uint64_t rx_begin;
  uint64_t nrx;
  uint64_t max_mtu;
  uint16_t queue_id;
  uint16_t pad0, pad1, pad2;
} nicgpu_qp_segment; /* 40 B */
#define NICGPU_QP_SLOT_UNUSED 0xFFFFFFFFu
#define NICGPU_QP_MAX_SEGMENTS 1024u
/* Segments for the following plans/resolves of q (host array, copied; nseg 0:
 * back to one queue pair).  ntx: the batch's TX descriptors (sizes the block
 * map: each grid block serves one segment, blocks in proportion to its TX
 * descriptors).  Enqueued on `stream`. */
int nicgpu_qp_set_segments(nicgpu_qp* q, const nicgpu_qp_segment* seg, size_t nseg, size_t ntx, void* stream);
/* After a segmented nicgpu_qp_resolve_finish: per segment, the RX descriptors
 * its queue pair popped (used[nseg]) and its QueuePairStats (stats[nseg]). */
int nicgpu_qp_segment_results(const nicgpu_qp* q, uint64_t* used, nicgpu_qp_stats* stats);
/* After nicgpu_qp_group over a segmented batch's nrx slots with nq RSS queues:
 * the dispatch lists split per segment — entries rewritten to indices relative
 * to their segment's rx_begin, and split[s * nq + r] = the first entry of RSS
 * queue r's list (view.queue_which[queue_start[r], queue_end[r])) that belongs
 * to segment s or later, for s in [0, nseg] (split[nseg * nq + r] =
 * queue_end[r]).  split_host: (nseg + 1) * nq words; synchronises `stream`. */
int nicgpu_qp_segment_lists(nicgpu_qp* q, size_t nrx, size_t nq, uint32_t* split_host, void* stream);
/* Per-segment RSS hits of the delivered frames (Success completions, hashed by
 * the delivery): hits_dev[s * table_n + h % table_n] (u64, set, not added).
 * For queue pairs that count into RssEngines of their own. */
int nicgpu_qp_segment_hits(nicgpu_qp* q, size_t nrx, size_t table_n, uint64_t* hits_dev, void* stream);
/* Gathers the queue pairs' device-resident descriptor arrays into the
 * concatenated view.tx / view.rx in ONE launch: dst[i] <- src[i] (bytes[i]
 * each) for i < n, all device-accessible, ranges not overlapping.  (The n
 * separate copies cost a launch each — 2 per queue pair.)  n <= 64 per call. */
typedef struct nicgpu_copy_range {
  void* dst;
  const void* src;
  uint64_t bytes;
} nicgpu_copy_range;
#define NICGPU_COPY_BATCH_MAX 64u
int nicgpu_memcpy_batch(const nicgpu_copy_range* ranges, size_t n, void* stream);

/* ---- Host-image staging (row f1 on the reference's HostMemory) ----
 * nic::BatchedQueuePair::process_batch(HostMemory&, ...) runs the stage on an
 * HBM mirror of the memory's flat window (SimpleHostMemory's std::vector,
 * src/simple_host_memory.cpp:16, 70-109): the TX buffers' bytes go up before a
 * batch (QueuePair's DMA read, queue_pair.cpp:86-92) and exactly the bytes its
 * DMA writes delivered come back (queue_pair.cpp:416-426). */
/* Waits for the event's last record on the calling thread. */
int nicgpu_event_synchronize(void* event);
/* Page-locks exactly host memory [host_ptr, host_ptr + bytes) (hipHostRegister
 * of that range, no page extension: heap neighbours sharing its pages stay
 * ordinary pageable memory for every other copy) and maps it for the device:
 * *dev_alias = the device-visible address of host_ptr.  Registrations are
 * reference counted: a range inside one this library registered shares it,
 * and each successful call (*owned = 1) is released by one
 * nicgpu_host_unregister of the same host_ptr; the last release unregisters.
 * A range registered by someone else (hipHostMalloc, the application) is
 * refused with NICGPU_ERR_INVALID: its lifetime is not this library's.
 * Kernels reading through the alias never read past host_ptr + bytes. */
int nicgpu_host_register(void* host_ptr, size_t bytes, void** dev_alias, int* owned);
int nicgpu_host_unregister(void* host_ptr);
/* image[a, a + len) <- host[a, a + len) for every TX descriptor tx[0, ntx)
 * (device array) whose buffer is inside mem_size (a = buffer_address, len =
 * length): byte-exact, no byte outside the buffers is written.  host is a
 * device-visible alias (nicgpu_host_register) with 16-B alignment; image and
 * host both hold mem_size bytes; no byte past mem_size is read. */
int nicgpu_image_stage(uint8_t* image, const uint8_t* host, uint64_t mem_size, const nicgpu_tx_descriptor* tx,
                       size_t ntx, void* stream);
/* host[d, d + len) <- image[d, d + len) for every write w of writes[0, n)
 * (device array; d = w.dst, len = w.prefix_len + w.len_a + w.len_b, skipped
 * when empty or outside mem_size): the bytes nicgpu_segment_gather /
 * nicgpu_qp_deliver wrote, written back byte-exact (no other host byte is
 * stored to).  Same alignment rules as nicgpu_image_stage. */
int nicgpu_image_writeback(const uint8_t* image, uint8_t* host, uint64_t mem_size, const nicgpu_segment_write* writes,
                           size_t n, void* stream);

/* ---- RSS dispatch into per-queue completion rings (row f1) ----
 * nq rings of ring_size entries on one device, one nic::CompletionQueue each
 * (src/completion_queue.cpp:30-53; replaces its post_completion /
 * poll_completion for the completions a batch dispatches by RSS queue).
 * State per ring: producer, consumer, count (all < ring_size) and the entries
 * a full ring refused. */
typedef struct nicgpu_cq_set nicgpu_cq_set;
int nicgpu_cq_create(nicgpu_cq_set** out, int device, size_t nq, size_t ring_size);
int nicgpu_cq_destroy(nicgpu_cq_set* cq);
/* Posts, for every queue q < nlists, the device completions
 * rxc[which[start[q] .. end[q])] into ring q in that order, as
 * CompletionQueue::post_completion would one by one: entry i of the list
 * lands at (producer + i) % ring_size while the ring has room, the rest are
 * refused (counted).  No doorbell is rung here (the reference rings
 * Doorbell{queue_id, producer} per post, completion_queue.cpp:38-39):
 * nic::RssCompletionRings::set_doorbell rings that sequence on the host from
 * the lists and the state before the post.  start / end are host arrays (nicgpu_qp_group's lists,
 * RxBatchResult::dev.queue_start / queue_end), rxc and which device arrays.
 * Synchronises `stream`. */
int nicgpu_cq_post(nicgpu_cq_set* cq, const nicgpu_completion* rxc, const uint32_t* which, const uint32_t* start,
                   const uint32_t* end, size_t nlists, void* stream);
/* The rings' state into out_host[4 * nq]: producer[nq] | consumer[nq] |
 * count[nq] | refused[nq].  Synchronises `stream`. */
int nicgpu_cq_state(const nicgpu_cq_set* cq, uint32_t* out_host, void* stream);
/* CompletionQueue::poll_completion up to max times on ring q: the entries
 * into out_host, their number into *got.  Synchronises `stream`. */
int nicgpu_cq_poll(nicgpu_cq_set* cq, uint32_t q, nicgpu_completion* out_host, size_t max, size_t* got, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NICGPU_H */
