/*
 * oracle.h — CPU restatement of the smart_nic RX checksum + RSS path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker (or the timed CPU baseline), never as
 * the thing measured or shipped.
 *
 * Every function restates the reference algorithm literally (same loop
 * structure, same eager carry fold, same bit-serial Toeplitz with
 * `(bit + k) % key_bits`) and cites the reference file:line it follows.
 * Parity pinning: tests/test_oracle_golden.py checks every function here
 * against tests/golden/, which oracle/gen_golden.cpp produced by linking the
 * reference's own src/checksum.cpp, src/rss.cpp and src/queue_pair.cpp.
 */
#ifndef SMART_NIC_ORACLE_H
#define SMART_NIC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/checksum.cpp:10-34 */
uint16_t oracle_compute_checksum(const uint8_t* buf, size_t len);

/* src/rss.cpp:63-94 (toeplitz_hash; returns 0 for an empty key or data) */
uint32_t oracle_toeplitz(const uint8_t* key, size_t key_len, const uint8_t* data, size_t len);

/* src/rss.cpp:49-61 select_queue: returns table[h % n]; *tidx = h % n.
 * table_n must be > 0 (the reference guarantees a non-empty table). */
uint16_t oracle_select_queue(const uint8_t* key, size_t key_len, const uint16_t* table,
                             size_t table_n, const uint8_t* data, size_t len, uint32_t* hash,
                             uint32_t* tidx);

/* The 20-byte default key of src/rss.cpp:10-13; writes 20 bytes. */
void oracle_default_key(uint8_t out[20]);

/* Hash-input extraction (the reference has no parser: callers pass the
 * 12-byte src_ip|dst_ip|sport|dport tuple, tests/tutorial_lesson8_test.cpp:20-35,
 * docs/users_guide.md:1096-1103).  Frame layout follows
 * src/packet_generator.cpp:46-166.  Modes mirror include/nicgpu.h.
 * Returns the tuple length written to out (<= 64). */
#define ORACLE_TUPLE_NONE 0
#define ORACLE_TUPLE_AUTO 1
#define ORACLE_TUPLE_RAW 2
size_t oracle_extract_tuple(const uint8_t* frame, size_t len, int mode, size_t raw_off,
                            size_t raw_len, uint8_t out[64]);

/* Batch restatement: for each packet i (bytes frames[off_i, off_i+len_i)),
 * csum[i] = compute_checksum, and (if mode != NONE) hash/tidx/queue of the
 * extracted tuple.  hits (table_n entries, may be NULL) accumulates table-index
 * hits exactly like RssStats::queue_hits (src/rss.cpp:56-58).  desc[i] packs
 * offset (low 40 bits) and length (high 24 bits) as in include/nicgpu.h. */
void oracle_rx_batch(const uint8_t* frames, const uint64_t* desc, size_t n, int mode,
                     size_t raw_off, size_t raw_len, const uint8_t* key, size_t key_len,
                     const uint16_t* table, size_t table_n, uint16_t* csum, uint32_t* hash,
                     uint16_t* queue, uint32_t* tidx, uint64_t* hits);

/* Per-segment checksum of TSO/GSO segmentation, src/queue_pair.cpp:212-278:
 * segment k = pkt[0:H] || pkt[H + k*mss : min(L, H + (k+1)*mss)], each
 * checksummed with compute_checksum (queue_pair.cpp:434-447).  Returns the
 * number of segments written (the unsegmented cases give 1 segment = the
 * whole packet).  Returns -1 for InvalidMss, -2 for TooManySegments
 * (queue_pair.cpp:225-270).  out must hold up to max_out entries. */
int oracle_tso_segment_checksums(const uint8_t* pkt, size_t len, uint16_t hdr_len, uint16_t mss,
                                 int segmentation_enabled, uint16_t* out, size_t max_out);

/* L3/L4 checksum verification of one frame.  Flags:
 *   ORACLE_L34_IPV4     Ethernet (+ <= 2 0x8100/0x88A8 tags), ethertype 0x0800,
 *                       version 4, IHL >= 5 and the whole IP header in the frame
 *   ORACLE_L34_IPV4_OK  ... and ipv4_checksum(header) == 0
 *                       (packet_generator.cpp:200-202, validation_test.cpp:73-76)
 *   ORACLE_L34_L4       ... and protocol TCP/UDP, not a fragment (MF = 0,
 *                       offset = 0), IHL*4 <= total_length, the IP datagram
 *                       within the frame, and the L4 header present (TCP 20 B,
 *                       UDP 8 B)
 *   ORACLE_L34_L4_OK    ... and the checksum over pseudo-header (src, dst, 0,
 *                       proto, L4 length) || L4 segment is 0
 *                       (tcp_checksum / udp_checksum, packet_generator.cpp:204-305);
 *                       a UDP checksum field of 0 means "no checksum" (:303-304)
 *                       and counts as OK
 *   ORACLE_L34_UDP_NOCSUM  UDP with a zero checksum field.
 * The L4 segment ends at the IP total length: bytes after it (Ethernet
 * padding, trailers) are not part of it. */
#define ORACLE_L34_IPV4 0x01u
#define ORACLE_L34_IPV4_OK 0x02u
#define ORACLE_L34_L4 0x04u
#define ORACLE_L34_L4_OK 0x08u
#define ORACLE_L34_UDP_NOCSUM 0x10u
uint8_t oracle_l34_verify(const uint8_t* frame, size_t len);

/* TSO/GSO segmentation with VLAN insert/strip, materialised:
 * QueuePair::build_segments (src/queue_pair.cpp:212-278), the TX VLAN insert
 * (:320-331) and the RX VLAN strip (:389-395).  flags: ORACLE_SEG_* | tag.
 * Writes segment k's delivered bytes at out + k * stride, its length in
 * lens[k] and compute_checksum in csums[k].  Returns the segment count, -1
 * for InvalidMss, -2 for TooManySegments, -3 if a segment exceeds stride or
 * max_seg segments. */
#define ORACLE_SEG_TSO 0x10000u
#define ORACLE_SEG_VLAN_INSERT 0x20000u
#define ORACLE_SEG_VLAN_STRIP 0x40000u
#define ORACLE_SEG_VLAN_PRESENT 0x80000u
int oracle_tso_segment(const uint8_t* pkt, size_t len, uint16_t hdr_len, uint16_t mss, uint32_t flags,
                       uint8_t* out, size_t stride, size_t max_seg, uint32_t* lens, uint16_t* csums);

/* RoCEv2 ICRC as the reference computes it: nic::rocev2::IcrcCalculator
 * (src/rocev2/packet.cpp:14-56): CRC-32C, reflected polynomial 0x82F63B78,
 * table-driven byte at a time, initial value 0xFFFFFFFF, final xor
 * 0xFFFFFFFF, over the whole span (no field masking).  verify (:58-75): span
 * >= 4 bytes and calculate(span minus its last 4 bytes) equals those 4 bytes
 * read big-endian.  The reference TU is not buildable here (it includes
 * bit_fields); parity is pinned by the published CRC-32C vectors
 * (tests/golden/icrc_kat.json). */
uint32_t oracle_icrc_calculate(const uint8_t* buf, size_t len);
int oracle_icrc_verify(const uint8_t* buf, size_t len);

/* Batch loops over the functions above, for bench.py's CPU-baseline leg only
 * (one core; descriptors as in oracle_rx_batch).  out_csum receives every
 * frame's segment checksums back to back (at most 64 per frame); returns the
 * number written. */
size_t oracle_tso_checksum_batch(const uint8_t* frames, const uint64_t* desc, size_t n, const uint16_t* hdr_len,
                                 const uint16_t* mss, uint16_t* out_csum);
/* oracle_l34_verify over a packed batch (the CPU leg of bench.py's f3 row). */
void oracle_l34_batch(const uint8_t* frames, const uint64_t* desc, size_t n, uint8_t* out_flags);
void oracle_icrc_batch(const uint8_t* frames, const uint64_t* desc, size_t n, uint32_t* out_crc);

#ifdef __cplusplus
}
#endif

#endif
