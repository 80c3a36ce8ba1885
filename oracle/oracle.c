/*
 * oracle.c — CPU restatement of the smart_nic RX checksum + RSS path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Deliberately written as the
 * reference writes it — scalar, byte-pair, bit-serial — so it doubles as the
 * "port" CPU baseline in bench.py.  Parity of this file with the reference is
 * pinned by tests/test_oracle_golden.py against tests/golden/ (generated from
 * the compiled reference by oracle/gen_golden.cpp).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* src/checksum.cpp:10-34 — big-endian 16-bit words, carry folded after every
 * add (:19-21), odd trailing byte added as the high byte (:24-31), ~sum. */
uint16_t oracle_compute_checksum(const uint8_t* buf, size_t len) {
  uint32_t sum = 0;
  for (size_t i = 0; i + 1 < len; i += 2) {
    uint16_t word = (uint16_t) (((uint16_t) buf[i] << 8) | (uint16_t) buf[i + 1]);
    sum += word;
    if (sum & 0x10000u) {
      sum = (sum & 0xFFFFu) + 1u;
    }
  }
  if (len & 1u) {
    uint16_t last = (uint16_t) ((uint16_t) buf[len - 1] << 8);
    sum += last;
    if (sum & 0x10000u) {
      sum = (sum & 0xFFFFu) + 1u;
    }
  }
  return (uint16_t) ~sum;
}

/* src/rss.cpp:10-13 */
void oracle_default_key(uint8_t out[20]) {
  static const uint8_t k[20] = {0x6D, 0x5A, 0x56, 0x6B, 0x65, 0x4E, 0x67, 0x6E, 0x67, 0x55,
                                0x6A, 0x6B, 0x61, 0x4F, 0x6B, 0x65, 0x6F, 0x49, 0x4D, 0x42};
  memcpy(out, k, 20);
}

/* src/rss.cpp:63-94 — for every set data bit (MSB first within a byte, :75-77)
 * XOR in the 32-bit window whose k-th bit is key bit (bit + k) % key_bits
 * (:83-89); wraps when the data is longer than the key. */
uint32_t oracle_toeplitz(const uint8_t* key, size_t key_len, const uint8_t* data, size_t len) {
  if (key_len == 0 || len == 0) {
    return 0;
  }
  const size_t key_bits = key_len * 8;
  const size_t data_bits = len * 8;
  uint32_t hash_value = 0;
  for (size_t bit = 0; bit < data_bits; ++bit) {
    size_t byte_idx = bit / 8;
    size_t bit_idx = 7 - (bit % 8);
    if (((data[byte_idx] >> bit_idx) & 1u) == 0) {
      continue;
    }
    uint32_t segment = 0;
    for (size_t k = 0; k < 32; ++k) {
      size_t key_bit = (bit + k) % key_bits;
      size_t key_byte_idx = key_bit / 8;
      size_t key_bit_idx = 7 - (key_bit % 8);
      uint32_t key_bit_val = (key[key_byte_idx] >> key_bit_idx) & 1u;
      segment = (segment << 1) | key_bit_val;
    }
    hash_value ^= segment;
  }
  return hash_value;
}

/* src/rss.cpp:49-61 — idx = h % table.size(); return table[idx]. */
uint16_t oracle_select_queue(const uint8_t* key, size_t key_len, const uint16_t* table,
                             size_t table_n, const uint8_t* data, size_t len, uint32_t* hash,
                             uint32_t* tidx) {
  uint32_t h = oracle_toeplitz(key, key_len, data, len);
  uint32_t idx = (uint32_t) (h % (uint32_t) table_n);
  if (hash) *hash = h;
  if (tidx) *tidx = idx;
  return table[idx];
}

static inline unsigned be16(const uint8_t* p) { return ((unsigned) p[0] << 8) | p[1]; }

/* Tuple extraction.  The reference has no parser; this is
 * the build's own definition, restated here so the GPU kernel can be checked
 * against it.  Layout per src/packet_generator.cpp:46-166 (Ethernet, optional
 * 0x8100 / 0x88A8 tags, include/nic/offload.h:20-22), IPv4 src@+12 dst@+16,
 * ports at l3 + 4*IHL; tuple order src_ip|dst_ip|sport|dport as
 * tests/tutorial_lesson8_test.cpp:20-35.  Non-first fragments and non-TCP/UDP
 * hash the IP pair only; non-IP frames hash nothing (h = 0). */
size_t oracle_extract_tuple(const uint8_t* f, size_t len, int mode, size_t raw_off, size_t raw_len,
                            uint8_t out[64]) {
  if (mode == ORACLE_TUPLE_NONE) {
    return 0;
  }
  if (mode == ORACLE_TUPLE_RAW) {
    if (raw_off >= len) return 0;
    size_t end = raw_off + raw_len;
    if (end > len) end = len;
    memcpy(out, f + raw_off, end - raw_off);
    return end - raw_off;
  }
  if (len < 14) return 0;
  size_t l3 = 14;
  unsigned et = be16(f + 12);
  for (int tags = 0; tags < 2 && (et == 0x8100u || et == 0x88A8u); ++tags) {
    if (len < l3 + 4) return 0;
    et = be16(f + l3 + 2);
    l3 += 4;
  }
  if (et == 0x0800u) {
    if (len < l3 + 20) return 0;
    if ((f[l3] >> 4) != 4) return 0;
    size_t ihl = (size_t) (f[l3] & 15u) * 4;
    if (ihl < 20) return 0;
    memcpy(out, f + l3 + 12, 8);
    unsigned proto = f[l3 + 9];
    unsigned frag = be16(f + l3 + 6) & 0x3FFFu;
    size_t l4 = l3 + ihl;
    if ((proto == 6u || proto == 17u) && frag == 0 && l4 + 4 <= len) {
      memcpy(out + 8, f + l4, 4);
      return 12;
    }
    return 8;
  }
  if (et == 0x86DDu) {
    if (len < l3 + 40) return 0;
    if ((f[l3] >> 4) != 6) return 0;
    memcpy(out, f + l3 + 8, 32);
    unsigned nh = f[l3 + 6];
    if ((nh == 6u || nh == 17u) && l3 + 44 <= len) {
      memcpy(out + 32, f + l3 + 40, 4);
      return 36;
    }
    return 32;
  }
  return 0;
}

void oracle_rx_batch(const uint8_t* frames, const uint64_t* desc, size_t n, int mode,
                     size_t raw_off, size_t raw_len, const uint8_t* key, size_t key_len,
                     const uint16_t* table, size_t table_n, uint16_t* csum, uint32_t* hash,
                     uint16_t* queue, uint32_t* tidx, uint64_t* hits) {
  uint8_t tuple[64];
  for (size_t i = 0; i < n; ++i) {
    uint64_t off = desc[i] & ((1ull << 40) - 1);
    size_t len = (size_t) (desc[i] >> 40);
    const uint8_t* f = frames + off;
    if (csum) csum[i] = oracle_compute_checksum(f, len);
    if (mode == ORACLE_TUPLE_NONE) continue;
    size_t tl = oracle_extract_tuple(f, len, mode, raw_off, raw_len, tuple);
    uint32_t h, idx;
    uint16_t q = oracle_select_queue(key, key_len, table, table_n, tuple, tl, &h, &idx);
    if (hash) hash[i] = h;
    if (queue) queue[i] = q;
    if (tidx) tidx[i] = idx;
    if (hits) hits[idx] += 1;
  }
}

/* src/queue_pair.cpp:212-278 (build_segments) + :434-447 (per-segment RX
 * checksum).  kMinMss = 1, kMaxMss = 9000, kMaxTsoSegments = 64
 * (include/nic/offload.h:14-16). */
int oracle_tso_segment_checksums(const uint8_t* pkt, size_t len, uint16_t hdr_len, uint16_t mss,
                                 int segmentation_enabled, uint16_t* out, size_t max_out) {
  int enabled = segmentation_enabled && mss > 0 && len > mss;
  if (!enabled) {
    if (max_out < 1) return -3;
    out[0] = oracle_compute_checksum(pkt, len);
    return 1;
  }
  if (mss < 1 || mss > 9000) return -1;
  if (hdr_len > len) return -1;
  size_t h = hdr_len;
  if (h >= len) {
    if (max_out < 1) return -3;
    out[0] = oracle_compute_checksum(pkt, len);
    return 1;
  }
  size_t nseg = (len - h + mss - 1) / mss;
  if (nseg > 64) return -2;
  if (nseg > max_out) return -3;
  uint8_t* buf = (uint8_t*) malloc(h + mss);
  if (!buf) return -3;
  size_t k = 0;
  for (size_t p = h; p < len; p += mss, ++k) {
    size_t chunk = (len - p < mss) ? (len - p) : mss;
    memcpy(buf, pkt, h);
    memcpy(buf + h, pkt + p, chunk);
    out[k] = oracle_compute_checksum(buf, h + chunk);
  }
  free(buf);
  return (int) k;
}

/* internet_checksum / ipv4_checksum (packet_generator.cpp:200-202, 342-360):
 * big-endian word sum, odd byte as a high byte, folded, complemented. */
static uint16_t inet_csum(uint32_t sum, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i += 2) sum += ((uint32_t) p[i] << 8) | (i + 1 < n ? p[i + 1] : 0u);
  while (sum >> 16) sum = (sum & 0xFFFFu) + (sum >> 16);
  return (uint16_t) ~sum;
}

uint8_t oracle_l34_verify(const uint8_t* f, size_t len) {
  if (len < 14) return 0;
  size_t l3 = 14;
  unsigned et = be16(f + 12);
  for (int tags = 0; tags < 2 && (et == 0x8100u || et == 0x88A8u); ++tags) {
    if (len < l3 + 4) return 0;
    et = be16(f + l3 + 2);
    l3 += 4;
  }
  if (et != 0x0800u || len < l3 + 20 || (f[l3] >> 4) != 4) return 0;
  const size_t ihl = (size_t) (f[l3] & 15u) * 4;
  if (ihl < 20 || l3 + ihl > len) return 0;
  uint8_t flags = ORACLE_L34_IPV4;
  if (inet_csum(0, f + l3, ihl) == 0) flags |= ORACLE_L34_IPV4_OK;
  const unsigned proto = f[l3 + 9];
  const unsigned frag = be16(f + l3 + 6) & 0x3FFFu;
  const size_t total = be16(f + l3 + 2);
  if ((proto != 6u && proto != 17u) || frag != 0 || total < ihl || l3 + total > len) return flags;
  const size_t seg = total - ihl;
  if (seg < (proto == 6u ? 20u : 8u)) return flags;
  flags |= ORACLE_L34_L4;
  const uint8_t* l4 = f + l3 + ihl;
  if (proto == 17u && be16(l4 + 6) == 0) return flags | ORACLE_L34_L4_OK | ORACLE_L34_UDP_NOCSUM;
  /* pseudo-header: src_ip, dst_ip, zero, protocol, L4 length (tcp_checksum :208-225) */
  uint32_t sum = be16(f + l3 + 12) + be16(f + l3 + 14) + be16(f + l3 + 16) + be16(f + l3 + 18) + proto +
                 (uint32_t) (seg & 0xFFFFu);
  if (inet_csum(sum, l4, seg) == 0) flags |= ORACLE_L34_L4_OK;
  return flags;
}

/* IcrcCalculator::kCrc32cTable / update_crc / calculate / verify
 * (src/rocev2/packet.cpp:14-75), restated byte at a time. */
static uint32_t crc32c_table[256];
static int crc32c_ready = 0;

static void crc32c_init(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc32c_table[i] = c;
  }
  crc32c_ready = 1;
}

uint32_t oracle_icrc_calculate(const uint8_t* buf, size_t len) {
  if (!crc32c_ready) crc32c_init();
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < len; ++i) crc = crc32c_table[(uint8_t) (crc ^ buf[i])] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}

int oracle_icrc_verify(const uint8_t* buf, size_t len) {
  if (len < 4) return 0;
  const uint8_t* t = buf + len - 4;
  const uint32_t stored = ((uint32_t) t[0] << 24) | ((uint32_t) t[1] << 16) | ((uint32_t) t[2] << 8) | t[3];
  return oracle_icrc_calculate(buf, len - 4) == stored;
}

int oracle_tso_segment(const uint8_t* pkt, size_t len, uint16_t hdr_len, uint16_t mss, uint32_t flags,
                       uint8_t* out, size_t stride, size_t max_seg, uint32_t* lens, uint16_t* csums) {
  /* build_segments (queue_pair.cpp:212-278) */
  const int enabled = (flags & ORACLE_SEG_TSO) && mss > 0 && len > mss;
  size_t h = len, nseg = 1;
  if (enabled) {
    if (mss < 1 || mss > 9000) return -1;
    if (hdr_len > len) return -1;
    if (hdr_len < len) {
      h = hdr_len;
      nseg = (len - h + mss - 1) / mss;
      if (nseg > 64) return -2;
    }
  }
  if (nseg > max_seg) return -3;
  const int insert = (flags & ORACLE_SEG_VLAN_INSERT) != 0;
  const unsigned tag = flags & 0xFFFFu;
  for (size_t k = 0; k < nseg; ++k) {
    const size_t p = h + k * mss;
    const size_t chunk = h < len ? ((len - p < mss) ? len - p : mss) : 0;
    /* segment = header || chunk; TX VLAN insert prepends 81 00 tag (:324-331) */
    size_t n = 0;
    uint8_t* s = (uint8_t*) malloc(h + chunk + 4);
    if (!s) return -3;
    if (insert) {
      s[0] = 0x81; s[1] = 0x00; s[2] = (uint8_t) (tag >> 8); s[3] = (uint8_t) tag;
      n = 4;
    }
    memcpy(s + n, pkt, h);
    n += h;
    memcpy(s + n, pkt + p, chunk);
    n += chunk;
    /* RX strip of the first 4 bytes when the segment carries a VLAN (:389-395) */
    const int has_vlan = insert || (flags & ORACLE_SEG_VLAN_PRESENT);
    size_t from = 0;
    if ((flags & ORACLE_SEG_VLAN_STRIP) && has_vlan && n >= 4) from = 4;
    if (n - from > stride) { free(s); return -3; }
    memcpy(out + k * stride, s + from, n - from);
    lens[k] = (uint32_t) (n - from);
    csums[k] = oracle_compute_checksum(s + from, n - from);
    free(s);
  }
  return (int) nseg;
}

/* ---- batch loops (bench.py CPU baseline) ---- */
size_t oracle_tso_checksum_batch(const uint8_t* frames, const uint64_t* desc, size_t n, const uint16_t* hdr_len,
                                 const uint16_t* mss, uint16_t* out_csum) {
  size_t w = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t off = desc[i] & ((1ull << 40) - 1);
    const size_t len = (size_t) (desc[i] >> 40);
    const int r = oracle_tso_segment_checksums(frames + off, len, hdr_len[i], mss[i], 1, out_csum + w, 64);
    if (r > 0) w += (size_t) r;
  }
  return w;
}

void oracle_l34_batch(const uint8_t* frames, const uint64_t* desc, size_t n, uint8_t* out_flags) {
  for (size_t i = 0; i < n; ++i) {
    const uint64_t off = desc[i] & ((1ull << 40) - 1);
    out_flags[i] = oracle_l34_verify(frames + off, (size_t) (desc[i] >> 40));
  }
}

void oracle_icrc_batch(const uint8_t* frames, const uint64_t* desc, size_t n, uint32_t* out_crc) {
  for (size_t i = 0; i < n; ++i) {
    const uint64_t off = desc[i] & ((1ull << 40) - 1);
    out_crc[i] = oracle_icrc_calculate(frames + off, (size_t) (desc[i] >> 40));
  }
}
