// cq.hip — row f1's RSS dispatch into per-queue completion rings: every
// Success RX completion posted into the CompletionQueue of its RSS queue, on
// the device (nic::CompletionQueue::post_completion / poll_completion,
// src/completion_queue.cpp:30-53: a full ring refuses the entry; producer,
// consumer and count wrap at the ring size).  The batched stage hands over
// its completions already grouped by queue in posting order
// (nicgpu_qp_group: queue q's are which[start[q], end[q])), so queue q's
// i-th completion goes to slot (producer + i) % ring when i < ring - count —
// the order CompletionQueue::post_completion sees them.  DESIGN.md §4.6.

#include "common.h"
#include "host.h"

#include <cstring>
#include <vector>

using namespace nicgpu_detail;

struct nicgpu_cq_set {
  int device = 0;
  size_t nq = 0, ring = 0;
  nicgpu_completion* entries = nullptr;  // [nq][ring]
  uint32_t* state[2] = {nullptr, nullptr};  // [4][nq]: producer | consumer | count | refused, the current one ...
  int cur = 0;                              // ... and the one a post writes (reads of the current one race none)
  uint32_t* lists = nullptr;                // [2][nq]: the post's start | end
};

namespace {

constexpr unsigned kCqBlock = 256;
constexpr unsigned kCqBlocksPerQueue = 8;

__global__ __launch_bounds__(kCqBlock) void cq_post_kernel(nicgpu_completion* __restrict__ entries, uint32_t ring,
                                                           uint32_t nq, const uint32_t* __restrict__ in,
                                                           uint32_t* __restrict__ out,
                                                           const nicgpu_completion* __restrict__ rxc,
                                                           const uint32_t* __restrict__ which,
                                                           const uint32_t* __restrict__ lists, uint32_t nlists) {
  const uint32_t q = blockIdx.x / kCqBlocksPerQueue, part = blockIdx.x % kCqBlocksPerQueue;
  if (q >= nq) return;
  const uint32_t prod = in[q], cons = in[nq + q], count = in[2 * nq + q], refused = in[3 * nq + q];
  const uint32_t s = q < nlists ? lists[q] : 0u, e = q < nlists ? lists[nlists + q] : 0u;
  const uint32_t m = e > s ? e - s : 0u;
  const uint32_t space = ring - count;
  const uint32_t posted = m < space ? m : space;
  for (uint32_t i = part * kCqBlock + threadIdx.x; i < posted; i += kCqBlocksPerQueue * kCqBlock) {
    uint32_t slot = prod + i;
    if (slot >= ring) slot -= ring;  // prod < ring, i < ring
    entries[(size_t) q * ring + slot] = rxc[which[s + i]];
  }
  if (part == 0 && threadIdx.x == 0) {
    uint32_t np = prod + posted;
    if (np >= ring) np -= ring;
    out[q] = np;
    out[nq + q] = cons;
    out[2 * nq + q] = count + posted;
    out[3 * nq + q] = refused + (m - posted);
  }
}

}  // namespace

extern "C" {

int nicgpu_cq_create(nicgpu_cq_set** out, int device, size_t nq, size_t ring_size) {
  if (!out || nq == 0 || nq > 65536 || ring_size == 0 || ring_size > 0x7FFFFFFFu) return NICGPU_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NICGPU_ERR_NO_DEVICE;
  DeviceGuard g(device);
  auto* c = new nicgpu_cq_set();
  c->device = device;
  c->nq = nq;
  c->ring = ring_size;
  if (hipMalloc(&c->entries, nq * ring_size * sizeof(nicgpu_completion)) != hipSuccess ||
      hipMalloc(&c->state[0], 4 * nq * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->state[1], 4 * nq * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->lists, 2 * nq * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->state[0], 0, 4 * nq * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->entries, 0, nq * ring_size * sizeof(nicgpu_completion)) != hipSuccess) {
    nicgpu_cq_destroy(c);
    return NICGPU_ERR_NOMEM;
  }
  *out = c;
  return NICGPU_OK;
}

int nicgpu_cq_destroy(nicgpu_cq_set* c) {
  if (!c) return NICGPU_ERR_INVALID;
  DeviceGuard g(c->device);
  void* bufs[] = {c->entries, c->state[0], c->state[1], c->lists};
  for (void* b : bufs)
    if (b) (void) hipFree(b);
  delete c;
  return NICGPU_OK;
}

int nicgpu_cq_post(nicgpu_cq_set* c, const nicgpu_completion* rxc, const uint32_t* which, const uint32_t* start,
                   const uint32_t* end, size_t nlists, void* stream) {
  if (!c || nlists > c->nq || (nlists && (!start || !end))) return NICGPU_ERR_INVALID;
  DeviceGuard g(c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // a list longer than the batch's completions is the caller's error; the
  // lists themselves are checked on the host (they are host arrays)
  for (size_t q = 0; q < nlists; ++q)
    if (end[q] < start[q]) return NICGPU_ERR_INVALID;
  bool any = false;
  for (size_t q = 0; q < nlists && !any; ++q) any = end[q] > start[q];
  if (any && (!rxc || !which)) return NICGPU_ERR_INVALID;
  std::vector<uint32_t> l(2 * (nlists ? nlists : 1));
  if (nlists) {
    std::memcpy(l.data(), start, nlists * sizeof(uint32_t));
    std::memcpy(l.data() + nlists, end, nlists * sizeof(uint32_t));
    // (pageable source: the copy is staged before the call returns)
    int st = hip_status(hipMemcpyAsync(c->lists, l.data(), 2 * nlists * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    if (st != NICGPU_OK) return st;
  }
  const int nxt = c->cur ^ 1;
  hipLaunchKernelGGL(cq_post_kernel, dim3((unsigned) (c->nq * kCqBlocksPerQueue)), dim3(kCqBlock), 0, s, c->entries,
                     (uint32_t) c->ring, (uint32_t) c->nq, c->state[c->cur], c->state[nxt], rxc, which, c->lists,
                     (uint32_t) nlists);
  int st = hip_status(hipGetLastError());
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));  // the lists buffer and state are reused next call
  if (st == NICGPU_OK) c->cur = nxt;
  return st;
}

int nicgpu_cq_state(const nicgpu_cq_set* c, uint32_t* out_host, void* stream) {
  if (!c || !out_host) return NICGPU_ERR_INVALID;
  DeviceGuard g(c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int st = hip_status(hipMemcpyAsync(out_host, c->state[c->cur], 4 * c->nq * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  return st;
}

int nicgpu_cq_poll(nicgpu_cq_set* c, uint32_t q, nicgpu_completion* out_host, size_t max, size_t* got, void* stream) {
  if (!c || !got || q >= c->nq || (max && !out_host)) return NICGPU_ERR_INVALID;
  *got = 0;
  DeviceGuard g(c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<uint32_t> st4(4 * c->nq);
  int st = nicgpu_cq_state(c, st4.data(), stream);
  if (st != NICGPU_OK) return st;
  const uint32_t nq = (uint32_t) c->nq, ring = (uint32_t) c->ring;
  uint32_t cons = st4[nq + q], count = st4[2 * nq + q];
  const uint32_t k = (uint32_t) (max < count ? max : count);
  const nicgpu_completion* base = c->entries + (size_t) q * ring;
  const uint32_t first = k < ring - cons ? k : ring - cons;  // up to the ring's end, then from slot 0
  if (first)
    st = hip_status(hipMemcpyAsync(out_host, base + cons, first * sizeof(nicgpu_completion), hipMemcpyDeviceToHost, s));
  if (st == NICGPU_OK && k > first)
    st = hip_status(hipMemcpyAsync(out_host + first, base, (k - first) * sizeof(nicgpu_completion), hipMemcpyDeviceToHost, s));
  cons = (cons + k) % ring;
  count -= k;
  const uint32_t upd[2] = {cons, count};
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(c->state[c->cur] + nq + q, &upd[0], 4, hipMemcpyHostToDevice, s));
  if (st == NICGPU_OK) st = hip_status(hipMemcpyAsync(c->state[c->cur] + 2 * nq + q, &upd[1], 4, hipMemcpyHostToDevice, s));
  if (st == NICGPU_OK) st = hip_status(hipStreamSynchronize(s));
  if (st == NICGPU_OK) *got = k;
  return st;
}

}  // extern "C"
