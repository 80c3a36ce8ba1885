// nic/rx_stage.h — batched QueuePair RX stage on the GPU.
//
// The reference moves one TX descriptor at a time through
// QueuePair::process_once (src/queue_pair.cpp:67-119) and its helpers
// (validate_mtu :195-210, build_segments :212-278, process_segments :303-369,
// handle_rx_segment :385-460).  BatchedQueuePair runs a whole batch of TX
// descriptors against a batch of RX descriptors with the same observable
// results:
//   - every TX and RX CompletionEntry, in posting order, with identical fields;
//   - QueuePairStats, counter by counter;
//   - the bytes DMA-written into the RX buffers (TSO/GSO segments, VLAN
//     insert/strip);
//   - the same interrupt sequence (fire_tx_interrupt / fire_rx_interrupt),
//     delivered to a callback instead of an InterruptDispatcher.
// It adds RSS dispatch, which the reference lacks: every frame delivered with
// RX status Success is hashed by an RssEngine and listed under its queue.
//
// Host memory is either a device-resident image (DeviceHostMemory): host
// address a is byte a of the image; or the reference's own HostMemory
// (host_memory.h:49-73; e.g. SimpleHostMemory, simple_host_memory.cpp:16,
// 70-109): its flat window translate(0, size) is registered with the GPU and
// mirrored in HBM, each batch stages only the TX bytes it reads up and writes
// only the bytes it delivers back (see process_batch(HostMemory&, ...)).  In
// both, the bounds rule of SimpleHostMemory::translate_view
// (simple_host_memory.cpp:89-96) decides DMA faults.  Descriptors arrive
// already popped from their rings (DescriptorRing owns ring/doorbell state;
// the stage starts where pop_descriptor ends).
//
// GPU work per batch: one checksum pass over the TX bytes (the per-piece
// ones'-complement sums every TX/RX verify needs), one gather that
// materialises the written segments into the RX buffers, and one RX offload
// launch over the delivered frames (RSS).  The control flow between them —
// ring consumption, first-failure aborts, statuses, stats — is sequential in
// the reference.  It is resolved exactly from those sums: on the device when
// the batch's buffers are disjoint and no interrupt callback is set (ring
// positions by relaxation, nicgpu_qp_*; the host finishes in order after the
// first packet whose position did not settle), otherwise on the host.
//
// Buffers that overlap: the reference writes segment after
// segment, so of two RX buffers that share bytes the later write wins, and a
// TX buffer that overlaps an earlier RX buffer of the batch is read after that
// write.  When any RX buffer overlaps another RX buffer or a TX buffer
// (buffers_disjoint() is false), the batch runs as sub-batches, each ending
// before the first TX descriptor that reads bytes an earlier descriptor of the
// sub-batch wrote; within a sub-batch overlapping writes go to successive
// gather launches in posting order ("layers", schedule_writes()), sources are
// read from a copy of the image when a write lands on any source, and each
// layer's delivered frames are hashed before the next layer can overwrite
// them.  The results are the sequential reference's in every case.
//
// Faults of a HostMemory beyond the bounds rule (SimpleHostMemory's
// FaultInjector and AddressTranslator, simple_host_memory.cpp:76-87): by
// default the caller asserts the window is flat — no injector, no translator;
// bind_image probes translate() at three addresses and refuses a window it
// sees moved, but it cannot prove flatness.  With
// BatchedQueuePairConfig::host_memory_faults every DMA access goes through the
// memory's own translate_const / translate, so injected faults and IOMMU
// faults post the reference's Fault completions (queue_pair.cpp:96-103,
// 416-426); see that flag for what it requires.
//
// Failure: process_batch (or submit / collect) throws nic::GpuError on a HIP
// failure.  stats() is then unchanged, but the memory image may hold some of
// the batch's writes and the RSS engine's stats some of its hashes.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <span>
#include <utility>
#include <vector>

#include "nic/gpu_batch.h"
#include "nic/offload.h"
#include "nic/rss.h"
#include "nic/tx_rx.h"

#if __has_include("nic/completion_queue.h")
#include "nic/completion_queue.h"  // reference build: its CompletionEntry
#else
namespace nic {
// Same members, order and defaults as include/nic/completion_queue.h:13-26.
struct CompletionEntry {
  std::uint16_t queue_id{0};
  std::uint16_t descriptor_index{0};
  std::uint32_t status{0};
  bool checksum_offloaded{false};
  bool checksum_verified{false};
  bool tso_performed{false};
  bool gso_performed{false};
  bool vlan_inserted{false};
  bool vlan_stripped{false};
  bool gro_aggregated{false};
  std::uint16_t segments_produced{1};
  std::uint16_t vlan_tag{0};
};
static_assert(sizeof(CompletionEntry) == 20);
}  // namespace nic
#endif

#if __has_include("nic/queue_pair.h")
#include "nic/queue_pair.h"  // reference build: its QueuePairStats
#else
namespace nic {
// Same members and order as include/nic/queue_pair.h:36-53.
struct QueuePairStats {
  std::uint64_t tx_packets{0};
  std::uint64_t rx_packets{0};
  std::uint64_t tx_bytes{0};
  std::uint64_t rx_bytes{0};
  std::uint64_t drops_checksum{0};
  std::uint64_t drops_no_rx_desc{0};
  std::uint64_t drops_buffer_small{0};
  std::uint64_t drops_mtu_exceeded{0};
  std::uint64_t drops_invalid_mss{0};
  std::uint64_t drops_too_many_segments{0};
  std::uint64_t tx_tso_segments{0};
  std::uint64_t tx_gso_segments{0};
  std::uint64_t tx_vlan_insertions{0};
  std::uint64_t rx_vlan_strips{0};
  std::uint64_t rx_checksum_verified{0};
  std::uint64_t rx_gro_aggregated{0};
};
}  // namespace nic
#endif

struct nicgpu_segment_write;  // nicgpu.h

#if __has_include("nic/host_memory.h")
#include "nic/host_memory.h"  // reference build: its HostMemory interface
#else
namespace nic {
// Same declarations, in the same order (so the same vtable layout), as
// include/nic/host_memory.h:9-73: a reference HostMemory (SimpleHostMemory)
// compiled against that header is passed to this library as it is.
using HostAddress = std::uint64_t;
struct HostMemoryConfig {
  std::size_t size_bytes{0};
  std::size_t page_size{4096};
  bool iommu_enabled{false};
};
enum class HostMemoryError : std::uint8_t { None, OutOfBounds, IommuFault, FaultInjected };
struct HostMemoryResult {
  HostMemoryError error{HostMemoryError::None};
  std::size_t bytes_processed{0};
  [[nodiscard]] bool ok() const noexcept { return error == HostMemoryError::None; }
};
struct HostMemoryView {
  std::byte* data{nullptr};
  std::size_t length{0};
  HostAddress address{0};
};
struct ConstHostMemoryView {
  const std::byte* data{nullptr};
  std::size_t length{0};
  HostAddress address{0};
};
class HostMemory {
public:
  virtual ~HostMemory() = default;
  [[nodiscard]] virtual HostMemoryConfig config() const noexcept = 0;
  [[nodiscard]] virtual HostMemoryResult translate(HostAddress address, std::size_t length, HostMemoryView& view) = 0;
  [[nodiscard]] virtual HostMemoryResult translate_const(HostAddress address, std::size_t length,
                                                         ConstHostMemoryView& view) const = 0;
  [[nodiscard]] virtual HostMemoryResult read(HostAddress address, std::span<std::byte> buffer) const = 0;
  [[nodiscard]] virtual HostMemoryResult write(HostAddress address, std::span<const std::byte> data) = 0;
};
}  // namespace nic
#endif

namespace nic {

/// Device-resident image of the host memory the DMA engine addresses.  The
/// kernels read it in 16-B chunks: `base` must be 16-B aligned and the
/// allocation must cover `size` rounded up to a multiple of 16 (nicgpu.h,
/// "Batch layout in HBM").
struct DeviceHostMemory {
  std::byte* base{nullptr};  // device pointer; host address a <-> base[a]
  std::size_t size{0};
};

/// Descriptor arrays already in device memory — e.g. host-backed rings, whose
/// descriptors live in the image itself (mem.base + the ring's address).  The
/// stage copies them in stream order (no PCIe upload) and fetches host copies
/// only when a host step needs them (a ring whose RX buffers are not in
/// address order, a host tail, overlapping buffers).  The reference DMA-reads
/// each ring slot when it pops it (descriptor_ring.cpp:97-106), so an RX
/// buffer of the batch that overlaps the descriptor arrays inside the image
/// changes the descriptors popped after its write: such a batch runs on the
/// host path in sub-batches, each ending before the first TX descriptor whose
/// slot, or an RX slot it may pop, an earlier write touched, and the rest of
/// the descriptors are read again from the image (rx_stage_detail::RingSlots).
/// One case stays refused with GpuError (NICGPU_ERR_INVALID), found while
/// resolving, possibly after earlier sub-batches were written: a segment's
/// write that lands on an RX slot a later segment of the same TX descriptor
/// pops.
struct DeviceDescriptors {
  const TxDescriptor* tx{nullptr};
  std::size_t ntx{0};
  const RxDescriptor* rx{nullptr};
  std::size_t nrx{0};
};

struct BatchedQueuePairConfig {
  std::uint16_t queue_id{0};
  std::uint8_t weight{1};           // QueuePairConfig::weight (queue_pair.h:31): BatchedQueueManager's share (0 -> 1)
  std::size_t max_mtu{kJumboMtu};   // QueuePairConfig::max_mtu (queue_pair.h:32)
  bool enable_tx_interrupts{false};  // QueuePairConfig defaults (queue_pair.h:33-34)
  bool enable_rx_interrupts{true};
  /// Receives what InterruptDispatcher::on_completion would (queue_pair.cpp:371-383).
  std::function<void(std::uint16_t queue_id, const CompletionEntry&)> on_interrupt{};
  /// RSS over delivered frames; nullptr = no dispatch.  Not owned.
  RssEngine* rss{nullptr};
  TupleSpec tuple{};
  /// Threads for the host phases (plan, piece descriptors, resolve): 0 uses
  /// up to 16 on batches of 32 K descriptors and more (resolve stays
  /// sequential with an interrupt callback, or when most packets are
  /// multi-segment); 1 runs them all on the calling thread.  Workers are
  /// pinned to the allowed CPUs that follow the calling thread's.
  unsigned host_threads{0};
  /// Resolve on the device (nicgpu_qp_*, the decisions of qp_logic.h) when
  /// the batch's buffers do not overlap: the host then only moves descriptors
  /// and completions.  false: every batch is resolved on the host (the path
  /// the fuzz compares with the reference).  Interrupt callbacks do not change
  /// the path: every path resolves without firing them, and
  /// rx_stage_detail::replay_interrupts fires them from the batch's
  /// completions, in posting order, on the thread that completes the batch
  /// (process_batch, or collect for submitted batches).  Batches of more than
  /// NICGPU_QP_MAX_TX (2^32 / 256, about 16.7 M) TX descriptors, or more than
  /// NICGPU_QP_MAX_RX RX descriptors, take the host path (32-bit piece indices).
  bool device_resolve{true};
  /// Leave the results of device-resolved batches in device memory
  /// (RxBatchResult::dev) instead of copying them to the host vectors: for
  /// consumers that read completions, hashes and dispatch lists on the GPU.
  bool results_on_device{false};
  /// submit/collect: a batch's piece sums and resolve run beside the earlier
  /// pending batches' DMA writes (their own stream) when its TX frames lie
  /// outside every byte those writes can touch (the overlap check's bounds);
  /// otherwise — or when that is not known — they are redone after them.
  /// Results are the same either way.  Off by default: measured on C3 1 M
  ///  the resolve chain is as bandwidth-bound as the delivery
  /// beside it, so the overlap gains nothing at the default CU reserve and
  /// ≈ 4 % with 96 CUs kept free of delivery blocks.
  bool overlap_resolve{false};
  /// Device path: a batch in which no decision that moves ring positions reads
  /// a checksum (no TX verify, queue_pair.cpp:94-105; one segment per packet)
  /// skips its piece-sum pass over the TX frames; its RX verifies
  /// (:434-447) are made by the delivery from the bytes it writes — the bytes
  /// that verify covers — which patches any that fail into the reference's
  /// ChecksumError completion, and the statistics are corrected when the batch
  /// completes (nicgpu_qp_set_deferred_verify).  Results are the same either
  /// way (tests/cpp/rx_stage_gpu_fuzz.cpp).  NIC_DEFER_VERIFY=0 turns it off.
  bool defer_rx_verify{true};
  /// HostMemory batches: model the memory's own DMA faults.  Every TX read is
  /// the memory's translate_const(buffer_address, length) and every RX write
  /// its translate(buffer_address, size) — what DMAEngine::read / write reach
  /// (dma_engine.cpp:12-32) — so a FaultInjector or an IOMMU AddressTranslator
  /// that refuses an access makes the reference's Fault completion there
  /// (queue_pair.cpp:96-103, 416-426) and the ring positions that follow from
  /// it.  The reads are asked once per TX descriptor before the batch, the
  /// writes in posting order by the host resolve (the batch is resolved on the
  /// host; piece sums, DMA writes and RSS stay on the GPU).  Requires what
  /// every reference test's injector and translator are: functions of
  /// (address, length), and translators that map each access they allow onto
  /// itself (an IOMMU that grants or denies); a translation that moves an
  /// address throws GpuError (NICGPU_ERR_INVALID) — before anything is written
  /// when it is a TX read's.  Off: the caller asserts the memory is flat (no
  /// injector, no translator) and the bounds rule alone decides faults.
  bool host_memory_faults{false};
};

struct RxBatchResult {
  static constexpr std::uint16_t kNoQueue = 0xFFFF;
  std::size_t tx_processed{0};  // TX descriptors consumed (all of them)
  std::size_t rx_consumed{0};   // RX descriptors popped, in order from rx[0]
  std::vector<CompletionEntry> tx_completions;  // posting order
  std::vector<CompletionEntry> rx_completions;  // posting order
  /// Per RX completion: RSS hash / queue of the delivered frame
  /// (0 / kNoQueue unless status == Success and an RssEngine is configured).
  std::vector<std::uint32_t> rx_hash;
  std::vector<std::uint16_t> rx_queue;
  /// queues[q] = indices into rx_completions dispatched to RSS queue q.
  std::vector<std::vector<std::uint32_t>> queues;
  /// Wall time of each phase of process_batch (host clock, GPU phases
  /// include their stream synchronisation).
  /// With BatchedQueuePairConfig::results_on_device, for a batch resolved on
  /// the device (timings.device): the results in device memory, in the
  /// stage's buffers, and the vectors above (queues included) left empty.
  /// Valid until the stage's next process_batch() or submit(); ready when
  /// process_batch() / collect() returns.  Host-resolved batches fill the
  /// vectors as usual and leave this empty.
  struct DeviceResults {
    const CompletionEntry* tx_completions{nullptr};  // [ntx], posting order
    const CompletionEntry* rx_completions{nullptr};  // [nrx], posting order
    std::size_t ntx{0}, nrx{0};
    const std::uint32_t* rx_hash{nullptr};   // [nrx]; null without an RssEngine
    const std::uint16_t* rx_queue{nullptr};  // [nrx]; null without an RssEngine
    /// RX completion indices grouped by queue: queue q's are
    /// queue_which[queue_start[q] .. queue_end[q]) (host vectors, one entry per
    /// queue up to the largest with frames).
    const std::uint32_t* queue_which{nullptr};
    std::vector<std::uint32_t> queue_start, queue_end;
  } dev;
  struct Timings {
    double check_us{0};  // overlapping buffers? (nicgpu_qp_check on the device path, else buffers_disjoint)
    double plan_us{0}, sums_us{0}, resolve_us{0}, gather_us{0}, rss_us{0};
    double copy_us{0};   // device resolve: descriptors up, completions down
    bool device{false};     // resolved on the device
    bool host_tail{false};  // ... and the rest on the host (positions settled neither by relaxation nor by the walk)
    bool walked{false};     // ... positions made by the walk (8 relaxation steps did not settle them)
    bool overlapped{false};  // submit/collect: sums and resolve ran beside the earlier batches' DMA writes
    bool overlap_redone{false};  // ... but the frames lie where those write: redone after them
    bool deferred{false};   // RX verifies made by the delivery (BatchedQueuePairConfig::defer_rx_verify)
    bool host_image{false};  // run against a HostMemory: TX bytes staged up, delivered bytes written back
    bool staged_whole{false};  // ... the TX bytes' span went up in one copy (dense), else per descriptor
    unsigned replans{0};    // device plans redone because the first outgrew the piece buffers (at most 1)
    double irq_us{0};       // interrupt callbacks replayed (the whole replay, its waits included)
    double irq_wait_us{0};  // ... of which waiting for completions still landing
  } timings;
};

namespace rx_stage_detail {
struct SegmentWrite;
struct DmaWriteCheck;
struct RingSlots;
}

/// QueuePair::process_once over a batch (src/queue_pair.cpp:67-460).
class BatchedQueuePair {
public:
  explicit BatchedQueuePair(BatchedQueuePairConfig config);
  ~BatchedQueuePair();
  BatchedQueuePair(const BatchedQueuePair&) = delete;
  BatchedQueuePair& operator=(const BatchedQueuePair&) = delete;
  BatchedQueuePair(BatchedQueuePair&&) noexcept;
  BatchedQueuePair& operator=(BatchedQueuePair&&) noexcept;

  /// Process every descriptor of `tx` in order against the RX descriptors `rx`
  /// (the RX ring's contents, rx[0] first).  Synchronises `stream` (a
  /// hipStream_t; nullptr = default stream) before returning.
  RxBatchResult process_batch(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                              std::span<const RxDescriptor> rx, void* stream = nullptr);
  /// The same into `out`, reusing its storage: a caller that keeps one
  /// RxBatchResult across batches takes no page faults for the results.
  void process_batch(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                     RxBatchResult& out, void* stream = nullptr);

  /// Pipelined form of process_batch for a stream of batches: submit() puts
  /// the batch's descriptors on their way to the device and hands the rest
  /// (plan, resolve, DMA writes, RSS, downloads) to the stage's job thread,
  /// which works on `stream` in submission order; collect() waits for the
  /// oldest submitted batch and swaps its results into `out` (false: none
  /// pending).  At most three batches are pending, so batch k's completions
  /// come down while batch k+1 is resolved and batch k+2's descriptors go up.
  /// The descriptor arrays (and `mem`) must stay valid and unchanged until the
  /// batch is collected.  The results, the memory image and the statistics
  /// equal those of process_batch called in submission order; a batch's
  /// QueuePair and RSS statistics are added when it is collected, and a
  /// batch's error is thrown by its collect(), which also fires the batch's
  /// interrupt callbacks (on the caller's thread, in posting order).  Throws
  /// std::logic_error on a fourth submit() or a process_batch() while batches
  /// are pending.
  void submit(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
              void* stream = nullptr);
  bool collect(RxBatchResult& out);
  /// Both forms with descriptors already in device memory (DeviceDescriptors;
  /// they must stay valid until the batch is done or collected).
  void process_batch(const DeviceHostMemory& mem, const DeviceDescriptors& d, RxBatchResult& out,
                     void* stream = nullptr);
  void submit(const DeviceHostMemory& mem, const DeviceDescriptors& d, void* stream = nullptr);

  /// The same batch against the reference's HostMemory (host_memory.h:49-73),
  /// which is where QueuePair's DMAEngine reads and writes (dma_engine.cpp:12-32;
  /// queue_pair.cpp:86-92 reads each TX buffer, :416-426 writes each segment).
  /// The memory's window translate(0, config().size_bytes) must be flat and
  /// 16-B aligned (SimpleHostMemory without an address translator or fault
  /// injector: its std::vector, simple_host_memory.cpp:16); GpuError
  /// (NICGPU_ERR_INVALID) otherwise, before anything is read or written.  The
  /// window — exactly its bytes, so heap neighbours on its pages stay ordinary
  /// memory — is page-locked once (nicgpu_host_register, reference counted:
  /// stages bound to one memory share it; released when the stage binds
  /// another memory or is destroyed) and mirrored in HBM.  Per batch only
  /// the TX buffers' bytes go up (one copy of their span when it is dense,
  /// otherwise a gather of each buffer), the stage runs on the mirror, and
  /// exactly the bytes its DMA writes deliver are written back into the
  /// memory (a GPU kernel storing through the registered window); no other
  /// byte of the memory is touched.  Results, statistics, interrupts and the
  /// memory's bytes equal those of the reference QueuePair on the same memory.
  /// The memory must not be written by anyone else while a batch is pending.
  void process_batch(HostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                     RxBatchResult& out, void* stream = nullptr);
  RxBatchResult process_batch(HostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                              void* stream = nullptr);
  /// Pipelined: batch k's bytes are written back while batch k+1 is resolved
  /// and batch k+2's TX bytes go up; a batch that reads (or delivers into)
  /// bytes an earlier pending batch delivers into is ordered after that
  /// batch's write-back.  collect() returns once the batch's bytes are in the
  /// memory.  Mixing HostMemory and DeviceHostMemory batches in flight is not
  /// supported (std::logic_error).
  void submit(HostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
              void* stream = nullptr);
  [[nodiscard]] std::size_t pending() const noexcept;

  /// The batches processed or collected so far, counter by counter as the
  /// reference counts them; a submitted batch is added when it is collected
  /// (pending batches, whose deferred RX verifies may still correct their
  /// counts, are not in it).
  [[nodiscard]] const QueuePairStats& stats() const noexcept { return stats_; }
  void reset_stats() noexcept { stats_ = QueuePairStats{}; }
  [[nodiscard]] const BatchedQueuePairConfig& config() const noexcept { return config_; }

  struct Scratch;  // device, pinned and host buffers reused across batches (grown, never shrunk)
  struct Slot;     // one batch in flight on the device: its context, events and landing buffers
  struct HostImage;  // a registered HostMemory window and its HBM mirror

private:
  friend class BatchedQueueManager;
  // BatchedQueueManager's fused batch: the queue pairs' TX batches and RX
  // rings resolved as ONE device batch (nicgpu_qp_set_segments: each queue
  // pair's own queue id, MTU and ring), one plan / piece-sum / resolve /
  // delivery chain, the results split per queue pair (out[q], stats[q]).
  // `img` null: `mem` is the device image.  Returns false, having written
  // nothing, when the batch does not fit the fused path (overlapping or
  // unsorted buffers, positions that do not settle): the caller then runs the
  // queue pairs one by one.  Interrupts are the caller's to replay.
  // dev_desc: the spans point at device memory (copied in stream order after
  // `stream`'s earlier work; needs whole_check and no img).  whole_check: the
  // device checks the batch as one ring (the caller has not checked the queue
  // pairs against each other).
  bool process_queues(const DeviceHostMemory& mem, HostImage* img, std::span<const std::span<const TxDescriptor>> tx,
                      std::span<const std::span<const RxDescriptor>> rx, std::span<const BatchedQueuePairConfig> configs,
                      std::vector<RxBatchResult>& out, std::vector<QueuePairStats>& stats, void* stream,
                      bool dev_desc = false, bool whole_check = false);
  bool front_multi(Slot& sl, const DeviceHostMemory& mem, std::size_t ntx, std::size_t nrx, RxBatchResult& out,
                   void* stream, int& again, bool whole_check);
  void share_image(const BatchedQueuePair& owner);  // use owner's HostImage (one mirror per manager)
  // Device resolve of one batch in four steps: upload() sends the descriptors
  // up; front() plans and checks (false, nothing written, when the buffers
  // overlap), starts the resolve, enqueues the DMA writes and RSS of the
  // completions it settles and then waits for it; back() enqueues the rest of
  // the writes and starts the downloads (dispatch lists included) into `out`;
  // finish() waits for them and completes `out`.
  void upload(Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx, bool rx_beside);
  bool front(Slot& sl, const DeviceHostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
             QueuePairStats& stats, RxBatchResult& out, void* stream, int& disjoint, double& check_us);
  bool front_once(Slot& sl, const DeviceHostMemory& mem, std::span<const TxDescriptor> tx,
                  std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out, void* stream,
                  int& disjoint, double& check_us, int& again);
  // host-image batches (process_batch / submit with a HostMemory)
  HostImage& bind_image(HostMemory& mem, bool checked = false, std::byte* window = nullptr);
  // host_memory_faults: the batch's descriptors with refused reads moved out of
  // bounds (kept in the slot until collected) and the write verdicts
  std::span<const TxDescriptor> checked_tx(Slot& sl, HostMemory& mem, std::span<const TxDescriptor> tx,
                                           std::byte*& window);
  void image_prepare(Slot& sl, HostImage& img, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx);
  void image_host_path(Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
                       QueuePairStats& stats, RxBatchResult& out, void* stream, int disjoint, double& check_us);
  void image_stage(Slot& sl, std::size_t ntx, const TxDescriptor* tx_host, const void* tx_dev, void* stream);
  void* stage_stream() const;  // the stream host-image staging runs on
  void image_writeback(Slot& sl, const nicgpu_segment_write* writes_dev, std::size_t n, void* stream);
  void back(Slot& sl, const DeviceHostMemory& mem, RxBatchResult& out, void* stream);
  void deliver(Slot& sl, const DeviceHostMemory& mem, std::size_t a, std::size_t b, unsigned flags,
               const nicgpu_rss_ctx* rctx, std::uint64_t* hits, void* stream);
  void finish(Slot& sl, RxBatchResult& out, QueuePairStats* st);
  static void apply_fixups(Slot& sl, std::size_t s, QueuePairStats& st);
  void enqueue(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
               const DeviceDescriptors* d, void* stream, HostImage* img = nullptr);
  // true when a DMA write of the batch can land on its descriptor arrays inside
  // the image (then *slots their image offsets: the host path re-reads them)
  bool rings_written(Slot& sl, const DeviceHostMemory& mem, void* stream, rx_stage_detail::RingSlots* slots);
  void fire_interrupts(RxBatchResult& r, Slot* sl = nullptr);  // config_.on_interrupt over r's completions
  std::pair<std::span<const TxDescriptor>, std::span<const RxDescriptor>> host_spans(
      Slot& sl, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx, void* stream);
  // the host path (buffers_disjoint unless `disjoint` is known, then run_batch)
  // (applied: every DMA write made is appended — a host-image batch writes them back)
  void on_host(const DeviceHostMemory& mem, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx,
               QueuePairStats& stats, RxBatchResult& out, void* stream, int disjoint, double& check_us,
               std::vector<rx_stage_detail::SegmentWrite>* applied = nullptr,
               const rx_stage_detail::DmaWriteCheck* wcheck = nullptr, const rx_stage_detail::RingSlots* slots = nullptr);
  BatchedQueuePairConfig config_;
  BatchedQueuePairConfig quiet_;  // config_ without the interrupt callback (every resolve; replayed after)
  bool defer_multi_ = false;      // process_queues: this fused batch may defer its RX verifies
  QueuePairStats stats_{};
  std::unique_ptr<Scratch> scratch_;
};

// Building blocks of process_batch, public so that the host logic can be
// tested without a GPU (the piece sums then come from a CPU checker).
namespace rx_stage_detail {

/// A HostMemory's own verdict on each DMA write (host_memory_faults): true
/// when translate(address, length) allows it.  Asked by the host resolve in
/// posting order, once per write the bounds rule allows.
struct DmaWriteCheck {
  virtual ~DmaWriteCheck() = default;
  virtual bool write_ok(std::uint64_t address, std::uint64_t length) const = 0;
};

/// A byte range of host memory whose ones'-complement sum the GPU computes.
struct Piece {
  std::uint64_t addr;
  std::uint32_t len;  // <= NICGPU_MAX_PACKET
};

/// Which pieces make up the bytes each decision needs, per TX descriptor.
//   kNoBytes    no decision reads the bytes (DMA read fault, or dropped before
//               any checksum is needed)
//   kPlain      the segment is the whole packet: pieces [0, min(4, L)) then
//               [4, L) in runs of <= 65534 bytes
//   kSegmented  H >= 4: [0, 4), [4, H), then chunk k = [H + k*mss, +len_k);
//               H < 4:  [0, H), then per chunk [.., +min(4 - H, len_k)) and its rest
//   kPlainSplit (split plans, the device stage's) the whole packet in runs of
//               <= 65534 bytes: one piece below 64 KiB, the first piece's sum
//               taken split as its first min(4, L) bytes and the rest
// Segment sums are composed from pieces (first 4 bytes | the rest, so that a
// VLAN strip of a segment's first 4 bytes, queue_pair.cpp:392-395, is exact).
struct PacketPlan {
  enum Kind : std::uint8_t { kNoBytes, kPlain, kSegmented, kPlainSplit };
  Kind kind{kNoBytes};
  std::uint32_t nseg{0};  // segments build_segments produces (kSegmented)
  std::uint32_t first_piece{0};
  std::uint32_t npieces{0};
  std::uint32_t hdr_len{0};  // H (kSegmented)
  std::uint32_t mss{0};      // (kSegmented)
};

/// Piece sums of a plan: piece_csum[i] = compute_checksum(bytes of pieces[i]);
/// for a split plan (split4) 2 x pieces.size() entries instead — those of every
/// piece's bytes past its first 4, then those of its first min(4, len) bytes
/// (nicgpu_checksum_batch_split's two outputs).
struct Plan {
  std::vector<PacketPlan> packets;
  std::vector<Piece> pieces;
  bool split4{false};
};

/// One DMA write: dst <- prefix (0 or 4 bytes) || [src_a, +len_a) || [src_b, +len_b).
struct SegmentWrite {
  std::uint64_t dst;
  std::uint64_t src_a;
  std::uint64_t src_b;
  std::uint32_t len_a;
  std::uint32_t len_b;
  std::uint32_t prefix;      // bytes in memory order (little-endian word)
  std::uint32_t prefix_len;  // 0 or 4
};
static_assert(sizeof(SegmentWrite) == 40);

/// True when no RX buffer of `rx` (as far as it lies inside the image) shares a
/// byte with another RX buffer or with a TX buffer of `tx`: then every DMA
/// write of the batch can run in one parallel gather and read its source in
/// place.  O(n + m) for buffers laid out in ascending order, a sort otherwise.
bool buffers_disjoint(std::size_t mem_size, std::span<const TxDescriptor> tx, std::span<const RxDescriptor> rx);

/// split4: kPlainSplit plans for plain packets (Plan::split4), as the device plans them.
Plan make_plan(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               bool split4 = false);
/// The same into `plan`, reusing its storage (no page faults once it has grown).
void make_plan(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               Plan& plan, bool split4 = false);

/// The reference's sequential control flow over the batch, given the plan's
/// piece sums (Plan: piece_csum[i] = compute_checksum(bytes of plan.pieces[i]),
/// split in two halves for a split plan).  Fills
/// out.tx_completions / out.rx_completions (replacing their contents), sets
/// out.tx_processed / rx_consumed, adds to `stats`, fires interrupts in
/// posting order, and lists the DMA writes: writes[j] belongs to RX completion
/// j (zero-length when nothing reached the buffer) and write_of_rx[j] = j, or
/// -1 when nothing was written.
/// Without an interrupt callback it runs on `max_threads` threads (0: as
/// config.host_threads says; a nonzero value also drops the 32 K minimum, for
/// tests): every packet's ring position is predicted by a
/// scan that assumes no RX-side abort before a packet's last segment, chunks
/// resolve in parallel from their predicted positions, and the batch is
/// finished sequentially from the first packet whose pops differ.  The result
/// equals the sequential one.
void resolve(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
             std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
             std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
             std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx, unsigned max_threads = 0,
             const DmaWriteCheck* wcheck = nullptr);

/// The sequential resolve, stopped before the first TX descriptor whose
/// pieces read bytes that an earlier descriptor of this call writes (that
/// descriptor must see the written bytes, so its sums are taken again after the
/// writes) — and, with slots (the offsets of tx[0] / rx[0] in the image),
/// before the first whose own slot or an RX slot it may pop such a write
/// touched.  Same outputs as resolve for the descriptors it covers; returns
/// their number (at least 1 when tx is not empty).
std::size_t resolve_prefix(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
                           std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
                           std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
                           std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx,
                           const DmaWriteCheck* wcheck = nullptr, const RingSlots* slots = nullptr);

/// The device resolve's algorithm (nicgpu_qp_resolve) on the host, for the
/// tests: ring positions by relaxation — every packet resolved at the
/// exclusive scan of the previous step's pops (clamped to the ring's end),
/// starting from rx_need — for at most max_steps steps, then the packets
/// before the first one whose position is not yet exact resolved at their
/// positions.  Returns that count; rx_used is its ring position and steps the
/// steps taken.  Outputs as resolve's for those packets.
std::size_t resolve_relaxed(const BatchedQueuePairConfig& config, std::size_t mem_size, const Plan& plan,
                            std::span<const std::uint16_t> piece_csum, std::span<const TxDescriptor> tx,
                            std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out,
                            std::vector<SegmentWrite>& writes, std::vector<std::int64_t>& write_of_rx, int max_steps,
                            std::size_t& rx_used, int& steps);

/// The interrupt callbacks of a batch (QueuePair::process_once with an
/// InterruptDispatcher, queue_pair.cpp:371-383), fired from its completions in
/// posting order — what resolve's own firing delivers, so every path can
/// resolve without a callback (on the device, in parallel) and fire after.
/// Per TX descriptor, in order: its RX completions (each an RX interrupt when
/// enable_rx_interrupts), then its TX completion's interrupt when
/// enable_tx_interrupts and the reference fires one: a drop before any RX
/// descriptor is popped (no RX completion), or every segment delivered with
/// Success.  The TX completions that fire none (BufferTooSmall, a DMA write
/// fault or a failed RX verify of a segment: queue_pair.cpp:398-399, 442-443)
/// are the ones whose packet ends at a non-Success RX completion, so the RX
/// completions a packet posted are its Success ones up to the first that is
/// not, at most segments_produced of them.
void replay_interrupts(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> tx_completions,
                       std::span<const CompletionEntry> rx_completions);
/// The same over TX completions [at.tx, at.tx + n) only, from RX completion
/// at.rx; `at` is advanced past them (a caller interleaving several queue
/// pairs' completions in the order a scheduler served them).
struct InterruptCursor {
  std::size_t tx{0}, rx{0};
};
void replay_interrupts(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> tx_completions,
                       std::span<const CompletionEntry> rx_completions, InterruptCursor& at, std::size_t n);

/// The same over completions that are still landing, chunk by chunk:
/// wait_chunk(0, c) is called before TX completion c * chunk_tx onwards is
/// first read, wait_chunk(1, c) before RX completion c * chunk_rx onwards
/// (each chunk once, in order) — so the callbacks start on the first chunk
/// while the later ones are still on their way down.
void replay_interrupts_chunked(const BatchedQueuePairConfig& config, std::span<const CompletionEntry> tx_completions,
                               std::span<const CompletionEntry> rx_completions, std::size_t chunk_tx,
                               std::size_t chunk_rx, const std::function<void(int, std::size_t)>& wait_chunk);

/// Order of the DMA writes of one resolved sub-batch for parallel gathers.
/// Writes (RX completions j with write_of_rx[j] >= 0 and at least one byte) are
/// split into layers: a write goes one layer above every earlier write it
/// overlaps, so no two writes of a layer overlap and, of two that do, the later
/// one lands later — the reference's last-write-wins order.
struct WriteSchedule {
  std::vector<std::uint32_t> order;        // RX completion indices, layer by layer, ascending within a layer
  std::vector<std::size_t> layer_begin;    // layer l = order[layer_begin[l], layer_begin[l + 1])
  bool from_copy{false};                   // a destination overlaps a source: gather from a copy of the image
};
void schedule_writes(std::span<const SegmentWrite> writes, std::span<const std::int64_t> write_of_rx,
                     WriteSchedule& schedule);

/// Descriptor arrays that live in the memory image itself (DeviceDescriptors
/// inside it): the image offsets of tx[0] and rx[0], ~0 when an array is not
/// in the image.  The reference pops each ring slot by a DMA read when it
/// reaches it (descriptor_ring.cpp:97-106), after the writes of the packets
/// before; run_batch reproduces that (see DeviceDescriptors).
struct RingSlots {
  std::uint64_t tx_at{~0ull};
  std::uint64_t rx_at{~0ull};
  [[nodiscard]] bool any() const noexcept { return tx_at != ~0ull || rx_at != ~0ull; }
};

/// Device work of run_batch: nicgpu_* launches in BatchedQueuePair; tests run
/// the same driver with a CPU implementation (tests/cpp/cpu_backend.h).
class Backend {
public:
  virtual ~Backend() = default;
  /// The descriptors at image offsets tx_at / rx_at (~0: none) as the image
  /// holds them now, into tx / rx (run_batch with RingSlots).
  virtual void descriptors(std::uint64_t tx_at, std::span<TxDescriptor> tx, std::uint64_t rx_at,
                           std::span<RxDescriptor> rx);
  /// compute_checksum of every piece over the image as it is now; the span
  /// stays valid until the next call.
  virtual std::span<const std::uint16_t> piece_sums(std::span<const Piece> pieces) = 0;
  /// Keep a copy of the image as it is now (the sources of from_copy gathers).
  virtual void snapshot() = 0;
  /// Apply writes whose destinations do not overlap one another; sources are
  /// read from the image, or from the last snapshot when from_copy.
  virtual void gather(std::span<const SegmentWrite> writes, bool from_copy) = 0;
  /// Buffer for n frame descriptors (NICGPU_DESC(address, length)) for rss().
  virtual std::uint64_t* frame_desc(std::size_t n) = 0;
  /// config.rss->select_queue_batch over the n frames of frame_desc(n) in the
  /// image as it is now (stats updated); hash/queue point at n results, valid
  /// until the next call.
  virtual void rss(std::size_t n, const std::uint32_t*& hash, const std::uint16_t*& queue) = 0;
};

/// Host state run_batch reuses across batches.
struct BatchScratch {
  Plan plan;
  std::vector<TxDescriptor> ring_tx;  // run_batch with RingSlots: the descriptors as last read
  std::vector<RxDescriptor> ring_rx;
  std::vector<SegmentWrite> writes, layer;
  std::vector<std::int64_t> write_of_rx;
  std::vector<std::uint32_t> which;
  WriteSchedule schedule;
  RxBatchResult part;
};

/// process_batch's driver over any Backend: plan, piece sums, resolve, DMA
/// writes and RSS, in sub-batches and layers when buffers overlap (see the top
/// of this header).  Adds to `stats`; replaces out's contents.
/// Per-queue dispatch lists (out.queues) of the Success completions, from out.rx_queue.
void build_queue_lists(RxBatchResult& out);

/// disjoint: buffers_disjoint(mem_size, tx, rx) when the caller knows it (-1:
/// computed here).  wcheck: the memory's verdict on each DMA write (the
/// resolve then runs sequentially, on the calling thread).
void run_batch(const BatchedQueuePairConfig& config, std::size_t mem_size, std::span<const TxDescriptor> tx,
               std::span<const RxDescriptor> rx, QueuePairStats& stats, RxBatchResult& out, BatchScratch& scratch,
               Backend& backend, int disjoint = -1, const DmaWriteCheck* wcheck = nullptr,
               const RingSlots* slots = nullptr);

/// host_memory_faults' TX reads: tx with every descriptor whose read
/// m.translate_const(buffer_address, length) refuses moved out of bounds
/// (mem_size + 1: the bounds rule then faults it exactly as the reference's
/// read does).  Returns the window's address (data - address of any read it
/// allows; null when none does).  Throws GpuError (NICGPU_ERR_INVALID) when a
/// read is translated to another address or the allowed reads disagree on
/// the window.
std::byte* checked_reads(const HostMemory& m, std::span<const TxDescriptor> tx, std::vector<TxDescriptor>& out);

}  // namespace rx_stage_detail

}  // namespace nic
