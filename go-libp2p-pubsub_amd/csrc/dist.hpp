// dist.hpp -- frontier-exchange transports of the multi-GPU engine.
//
// One engine per GPU (rank).  Each synchronous round the ranks exchange the
// deliveries addressed to tree nodes owned by another rank: every rank sends
// rank d one region of fixed, host-known size (header + capacity items), so
// the exchange is stream-ordered and needs no host synchronisation.
//   RcclTransport      ncclSend / ncclRecv pairs in one group (all-to-allv over
//                      xGMI), the production transport.
//   LoopbackTransport  `world` engines of one process (threads) copy each
//                      other's regions device-to-device (compaction mode;
//                      level mode with PS_DIST_F_COPY) or, in level mode, read
//                      them in place (zero-copy); lets the real kernels and
//                      routing be tested on a single GPU.
//   IpcTransport       one process per rank (several may share a GPU): the
//                      loopback's three data paths over IPC-mapped device
//                      memory, ordered by device flags instead of events.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace psamd {
// Level mode's send buffer: one part per round, cycling (round r ships into
// part r % kSendBufs), so that a round's readers and the writers of the
// round after it need not wait for each other (zero copy: reuse()).
constexpr uint32_t kSendBufs = 3;
// Events that only order streams of this device (cross-stream waits, the
// prefix/gate/reduce hand-offs, the loopback exchange): a device-scope
// release.  The default system-scope fence writes back and invalidates the
// caches at every record -- ~10 us on the recording queue after a launch that
// wrote rows (cfg2: the gap between a window's chain and the next window).
// (A/B: PSAMD_SYSTEM_EVENTS=1 restores the system-scope default)
unsigned stream_event_flags();
#define kStreamEvent (::psamd::stream_event_flags())
// A window's start mark: timing only (its end event keeps the system fence:
// the host reads the window's counters from pinned memory after it).
constexpr unsigned kStartEvent = hipEventReleaseToDevice;
}  // namespace psamd

namespace psamd {

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // All-to-allv of device byte ranges on stream s: region d of `send` goes to
  // rank d, region s of `recv` comes from rank s (sizes agree pairwise).
  virtual hipError_t exchange(const uint8_t* send, const std::vector<uint64_t>& send_off,
                              const std::vector<uint64_t>& send_len, uint8_t* recv,
                              const std::vector<uint64_t>& recv_off,
                              const std::vector<uint64_t>& recv_len, hipStream_t s,
                              std::string* err) = 0;
  virtual const char* name() const = 0;
  // Zero-copy exchange (level mode; only transports whose ranks share one
  // address space): publish this round's send regions and get, per source
  // rank a, the address of a's region for this rank (peer[a]); the caller's
  // launches read the records there, then call consumed(round) on the same
  // stream once they are enqueued; before a's launches rewrite that region
  // (kSendBufs rounds later) a calls reuse(round), which orders its stream
  // after every reader's consumed(round) point.
  virtual bool zero_copy() const { return false; }
  virtual hipError_t exchange_zc(const uint8_t* send, const std::vector<uint64_t>& send_off,
                                 std::vector<const uint8_t*>& peer, hipStream_t s, std::string* err) {
    (void)send, (void)send_off, (void)peer, (void)s;
    if (err) *err = "zero-copy exchange not supported by this transport";
    return hipErrorNotSupported;
  }
  virtual hipError_t consumed(hipStream_t s, uint32_t round, std::string* err) {
    (void)s, (void)round;
    if (err) *err = "zero-copy exchange not supported by this transport";
    return hipErrorNotSupported;
  }
  virtual hipError_t reuse(hipStream_t s, uint32_t round, std::string* err) {
    (void)s, (void)round;
    if (err) *err = "zero-copy exchange not supported by this transport";
    return hipErrorNotSupported;
  }
  // In-place rows (PS_DIST_F_INPLACE; ranks sharing one address space): a
  // receiver reads a ghost parent's row where its owner wrote it.  share()
  // swaps every rank's row-set addresses and per-topic layout (host data,
  // all ranks call it together, at each change of the ghost plan).
  struct Share {
    const void* seen = nullptr;
    const void* gen = nullptr;
    uint32_t gen_cur = 0;
    std::vector<uint64_t> topics;  // per topic: wbase, n_nodes, nbase, flags
  };
  virtual bool in_place() const { return false; }
  virtual hipError_t share(const Share& mine, std::vector<Share>& all, std::string* err) {
    (void)mine, (void)all;
    if (err) *err = "in-place rows not supported by this transport";
    return hipErrorNotSupported;
  }
};

std::unique_ptr<Transport> make_rccl_transport(int rank, int world, const uint8_t id[128],
                                               std::string* err);
int rccl_unique_id(uint8_t id_out[128]);

// Process-shared transport: one process per rank on one node (several may
// share a GPU).  Host-side rendezvous in a POSIX shared-memory segment named
// by `id` (ipc_group_id on one rank, shipped by the caller like the RCCL id);
// device buffers mapped across processes with hipIpcGetMemHandle /
// hipIpcOpenMemHandle; stream order between ranks by monotonic device flags
// (launch_flag_set / launch_flag_wait) in IPC-mapped memory.  Modes as the
// loopback's: copy (exchange into the receive buffer), zero copy (read the
// sender's region in place), in-place rows.
int ipc_group_id(uint8_t id_out[128]);
std::unique_ptr<Transport> make_ipc_transport(int rank, int world, int device, const uint8_t id[128],
                                             uint32_t n_topics, bool copy, bool in_place, std::string* err);
// Every device free bumps this epoch: an IPC export of an address range is
// reused only while no range was freed since (a freed range's address may
// come back as another allocation).
void note_device_free();
uint64_t device_free_epoch();

struct LoopbackGroup;
LoopbackGroup* loopback_create(int world);
void loopback_destroy(LoopbackGroup* g);
// copy: level mode copies the records into the receive buffer (the RCCL data
// path) instead of reading them in place (zero copy)
std::unique_ptr<Transport> make_loopback_transport(LoopbackGroup* g, int rank, int device, bool copy,
                                                  bool in_place = false);

}  // namespace psamd
