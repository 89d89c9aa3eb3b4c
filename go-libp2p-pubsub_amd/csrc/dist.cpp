// dist.cpp -- RCCL and in-process loopback frontier-exchange transports.
#include "dist.hpp"

#include <cstdlib>

#include "kernels.hpp"

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>

namespace psamd {

// ------------------------------------------------------------------ RCCL ---
namespace {

class RcclTransport final : public Transport {
 public:
  RcclTransport(int rank, int world, ncclComm_t comm) : rank_(rank), world_(world), comm_(comm) {}
  ~RcclTransport() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "rccl"; }
  hipError_t exchange(const uint8_t* send, const std::vector<uint64_t>& send_off,
                      const std::vector<uint64_t>& send_len, uint8_t* recv,
                      const std::vector<uint64_t>& recv_off, const std::vector<uint64_t>& recv_len,
                      hipStream_t s, std::string* err) override {
    ncclResult_t r = ncclGroupStart();
    for (int p = 0; p < world_ && r == ncclSuccess; ++p) {
      if (p == rank_) continue;
      if (send_len[p])
        r = ncclSend(send + send_off[p], send_len[p], ncclUint8, p, comm_, s);
      if (r == ncclSuccess && recv_len[p])
        r = ncclRecv(recv + recv_off[p], recv_len[p], ncclUint8, p, comm_, s);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) {
      if (err) *err = std::string("rccl exchange: ") + ncclGetErrorString(r);
      return hipErrorUnknown;
    }
    return hipSuccess;
  }

 private:
  int rank_, world_;
  ncclComm_t comm_;
};

}  // namespace

int rccl_unique_id(uint8_t id_out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "NCCL unique id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

std::unique_ptr<Transport> make_rccl_transport(int rank, int world, const uint8_t id_bytes[128],
                                               std::string* err) {
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    return nullptr;
  }
  return std::make_unique<RcclTransport>(rank, world, comm);
}

// -------------------------------------------------------------- loopback ---
struct LoopbackGroup {
  int world;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  struct Slot {
    const uint8_t* send = nullptr;
    const std::vector<uint64_t>* send_off = nullptr;
    hipEvent_t sent = nullptr;        // send regions complete (stream order)
    hipEvent_t read[2] = {nullptr, nullptr};  // this rank finished copying from the others:
                                              // exchange k records read[k & 1]
    hipEvent_t used[kSendBufs] = {};  // zero copy: this rank's launches that read the others'
                                      // regions of round r are done (used[r % kSendBufs])
    const Transport::Share* share = nullptr;  // in-place rows: published by share()
  };
  std::vector<Slot> slot;

  explicit LoopbackGroup(int w) : world(w), slot(w) {}

  bool broken = false;

  // false when a rank did not arrive within 60 s (it failed): the group is
  // broken for good and every later exchange fails instead of hanging
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) return false;
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return generation != gen || broken; }) ||
        broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

unsigned stream_event_flags() {
  static const unsigned f = [] {
    const char* v = std::getenv("PSAMD_SYSTEM_EVENTS");
    return (v && std::atoi(v) != 0) ? static_cast<unsigned>(hipEventDisableTiming)
                                     : static_cast<unsigned>(hipEventDisableTiming | hipEventReleaseToDevice);
  }();
  return f;
}

LoopbackGroup* loopback_create(int world) {
  if (world < 1) return nullptr;
  return new LoopbackGroup(world);
}

void loopback_destroy(LoopbackGroup* g) { delete g; }

namespace {

class LoopbackTransport final : public Transport {
 public:
  LoopbackTransport(LoopbackGroup* g, int rank, int device, bool copy, bool in_place)
      : g_(g), rank_(rank), device_(device), copy_(copy), in_place_(in_place) {
    (void)hipSetDevice(device_);
    (void)hipEventCreateWithFlags(&sent_, kStreamEvent);
    for (auto& r : read_) (void)hipEventCreateWithFlags(&r, kStreamEvent);
    for (auto& r : used_) (void)hipEventCreateWithFlags(&r, kStreamEvent);  // (never recorded: no-op waits)
    for (int k = 0; k < 2; ++k) g_->slot[rank_].read[k] = read_[k];
    for (uint32_t k = 0; k < kSendBufs; ++k) g_->slot[rank_].used[k] = used_[k];
  }
  ~LoopbackTransport() override {
    if (sent_) (void)hipEventDestroy(sent_);
    for (auto& r : read_)
      if (r) (void)hipEventDestroy(r);
    for (auto& r : used_)
      if (r) (void)hipEventDestroy(r);
  }
  int rank() const override { return rank_; }
  int world() const override { return g_->world; }
  const char* name() const override { return "loopback"; }

  hipError_t exchange(const uint8_t* send, const std::vector<uint64_t>& send_off,
                      const std::vector<uint64_t>& send_len, uint8_t* recv,
                      const std::vector<uint64_t>& recv_off, const std::vector<uint64_t>& recv_len,
                      hipStream_t s, std::string* err) override {
    // Two host barriers per exchange (every rank runs the same exchanges in
    // the same order).  `sent` is re-recorded only after the next exchange's
    // first barrier, which every rank reaches once it has enqueued its waits
    // on it; the `read` events alternate, so one is re-recorded two exchanges
    // later, after every rank's waits on it.
    (void)send_len;
    const int par = parity_;
    parity_ ^= 1;
    hipEvent_t rd = read_[par];
    hipError_t e = hipEventRecord(sent_, s);
    if (e != hipSuccess) return fail(e, err);
    auto& me = g_->slot[rank_];
    me.send = send;
    me.send_off = &send_off;
    me.sent = sent_;
    if (!g_->barrier()) return timeout(err);  // every rank published regions + `sent`
    CopyRegions c{};
    for (int src = 0; src < g_->world; ++src) {
      if (src == rank_ || recv_len[src] == 0) continue;
      const auto& o = g_->slot[src];
      if ((e = hipStreamWaitEvent(s, o.sent, 0)) != hipSuccess) return fail(e, err);
      const uint8_t* from = o.send + (*o.send_off)[rank_];
      uint8_t* to = recv + recv_off[src];
      if (c.n < kMaxCopyRegions && recv_len[src] % 16 == 0 && reinterpret_cast<uintptr_t>(from) % 16 == 0 &&
          reinterpret_cast<uintptr_t>(to) % 16 == 0) {  // (ghost records: whole 16-B units)
        c.src[c.n] = reinterpret_cast<const uint4*>(from);
        c.dst[c.n] = reinterpret_cast<uint4*>(to);
        c.units[c.n++] = recv_len[src] / 16;
      } else if ((e = hipMemcpyAsync(to, from, recv_len[src], hipMemcpyDeviceToDevice, s)) != hipSuccess) {
        return fail(e, err);
      }
    }
    if ((e = launch_copy_regions(c, s)) != hipSuccess) return fail(e, err);
    if ((e = hipEventRecord(rd, s)) != hipSuccess) return fail(e, err);
    if (!g_->barrier()) return timeout(err);  // every rank enqueued copies + `read`
    // our send regions may be rewritten only after every reader copied them
    for (int q = 0; q < g_->world; ++q) {
      if (q == rank_) continue;
      if ((e = hipStreamWaitEvent(s, g_->slot[q].read[par], 0)) != hipSuccess) return fail(e, err);
    }
    return hipSuccess;
  }

  // Zero copy (level mode): the ranks share one process and one device, so a
  // receiving launch reads the sender's region where it lies -- no copy
  // launch, no receive buffer.  Two barriers as in exchange(): `sent` is
  // re-recorded only after every rank has enqueued its waits on it.  With
  // PS_DIST_F_COPY (copy_) level mode takes exchange() instead, the RCCL
  // transport's data path: the records land in the receive buffer.
  bool zero_copy() const override { return !copy_; }
  bool in_place() const override { return in_place_; }
  hipError_t share(const Share& mine, std::vector<Share>& all, std::string* err) override {
    g_->slot[rank_].share = &mine;
    if (!g_->barrier()) return timeout(err);  // every rank published
    all.assign(g_->world, Share{});
    for (int q = 0; q < g_->world; ++q) all[q] = *g_->slot[q].share;
    if (!g_->barrier()) return timeout(err);  // every rank copied (`mine` may go)
    return hipSuccess;
  }
  hipError_t exchange_zc(const uint8_t* send, const std::vector<uint64_t>& send_off,
                         std::vector<const uint8_t*>& peer, hipStream_t s, std::string* err) override {
    hipError_t e = hipEventRecord(sent_, s);
    if (e != hipSuccess) return fail(e, err);
    auto& me = g_->slot[rank_];
    me.send = send;
    me.send_off = &send_off;
    me.sent = sent_;
    if (!g_->barrier()) return timeout(err);  // every rank published regions + `sent`
    peer.assign(g_->world, nullptr);
    for (int src = 0; src < g_->world; ++src) {
      if (src == rank_) continue;
      const auto& o = g_->slot[src];
      if ((e = hipStreamWaitEvent(s, o.sent, 0)) != hipSuccess) return fail(e, err);
      peer[src] = o.send + (*o.send_off)[rank_];
    }
    if (!g_->barrier()) return timeout(err);  // every rank enqueued its waits on `sent`
    return hipSuccess;
  }
  // After the launches that read the others' regions of round r: used[r %
  // kSendBufs] marks them done.  The writers wait for it in reuse(r), before
  // their launches of round r + kSendBufs - 1 rewrite those regions -- one
  // round later than a wait here, so a round's readers and the next round's
  // writers overlap.  An event is re-recorded kSendBufs rounds later, after
  // that round's exchange barrier, which every rank reaches only once it has
  // enqueued its reuse wait on it.
  hipError_t consumed(hipStream_t s, uint32_t round, std::string* err) override {
    hipError_t e = hipEventRecord(used_[round % kSendBufs], s);
    if (e != hipSuccess) return fail(e, err);
    if (!g_->barrier()) return timeout(err);  // every rank recorded its `used`
    return hipSuccess;
  }
  hipError_t reuse(hipStream_t s, uint32_t round, std::string* err) override {
    for (int q = 0; q < g_->world; ++q) {
      if (q == rank_) continue;
      const hipError_t e = hipStreamWaitEvent(s, g_->slot[q].used[round % kSendBufs], 0);
      if (e != hipSuccess) return fail(e, err);
    }
    return hipSuccess;
  }

 private:
  static hipError_t timeout(std::string* err) {
    if (err) *err = "loopback exchange: a rank did not arrive (group broken)";
    return hipErrorUnknown;
  }
  static hipError_t fail(hipError_t e, std::string* err) {
    if (err) *err = std::string("loopback exchange: ") + hipGetErrorString(e);
    return e;
  }
  LoopbackGroup* g_;
  int rank_, device_;
  bool copy_, in_place_;
  hipEvent_t sent_ = nullptr, read_[2] = {nullptr, nullptr}, used_[kSendBufs] = {};
  int parity_ = 0;
};

}  // namespace

std::unique_ptr<Transport> make_loopback_transport(LoopbackGroup* g, int rank, int device, bool copy,
                                                  bool in_place) {
  if (!g || rank < 0 || rank >= g->world) return nullptr;
  return std::make_unique<LoopbackTransport>(g, rank, device, copy, in_place);
}

}  // namespace psamd
