// dist.cpp -- RCCL, in-process loopback and process-shared IPC frontier-exchange
// transports.
#include "dist.hpp"

#include <cstdlib>

#include "kernels.hpp"

#include <rccl/rccl.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdarg>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>

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

// ------------------------------------------------------------------- IPC ---
namespace {
std::atomic<uint64_t> g_free_epoch{0};
}  // namespace

void note_device_free() { g_free_epoch.fetch_add(1, std::memory_order_relaxed); }
uint64_t device_free_epoch() { return g_free_epoch.load(std::memory_order_relaxed); }

int ipc_group_id(uint8_t id_out[128]) {
  std::memset(id_out, 0, 128);
  std::random_device rd;
  const uint64_t salt = (static_cast<uint64_t>(rd()) << 32) ^ rd() ^
                        static_cast<uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
  std::snprintf(reinterpret_cast<char*>(id_out), 128, "/psamd-ipc-%d-%016llx", static_cast<int>(getpid()),
                static_cast<unsigned long long>(salt));
  return 0;
}

namespace {

constexpr uint64_t kIpcMagic = 0x70736970632d3036ull;
// device flag words (u64 index into a rank's flag block, one 128-B line each)
constexpr uint32_t kFlagSent = 0, kFlagRead = 16, kFlagUsed = 32, kFlagWords = 48;
constexpr uint64_t kFlagTimeoutTicks = 30ull * 100000000ull;  // 30 s of the 100 MHz clock
constexpr int kBarrierSeconds = 120;
enum IpcKind { kSend = 0, kSeen = 1, kGen = 2, kKinds = 3 };

struct IpcExport {  // where a device pointer lies: one allocation, exported once
  uint64_t ver = 0;
  hipIpcMemHandle_t h{};
  uint64_t off = 0;  // pointer - allocation base
};

struct alignas(64) IpcPub {  // one exchange's send regions (double-buffered by sequence)
  uint64_t seq;
  IpcExport send;
  uint64_t off[kMaxRanks];
};

struct alignas(64) IpcSlot {
  int32_t pid;
  int32_t world;
  uint32_t topic_words;
  uint32_t pad;
  hipIpcMemHandle_t flags;
  IpcPub pub[2];
  IpcExport seen, gen;  // share()
  uint32_t gen_cur;
  uint32_t n_words;
};

struct IpcShm {
  std::atomic<uint64_t> magic;
  alignas(64) std::atomic<uint32_t> arrived;
  alignas(64) std::atomic<uint32_t> generation;
  std::atomic<uint32_t> broken;
  IpcSlot slot[kMaxRanks];
  // followed by world x topic_words u64: share()'s per-topic layouts
};

class IpcTransport final : public Transport {
 public:
  IpcTransport(int rank, int world, int device, bool copy, bool in_place)
      : rank_(rank), world_(world), device_(device), copy_(copy), in_place_(in_place) {
    const char* t = std::getenv("PSAMD_IPC_TRACE");  // (debug: every call and barrier on stderr)
    trace_ = t && std::atoi(t) != 0;
    const char* b = std::getenv("PSAMD_IPC_BARRIER_S");
    barrier_s_ = b && std::atoi(b) > 0 ? std::atoi(b) : kBarrierSeconds;
  }

  ~IpcTransport() override {
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();  // (no launch may still read a mapping closed below)
    for (void* p : opened_)
      if (p) (void)hipIpcCloseMemHandle(p);
    if (flags_) (void)hipFree(flags_);
    if (err_) (void)hipHostFree(err_);
    if (shm_) munmap(shm_, shm_bytes_);
  }

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "ipc"; }
  bool zero_copy() const override { return !copy_; }
  bool in_place() const override { return in_place_; }

  // Opens (or creates) the group's segment, exports this rank's flag block and
  // maps every other rank's; all ranks arrive, then rank 0 unlinks the name.
  // A rank that fails unlinks it too (the other ranks' barrier times out), so
  // no segment outlives a failed group in /dev/shm.
  bool open(const char* name, uint32_t n_topics, std::string* err) {
    const bool ok = open_group(name, n_topics, err);
    if (!ok) shm_unlink(name);
    return ok;
  }

 private:
  bool open_group(const char* name, uint32_t n_topics, std::string* err) {
    topic_words_ = 4 * n_topics;
    shm_bytes_ = sizeof(IpcShm) + static_cast<size_t>(world_) * topic_words_ * 8;
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return fail_host(std::string("shm_open ") + name + ": " + std::strerror(errno), err);
    if (ftruncate(fd, static_cast<off_t>(shm_bytes_)) != 0) {
      close(fd);
      return fail_host(std::string("ftruncate: ") + std::strerror(errno), err);
    }
    void* m = mmap(nullptr, shm_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return fail_host(std::string("mmap: ") + std::strerror(errno), err);
    shm_ = static_cast<IpcShm*>(m);
    uint64_t zero = 0;
    if (!shm_->magic.compare_exchange_strong(zero, kIpcMagic) && zero != kIpcMagic)
      return fail_host("shared segment is not an ipc group", err);
    hipError_t e;
    if ((e = hipSetDevice(device_)) != hipSuccess) return fail(e, err);
    if ((e = hipMalloc(&flags_, kFlagWords * 8)) != hipSuccess) return fail(e, err);
    if ((e = hipMemset(flags_, 0, kFlagWords * 8)) != hipSuccess) return fail(e, err);
    if ((e = hipHostMalloc(&err_, 64)) != hipSuccess) return fail(e, err);
    *err_ = 0;
    IpcSlot& me = shm_->slot[rank_];
    me.pid = static_cast<int32_t>(getpid());
    me.world = world_;
    me.topic_words = topic_words_;
    if ((e = hipIpcGetMemHandle(&me.flags, flags_)) != hipSuccess) return fail(e, err);
    if (!barrier("open")) return timeout(err);
    for (int q = 0; q < world_; ++q) {
      const IpcSlot& o = shm_->slot[q];
      if (o.world != world_ || o.topic_words != topic_words_)
        return fail_host("ranks disagree on world size or topic count", err);
      if (q == rank_) {
        peer_flags_[q] = flags_;
        continue;
      }
      void* p = nullptr;
      if ((e = hipIpcOpenMemHandle(&p, o.flags, hipIpcMemLazyEnablePeerAccess)) != hipSuccess) {
        if (err) *err = std::string("ipc transport: hipIpcOpenMemHandle of rank ") + std::to_string(q) +
                        "'s flags: " + hipGetErrorString(e);
        return false;
      }
      opened_.push_back(p);
      peer_flags_[q] = static_cast<uint64_t*>(p);
    }
    if (!barrier("mapped")) return timeout(err);  // every rank mapped every flag block
    if (rank_ == 0) shm_unlink(name);
    return true;
  }

 public:
  hipError_t exchange(const uint8_t* send, const std::vector<uint64_t>& send_off,
                      const std::vector<uint64_t>& send_len, uint8_t* recv,
                      const std::vector<uint64_t>& recv_off, const std::vector<uint64_t>& recv_len,
                      hipStream_t s, std::string* err) override {
    (void)send_len;
    hipError_t e;
    const uint64_t seq = ++seq_;
    if ((e = publish(send, send_off, seq, s, err)) != hipSuccess) return e;
    FlagWait w{};
    CopyRegions c{};
    for (int src = 0; src < world_; ++src) {
      if (src == rank_ || recv_len[src] == 0) continue;
      const uint8_t* from = nullptr;
      if ((e = region(src, seq, &from, err)) != hipSuccess) return e;
      w.flag[src] = peer_flags_[src] + kFlagSent;
      w.value[src] = seq;
      uint8_t* to = recv + recv_off[src];
      if (c.n < kMaxCopyRegions && recv_len[src] % 16 == 0 && reinterpret_cast<uintptr_t>(from) % 16 == 0 &&
          reinterpret_cast<uintptr_t>(to) % 16 == 0) {
        c.src[c.n] = reinterpret_cast<const uint4*>(from);
        c.dst[c.n] = reinterpret_cast<uint4*>(to);
        c.units[c.n++] = recv_len[src] / 16;
      } else {
        pending_.push_back({from, to, recv_len[src]});
      }
    }
    if ((e = launch_flag_wait(w, err_, kFlagTimeoutTicks, s)) != hipSuccess) return fail(e, err);
    for (const auto& p : pending_)
      if ((e = hipMemcpyAsync(p.to, p.from, p.n, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(e, err);
    pending_.clear();
    if ((e = launch_copy_regions(c, s)) != hipSuccess) return fail(e, err);
    // our send regions may be rewritten only after every reader copied them
    if ((e = launch_flag_set(flags_ + kFlagRead, seq, s)) != hipSuccess) return fail(e, err);
    return wait_all(kFlagRead, seq, s, err);
  }

  hipError_t exchange_zc(const uint8_t* send, const std::vector<uint64_t>& send_off,
                         std::vector<const uint8_t*>& peer, hipStream_t s, std::string* err) override {
    hipError_t e;
    const uint64_t seq = ++seq_;
    if ((e = publish(send, send_off, seq, s, err)) != hipSuccess) return e;
    peer.assign(world_, nullptr);
    for (int src = 0; src < world_; ++src) {
      if (src == rank_) continue;
      const uint8_t* from = nullptr;
      if ((e = region(src, seq, &from, err)) != hipSuccess) return e;
      peer[src] = from;
    }
    return wait_all(kFlagSent, seq, s, err);
  }

  // consumed(r): the launches that read round r's regions are enqueued; the
  // writers' reuse(r) waits for this rank's count of such points to reach the
  // same number (every rank makes the same calls in the same order)
  hipError_t consumed(hipStream_t s, uint32_t round, std::string* err) override {
    const uint64_t n = ++used_;
    used_at_[round % kSendBufs] = n;
    if (trace_) log("consumed round %u -> used %llu", round, static_cast<unsigned long long>(n));
    const hipError_t e = launch_flag_set(flags_ + kFlagUsed, n, s);
    return e == hipSuccess ? hipSuccess : fail(e, err);
  }
  hipError_t reuse(hipStream_t s, uint32_t round, std::string* err) override {
    if (const hipError_t e = check(err)) return e;
    if (trace_) log("reuse round %u waits used %llu", round, static_cast<unsigned long long>(used_at_[round % kSendBufs]));
    return wait_all(kFlagUsed, used_at_[round % kSendBufs], s, err);
  }

  hipError_t share(const Share& mine, std::vector<Share>& all, std::string* err) override {
    if (mine.topics.size() > topic_words_) {
      fail_host("share: more topic words than the group holds", err);
      return hipErrorInvalidValue;
    }
    IpcSlot& me = shm_->slot[rank_];
    hipError_t e;
    if ((e = export_ptr(kSeen, mine.seen, &me.seen)) != hipSuccess) return fail(e, err);
    if ((e = export_ptr(kGen, mine.gen, &me.gen)) != hipSuccess) return fail(e, err);
    me.gen_cur = mine.gen_cur;
    me.n_words = static_cast<uint32_t>(mine.topics.size());
    std::memcpy(topic_block(rank_), mine.topics.data(), mine.topics.size() * 8);
    if (!barrier("share")) return timeout(err);  // every rank published
    all.assign(world_, Share{});
    static const bool serial = [] {
      const char* v = std::getenv("PSAMD_IPC_SERIAL_OPEN");
      return v && std::atoi(v) != 0;
    }();
    for (int turn = 0; serial && turn < rank_; ++turn)
      if (!barrier("turn", turn)) return timeout(err);
    for (int q = 0; q < world_; ++q) {
      const IpcSlot& o = shm_->slot[q];
      Share& a = all[q];
      a.gen_cur = o.gen_cur;
      a.topics.assign(topic_block(q), topic_block(q) + o.n_words);
      if (q == rank_) {
        a.seen = mine.seen;
        a.gen = mine.gen;
        continue;
      }
      const uint8_t* b = nullptr;
      if ((e = import(q, kSeen, o.seen, &b, err)) != hipSuccess) return e;
      a.seen = b;
      if ((e = import(q, kGen, o.gen, &b, err)) != hipSuccess) return e;
      a.gen = b;
    }
    for (int turn = rank_; serial && turn < world_; ++turn)
      if (!barrier("turn", turn)) return timeout(err);
    if (!barrier("shared")) return timeout(err);  // every rank copied the slots (they may change)
    return hipSuccess;
  }

 private:
  struct Import {
    uint64_t ver = 0;
    uint8_t* base = nullptr;
  };
  struct Pending {
    const uint8_t* from;
    uint8_t* to;
    uint64_t n;
  };

  uint64_t* topic_block(int q) {
    return reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(shm_) + sizeof(IpcShm)) +
           static_cast<size_t>(q) * topic_words_;
  }

  // a rank's pointer as (allocation export, offset); re-exported only when the
  // pointer leaves the cached range or any device range was freed since
  hipError_t export_ptr(int kind, const void* p, IpcExport* out) {
    Cache& c = cache_[kind];
    const auto* u = static_cast<const uint8_t*>(p);
    if (!(c.base && u >= c.base && u < c.base + c.size && c.epoch == device_free_epoch())) {
      void* base = nullptr;
      size_t size = 0;
      hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(p));
      if (e != hipSuccess) return e;
      hipIpcMemHandle_t h;
      if ((e = hipIpcGetMemHandle(&h, base)) != hipSuccess) return e;
      c.base = static_cast<const uint8_t*>(base);
      c.size = size;
      c.epoch = device_free_epoch();
      c.ex.h = h;
      c.ex.ver = ++exports_;
      if (trace_) log("export kind %d base %p size %zu ver %llu", kind, base, size, static_cast<unsigned long long>(c.ex.ver));
    }
    *out = c.ex;
    out->off = static_cast<uint64_t>(u - c.base);
    return hipSuccess;
  }

  hipError_t import(int q, int kind, const IpcExport& ex, const uint8_t** out, std::string* err) {
    Import& im = imports_[q][kind];
    if (im.ver != ex.ver) {
      void* p = nullptr;
      if (trace_) log("open rank %d kind %d ver %llu", q, kind, static_cast<unsigned long long>(ex.ver));
      std::atomic<bool> done{false};
      std::thread dog;
      if (trace_)  // (debug: where every thread of this process waits, if the open stalls)
        dog = std::thread([&] {
          for (int i = 0; i < 800 && !done.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
          if (done.load()) return;
          for (int round = 0; round < 3 && !done.load(); ++round) {
            DIR* d = opendir("/proc/self/task");
            for (dirent* de = d ? readdir(d) : nullptr; de; de = readdir(d)) {
              if (de->d_name[0] == '.') continue;
              auto slurp = [&](const char* f) {
                std::string path = std::string("/proc/self/task/") + de->d_name + "/" + f, out;
                if (FILE* fp = std::fopen(path.c_str(), "r")) {
                  char b[256];
                  const size_t k = std::fread(b, 1, sizeof b - 1, fp);
                  b[k] = 0;
                  std::fclose(fp);
                  out = b;
                  while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
                }
                return out;
              };
              log("stall: task %s %s wchan=%s syscall=%s", de->d_name, slurp("comm").c_str(), slurp("wchan").c_str(),
                  slurp("syscall").substr(0, 24).c_str());
            }
            if (d) closedir(d);
            std::this_thread::sleep_for(std::chrono::seconds(4));
          }
        });
      const hipError_t e = hipIpcOpenMemHandle(&p, ex.h, hipIpcMemLazyEnablePeerAccess);
      done.store(true);
      if (dog.joinable()) dog.join();
      if (trace_) log("opened rank %d kind %d -> %p (%s)", q, kind, p, hipGetErrorString(e));
      if (e != hipSuccess) {
        if (err) *err = std::string("ipc transport: hipIpcOpenMemHandle of rank ") + std::to_string(q) + ": " +
                        hipGetErrorString(e);
        return e;
      }
      opened_.push_back(p);  // (an older mapping may still be read by enqueued launches: closed at the end)
      im.ver = ex.ver;
      im.base = static_cast<uint8_t*>(p);
    }
    *out = im.base + ex.off;
    return hipSuccess;
  }

  // this exchange's regions into the slot, the `sent` flag behind the
  // launches that wrote them, then the host barrier (every rank published)
  hipError_t publish(const uint8_t* send, const std::vector<uint64_t>& send_off, uint64_t seq, hipStream_t s,
                     std::string* err) {
    if (const hipError_t e = check(err)) return e;
    IpcPub& pub = shm_->slot[rank_].pub[seq & 1];
    hipError_t e;
    if ((e = export_ptr(kSend, send, &pub.send)) != hipSuccess) return fail(e, err);
    for (int q = 0; q < kMaxRanks; ++q) pub.off[q] = q < static_cast<int>(send_off.size()) ? send_off[q] : 0;
    pub.seq = seq;
    if ((e = launch_flag_set(flags_ + kFlagSent, seq, s)) != hipSuccess) return fail(e, err);
    if (!barrier("exchange", seq)) return timeout(err);
    return hipSuccess;
  }

  // src's region for this rank in exchange `seq` (its slot's half seq & 1 is
  // rewritten only after the next exchange's barrier, which this rank has not
  // reached yet)
  hipError_t region(int src, uint64_t seq, const uint8_t** from, std::string* err) {
    const IpcPub& pub = shm_->slot[src].pub[seq & 1];
    if (pub.seq != seq) {
      if (err) *err = "ipc transport: rank " + std::to_string(src) + " published exchange " + std::to_string(pub.seq) +
                      ", this rank expected " + std::to_string(seq) + " (the ranks' plans differ)";
      return hipErrorInvalidValue;
    }
    const uint8_t* base = nullptr;
    if (const hipError_t e = import(src, kSend, pub.send, &base, err)) return e;
    *from = base + pub.off[rank_];
    return hipSuccess;
  }

  hipError_t wait_all(uint32_t word, uint64_t value, hipStream_t s, std::string* err) {
    FlagWait w{};
    for (int q = 0; q < world_; ++q)
      if (q != rank_) {
        w.flag[q] = peer_flags_[q] + word;
        w.value[q] = value;
      }
    const hipError_t e = launch_flag_wait(w, err_, kFlagTimeoutTicks, s);
    return e == hipSuccess ? hipSuccess : fail(e, err);
  }

  // a flag wait that timed out (a peer died or its plan diverged) fails the
  // next call: the windows enqueued since may have read stale rows
  hipError_t check(std::string* err) {
    if (__atomic_load_n(err_, __ATOMIC_ACQUIRE) == 0) return hipSuccess;
    if (err) *err = "ipc transport: a peer's device flag did not arrive within 30 s (rank died or plans diverged)";
    return hipErrorLaunchTimeOut;
  }

  void log(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "[ipc %d/%d %.6f] %s\n", rank_, world_, t, buf);
  }

  bool barrier(const char* what, uint64_t seq = 0) {
    if (trace_) log("barrier %s %llu", what, static_cast<unsigned long long>(seq));
    const uint32_t gen = shm_->generation.load(std::memory_order_acquire);
    if (shm_->broken.load(std::memory_order_acquire)) return false;
    if (shm_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == static_cast<uint32_t>(world_)) {
      shm_->arrived.store(0, std::memory_order_relaxed);
      shm_->generation.store(gen + 1, std::memory_order_release);
      return true;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      if (shm_->generation.load(std::memory_order_acquire) != gen) return true;
      if (shm_->broken.load(std::memory_order_acquire)) return false;
      if (spin < 4096) {
        std::this_thread::yield();
        continue;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(barrier_s_)) {
        log("barrier %s %llu: timed out after %d s", what, static_cast<unsigned long long>(seq), barrier_s_);
        shm_->broken.store(1, std::memory_order_release);
        return false;
      }
    }
  }

  static hipError_t timeout(std::string* err) {
    if (err) *err = "ipc transport: a rank did not arrive in time (group broken)";
    return hipErrorUnknown;
  }
  static hipError_t fail(hipError_t e, std::string* err) {
    if (err) *err = std::string("ipc transport: ") + hipGetErrorString(e);
    return e;
  }
  static bool fail_host(const std::string& what, std::string* err) {
    if (err) *err = "ipc transport: " + what;
    return false;
  }

  struct Cache {
    const uint8_t* base = nullptr;
    size_t size = 0;
    uint64_t epoch = 0;
    IpcExport ex;
  };
  int rank_, world_, device_;
  bool copy_, in_place_;
  IpcShm* shm_ = nullptr;
  size_t shm_bytes_ = 0;
  uint32_t topic_words_ = 0;
  uint64_t* flags_ = nullptr;
  uint32_t* err_ = nullptr;
  uint64_t* peer_flags_[kMaxRanks] = {};
  uint64_t seq_ = 0, used_ = 0, used_at_[kSendBufs] = {};
  uint64_t exports_ = 0;
  Cache cache_[kKinds];
  Import imports_[kMaxRanks][kKinds];
  std::vector<void*> opened_;
  std::vector<Pending> pending_;
  bool trace_ = false;
  int barrier_s_ = kBarrierSeconds;
};

}  // namespace

std::unique_ptr<Transport> make_ipc_transport(int rank, int world, int device, const uint8_t id[128],
                                             uint32_t n_topics, bool copy, bool in_place, std::string* err) {
  char name[129];
  std::memcpy(name, id, 128);
  name[128] = 0;
  if (name[0] != '/' || std::strchr(name + 1, '/')) {
    if (err) *err = "ipc transport: group id is not a shared-memory name (ps_dist_ipc_id)";
    return nullptr;
  }
  auto t = std::make_unique<IpcTransport>(rank, world, device, copy, in_place);
  if (!t->open(name, n_topics, err)) return nullptr;
  return t;
}

}  // namespace psamd
