// ipc_probe -- can processes sharing one GPU map each other's allocations
// (hipIpcGetMemHandle / hipIpcOpenMemHandle), and what does a stream-ordered
// device-flag handshake between them cost?
//
//   ipc_probe [procs=2] [iters=2000]
//
// The parent forks `procs` children before any HIP call (it never touches the
// GPU) and hands them a shared-memory mailbox.  Child r allocates a row
// buffer and a flag word, fills the buffer with r-tagged words, publishes both
// IPC handles, opens every other child's, checks the rows it reads through the
// mapping, then runs `iters` rounds of: set own flag = i; wait every other
// flag >= i (all on one stream: a one-wave set kernel and a one-wave poll
// kernel with a 5 s timeout).  Prints per-round latency.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "rank %d: %s -> %s\n", rank, #x, hipGetErrorString(e_)); \
      std::_Exit(2);                                                                  \
    }                                                                                 \
  } while (0)

constexpr int kMax = 16;
constexpr size_t kWords = 1 << 20;

struct Mail {
  std::atomic<int> arrived;
  std::atomic<int> gen;
  hipIpcMemHandle_t rows[kMax];
  hipIpcMemHandle_t flag[kMax];
};

static void barrier(Mail* m, int n) {
  const int g = m->gen.load();
  if (m->arrived.fetch_add(1) + 1 == n) {
    m->arrived.store(0);
    m->gen.fetch_add(1);
  } else {
    while (m->gen.load() == g) std::this_thread::yield();
  }
}

__global__ void k_fill(uint64_t* p, size_t n, uint64_t tag) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = tag << 32 | i;
}
__global__ void k_check(const uint64_t* p, size_t n, uint64_t tag, unsigned* bad) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (p[i] != (tag << 32 | i)) atomicAdd(bad, 1u);
}
__global__ void k_set(uint64_t* f, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
struct Flags {
  const uint64_t* f[kMax];
};
__global__ void k_wait(Flags fl, int n, int me, uint64_t v, unsigned* timeout) {
  const int q = threadIdx.x;
  if (q >= n || q == me) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(fl.f[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    if (wall_clock64() - t0 > 500000000ull) {  // 5 s at 100 MHz
      atomicAdd(timeout, 1u);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

static int child(Mail* m, int rank, int n, int iters) {
  CK(hipSetDevice(0));
  uint64_t *rows, *flag;
  unsigned* cnt;
  CK(hipMalloc(&rows, kWords * 8));
  CK(hipMalloc(&flag, 256));
  CK(hipMemset(flag, 0, 256));
  CK(hipHostMalloc(&cnt, 8));
  cnt[0] = cnt[1] = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  k_fill<<<1024, 256, 0, s>>>(rows, kWords, rank + 1);
  CK(hipStreamSynchronize(s));
  CK(hipIpcGetMemHandle(&m->rows[rank], rows));
  {  // is the handle of one allocation stable?  what does an export cost?
    hipIpcMemHandle_t h2;
    auto a0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100; ++i) CK(hipIpcGetMemHandle(&h2, rows));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a0).count();
    void* base = nullptr;
    size_t sz = 0;
    CK(hipMemGetAddressRange(&base, &sz, rows + 12345));
    std::printf("rank %d: handle stable %d, %.2f us/export, interior base ok %d size %zu\n", rank,
                std::memcmp(&h2, &m->rows[rank], sizeof(h2)) == 0, us / 100, base == rows, sz);
  }
  CK(hipIpcGetMemHandle(&m->flag[rank], flag));
  barrier(m, n);
  Flags fl{};
  const uint64_t* peer_rows[kMax] = {};
  for (int q = 0; q < n; ++q) {
    if (q == rank) {
      fl.f[q] = flag;
      continue;
    }
    void *pr, *pf;
    CK(hipIpcOpenMemHandle(&pr, m->rows[q], hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle(&pf, m->flag[q], hipIpcMemLazyEnablePeerAccess));
    k_check<<<1024, 256, 0, s>>>(static_cast<uint64_t*>(pr), kWords, q + 1, cnt);
    fl.f[q] = static_cast<uint64_t*>(pf);
    peer_rows[q] = static_cast<uint64_t*>(pr);
  }
  CK(hipStreamSynchronize(s));
  std::printf("rank %d: opened %d peers' rows, %u bad words\n", rank, n - 1, cnt[0]);
  barrier(m, n);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 1; i <= iters; ++i) {
    k_set<<<1, 64, 0, s>>>(flag, i);
    k_wait<<<1, 64, 0, s>>>(fl, n, rank, i, cnt + 1);
  }
  CK(hipStreamSynchronize(s));
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::printf("rank %d: %d flag rounds, %.2f us/round, %u timeouts\n", rank, iters, us / iters, cnt[1]);
  // rows rewritten by their owner after a flag, read by the others after the wait
  for (int i = 0; i < 4; ++i) {
    k_fill<<<1024, 256, 0, s>>>(rows, kWords, 100 * (i + 1) + rank);
    k_set<<<1, 64, 0, s>>>(flag, iters + 1 + 2 * i);
    k_wait<<<1, 64, 0, s>>>(fl, n, rank, iters + 1 + 2 * i, cnt + 1);
    for (int q = 0; q < n; ++q)
      if (q != rank) k_check<<<1024, 256, 0, s>>>(peer_rows[q], kWords, 100 * (i + 1) + q, cnt);
    CK(hipStreamSynchronize(s));
    barrier(m, n);
  }
  const bool ok = cnt[0] == 0 && cnt[1] == 0;
  std::printf("rank %d: %s\n", rank, ok ? "IPC_PROBE OK" : "IPC_PROBE FAIL");
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (n < 2 || n > kMax) return 2;
  setvbuf(stdout, nullptr, _IOLBF, 0);
  void* mem = mmap(nullptr, sizeof(Mail), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  auto* m = new (mem) Mail{};
  for (int r = 0; r < n; ++r)
    if (fork() == 0) std::_Exit(child(m, r, n, iters));
  int rc = 0;
  for (int r = 0; r < n; ++r) {
    int st = 0;
    wait(&st);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  std::printf("%s\n", rc ? "IPC_PROBE children failed" : "IPC_PROBE all ok");
  return rc;
}
