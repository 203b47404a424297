// Multi-GPU hand-off of accepted constraints to rank 0: the
// constraint queue is sharded across ranks with no data-path collective; the
// one exchange is each rank's accepted-constraint records gathered to rank 0,
// where ConstraintBuilder2D::WhenDone's submission order is restored
// (constraint_builder_2d.cc:279-300) before the CPU pose-graph solve.
//
// Two transports behind one C-ABI (include/csm_amd.h, csm_comm_*):
//  * RCCL over xGMI (one process per GPU): counts by ncclAllGather, payloads
//    by grouped ncclSend/ncclRecv of the exact sizes into device staging on
//    the context's stream. librccl is loaded with dlopen on first use, so
//    libcsm_amd.so itself has no RCCL dependency.
//  * TCP (host sockets): the same operations between CPU processes, for the
//    world_size > 1 tests without GPUs and for rehearsals on one card.

#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <hip/hip_runtime.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/csm_amd.h"
#include "csm_internal.h"

namespace {

// ---- RCCL through dlopen ------------------------------------------------------
// The few entry points used, with the types of rccl.h reduced to what the
// ABI passes (ncclComm_t is a pointer, enums are ints, the unique id is 128 B).
using ncclComm_p = void*;
struct RcclApi {
  void* lib = nullptr;
  int (*GetUniqueId)(void* id) = nullptr;
  void* CommInitRank = nullptr;  // int(ncclComm_t*, int nranks, ncclUniqueId, int rank)
  int (*CommDestroy)(ncclComm_p) = nullptr;
  int (*AllGather)(const void*, void*, size_t, int, ncclComm_p, hipStream_t) = nullptr;
  int (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_p, hipStream_t) = nullptr;
  int (*Send)(const void*, size_t, int, int, ncclComm_p, hipStream_t) = nullptr;
  int (*Recv)(void*, size_t, int, int, ncclComm_p, hipStream_t) = nullptr;
  int (*GroupStart)() = nullptr;
  int (*GroupEnd)() = nullptr;
};

constexpr int kNcclInt8 = 0, kNcclInt64 = 4;  // ncclDataType_t
constexpr int kNcclSum = 0, kNcclMax = 2;      // ncclRedOp_t
constexpr int kIdBytes = CSM_COMM_ID_BYTES;

struct UniqueId {
  char internal[kIdBytes];
};

RcclApi* Rccl() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api.lib ? &api : nullptr;
  tried = true;
  // CSM_RCCL_LIB names another library with the same entry points (tests:
  // tests/comm_standin/, a TCP stand-in that lets several ranks share one GPU
  // box and run this file's RCCL code paths with N > 1).
  const char* over = std::getenv("CSM_RCCL_LIB");
  void* h = over && *over ? dlopen(over, RTLD_NOW | RTLD_LOCAL) : nullptr;
  if (over && *over && !h) return nullptr;  // asked for, not loadable: fail, no silent swap
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return nullptr;
  auto sym = [&](const char* n) { return dlsym(h, n); };
  api.GetUniqueId = reinterpret_cast<int (*)(void*)>(sym("ncclGetUniqueId"));
  api.CommInitRank = sym("ncclCommInitRank");
  api.CommDestroy = reinterpret_cast<int (*)(ncclComm_p)>(sym("ncclCommDestroy"));
  api.AllGather = reinterpret_cast<decltype(api.AllGather)>(sym("ncclAllGather"));
  api.AllReduce = reinterpret_cast<decltype(api.AllReduce)>(sym("ncclAllReduce"));
  api.Send = reinterpret_cast<decltype(api.Send)>(sym("ncclSend"));
  api.Recv = reinterpret_cast<decltype(api.Recv)>(sym("ncclRecv"));
  api.GroupStart = reinterpret_cast<int (*)()>(sym("ncclGroupStart"));
  api.GroupEnd = reinterpret_cast<int (*)()>(sym("ncclGroupEnd"));
  if (!api.GetUniqueId || !api.CommInitRank || !api.CommDestroy || !api.AllGather ||
      !api.AllReduce || !api.Send || !api.Recv || !api.GroupStart || !api.GroupEnd) {
    dlclose(h);
    return nullptr;
  }
  api.lib = h;
  return &api;
}

// ---- TCP helpers ----------------------------------------------------------------
// A signal delivered to this thread interrupts poll / send / recv (EINTR;
// Linux never restarts poll after a handler): retried, never read as a peer
// failure. A bounded wait keeps its deadline across the retries.
bool SendAll(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool RecvAll(int fd, void* p, size_t n, int timeout_ms) {
  char* c = static_cast<char*>(p);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(
                                                                  std::max(timeout_ms, 0));
  while (n) {
    int wait = -1;
    if (timeout_ms >= 0) {
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(
          deadline - std::chrono::steady_clock::now()).count();
      wait = static_cast<int>(std::max<long long>(left, 0));
    }
    pollfd pf{fd, POLLIN, 0};
    const int pr = ::poll(&pf, 1, wait);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Connection set-up (connect / accept) gives up after this long.
constexpr int kTcpTimeoutMs = 120000;

// Data receives of the collectives wait for the slowest rank: a rank reaches a
// gather only after its own share of the search, and at C3 scale ranks run
// for minutes, so the default is no limit (-1). CSM_COMM_TIMEOUT_MS bounds it
// (tests use a short one to exercise a late rank).
int DataTimeoutMs() {
  static const int v = [] {
    const char* e = std::getenv("CSM_COMM_TIMEOUT_MS");
    if (!e || !*e) return -1;
    const long t = std::strtol(e, nullptr, 10);
    return t > 0 ? static_cast<int>(std::min<long>(t, 0x7fffffff)) : -1;
  }();
  return v;
}

struct ClaimService;
void DestroyClaims(ClaimService* s);
struct ClaimDeleter {
  void operator()(ClaimService* s) const { DestroyClaims(s); }
};

}  // namespace

struct csm_comm {
  int rank = 0, size = 1;
  bool rccl = false;
  // RCCL
  csm_context* ctx = nullptr;
  ncclComm_p nccl = nullptr;
  csm::DevBuf d_send, d_recv, d_counts;
  // TCP: the root holds one socket per peer (index = rank), peers one to the root.
  std::vector<int> peers;
  int root_fd = -1;
  // The root's last gather: every rank's blob in rank order, and the sizes.
  std::vector<char> gathered;
  std::vector<int64_t> sizes;
  // Dynamic work claiming (csm_comm_claim_open); destroyed before the sockets.
  std::unique_ptr<ClaimService, ClaimDeleter> claims;

  ~csm_comm() {
    claims.reset();
    if (nccl && Rccl()) Rccl()->CommDestroy(nccl);
    for (int fd : peers)
      if (fd >= 0) ::close(fd);
    if (root_fd >= 0) ::close(root_fd);
  }
};

namespace {

int TcpConnect(csm_comm* c, const char* host, int port) {
  if (c->rank == 0) {
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return CSM_EINVAL;
    const int one = 1;
    ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 || ::listen(ls, 64) < 0) {
      ::close(ls);
      return CSM_EINVAL;
    }
    c->peers.assign(c->size, -1);
    for (int k = 1; k < c->size; ++k) {
      pollfd pf{ls, POLLIN, 0};
      if (::poll(&pf, 1, kTcpTimeoutMs) <= 0) { ::close(ls); return CSM_EINVAL; }
      const int fd = ::accept(ls, nullptr, nullptr);
      int32_t r = -1;
      if (fd < 0 || !RecvAll(fd, &r, sizeof(r), kTcpTimeoutMs) || r <= 0 || r >= c->size ||
          c->peers[r] >= 0) {
        if (fd >= 0) ::close(fd);
        ::close(ls);
        return CSM_EINVAL;
      }
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      c->peers[r] = fd;
    }
    ::close(ls);
    return CSM_OK;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  if (::getaddrinfo(host, ps.c_str(), &hints, &res) != 0 || !res) return CSM_EINVAL;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(kTcpTimeoutMs);
  int fd = -1;
  while (std::chrono::steady_clock::now() < deadline) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    if (fd >= 0) ::close(fd);
    fd = -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  ::freeaddrinfo(res);
  if (fd < 0) return CSM_EINVAL;
  const int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  const int32_t r = c->rank;
  if (!SendAll(fd, &r, sizeof(r))) { ::close(fd); return CSM_EINVAL; }
  c->root_fd = fd;
  return CSM_OK;
}

// Root receives every rank's blob into c->gathered (rank order).
int TcpGather(csm_comm* c, const void* send, int64_t bytes) {
  if (c->rank != 0) {
    if (!SendAll(c->root_fd, &bytes, sizeof(bytes)) ||
        (bytes > 0 && !SendAll(c->root_fd, send, static_cast<size_t>(bytes))))
      return CSM_EINVAL;
    return CSM_OK;
  }
  c->sizes.assign(c->size, 0);
  c->sizes[0] = bytes;
  for (int r = 1; r < c->size; ++r)
    if (!RecvAll(c->peers[r], &c->sizes[r], sizeof(int64_t), DataTimeoutMs()) || c->sizes[r] < 0)
      return CSM_EINVAL;
  int64_t total = 0;
  for (int64_t v : c->sizes) total += v;
  c->gathered.resize(static_cast<size_t>(total));
  if (bytes > 0) std::memcpy(c->gathered.data(), send, static_cast<size_t>(bytes));
  int64_t at = bytes;
  for (int r = 1; r < c->size; ++r) {
    if (c->sizes[r] > 0 &&
        !RecvAll(c->peers[r], c->gathered.data() + at, static_cast<size_t>(c->sizes[r]), DataTimeoutMs()))
      return CSM_EINVAL;
    at += c->sizes[r];
  }
  return CSM_OK;
}

int TcpAllreduce(csm_comm* c, int64_t* v, int n, int op) {
  const size_t b = sizeof(int64_t) * static_cast<size_t>(n);
  if (c->rank != 0) {
    if (!SendAll(c->root_fd, v, b) || !RecvAll(c->root_fd, v, b, DataTimeoutMs())) return CSM_EINVAL;
    return CSM_OK;
  }
  std::vector<int64_t> o(static_cast<size_t>(n));
  for (int r = 1; r < c->size; ++r) {
    if (!RecvAll(c->peers[r], o.data(), b, DataTimeoutMs())) return CSM_EINVAL;
    for (int i = 0; i < n; ++i) v[i] = op == CSM_REDUCE_MAX ? std::max(v[i], o[i]) : v[i] + o[i];
  }
  for (int r = 1; r < c->size; ++r)
    if (!SendAll(c->peers[r], v, b)) return CSM_EINVAL;
  return CSM_OK;
}

#define NCCL_OK(x)                      \
  do {                                  \
    if ((x) != 0) return CSM_EHIP;      \
  } while (0)

// Every failure a rank can hit locally (staging allocation) is exchanged
// before any payload moves, so either all ranks move data or all return the
// same error; no rank is left blocked in a Send or Recv. The count buffer is
// allocated when the communicator is created (kCountWords), so the count
// exchange itself never depends on an allocation.
constexpr int kCountWords = 64;

int RcclGather(csm_comm* c, const void* send, int64_t bytes) {
  RcclApi* R = Rccl();
  hipStream_t st = c->ctx->stream;
  if (hipSetDevice(c->ctx->device) != hipSuccess) return CSM_EHIP;
  if (c->size + 2 > kCountWords) return CSM_ERANGE;  // same on every rank
  int64_t* dc = c->d_counts.as<int64_t>();
  // A peer that cannot stage its payload reports -1 instead of its size.
  int64_t mine = bytes;
  if (c->rank != 0 && bytes > 0 && c->d_send.Reserve(static_cast<size_t>(bytes)) != CSM_OK) mine = -1;
  CSM_HIP(hipMemcpyAsync(dc + c->size, &mine, sizeof(int64_t), hipMemcpyHostToDevice, st));
  NCCL_OK(R->AllGather(dc + c->size, dc, 1, kNcclInt64, c->nccl, st));
  std::vector<int64_t> sz(c->size);
  CSM_HIP(hipMemcpyAsync(sz.data(), dc, sizeof(int64_t) * c->size, hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  int64_t total = 0;
  bool failed = false;
  for (int64_t v : sz) {
    failed |= v < 0;
    total += std::max<int64_t>(v, 0);
  }
  if (failed) return CSM_ENOMEM;  // every rank saw the same -1
  // The root stages the receive side, then tells every rank whether it could.
  int64_t root_fail = 0;
  if (c->rank == 0 && total > bytes && c->d_recv.Reserve(static_cast<size_t>(total)) != CSM_OK)
    root_fail = 1;
  if (total > sz[0]) {  // some peer has a payload: agree on the root's staging
    CSM_HIP(hipMemcpyAsync(dc + c->size + 1, &root_fail, sizeof(int64_t), hipMemcpyHostToDevice, st));
    NCCL_OK(R->AllReduce(dc + c->size + 1, dc + c->size + 1, 1, kNcclInt64, kNcclMax, c->nccl, st));
    CSM_HIP(hipMemcpyAsync(&root_fail, dc + c->size + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    if (root_fail) return CSM_ENOMEM;
  }
  if (c->rank != 0) {
    if (bytes == 0) return CSM_OK;
    CSM_HIP(hipMemcpyAsync(c->d_send.ptr, send, static_cast<size_t>(bytes), hipMemcpyHostToDevice, st));
    NCCL_OK(R->Send(c->d_send.ptr, static_cast<size_t>(bytes), kNcclInt8, 0, c->nccl, st));
    CSM_HIP(hipStreamSynchronize(st));
    return CSM_OK;
  }
  c->sizes = sz;
  c->gathered.resize(static_cast<size_t>(total));
  if (bytes > 0) std::memcpy(c->gathered.data(), send, static_cast<size_t>(bytes));
  if (total == bytes) return CSM_OK;
  char* dr = static_cast<char*>(c->d_recv.ptr);
  NCCL_OK(R->GroupStart());
  int64_t at = bytes;
  for (int r = 1; r < c->size; ++r) {
    if (sz[r] > 0) NCCL_OK(R->Recv(dr + at, static_cast<size_t>(sz[r]), kNcclInt8, r, c->nccl, st));
    at += sz[r];
  }
  NCCL_OK(R->GroupEnd());
  CSM_HIP(hipMemcpyAsync(c->gathered.data() + bytes, dr + bytes, static_cast<size_t>(total - bytes),
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  return CSM_OK;
}

// In pieces of kCountWords through the buffer allocated at creation.
int RcclAllreduce(csm_comm* c, int64_t* v, int n, int op) {
  RcclApi* R = Rccl();
  hipStream_t st = c->ctx->stream;
  if (hipSetDevice(c->ctx->device) != hipSuccess) return CSM_EHIP;
  int64_t* d = c->d_counts.as<int64_t>();
  for (int at = 0; at < n; at += kCountWords) {
    const int k = std::min(kCountWords, n - at);
    CSM_HIP(hipMemcpyAsync(d, v + at, sizeof(int64_t) * k, hipMemcpyHostToDevice, st));
    NCCL_OK(R->AllReduce(d, d, static_cast<size_t>(k), kNcclInt64,
                         op == CSM_REDUCE_MAX ? kNcclMax : kNcclSum, c->nccl, st));
    CSM_HIP(hipMemcpyAsync(v + at, d, sizeof(int64_t) * k, hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
  }
  return CSM_OK;
}

// ---- Dynamic work claiming ------------------------------------------------------
// The reference balances one task per pair on a shared queue
// (common/thread_pool.cc:80-106: idle workers pop the next task). Across
// processes the queue head is a table of counters on rank 0, served by a host
// thread: a peer sends (key, delta) and gets the counter's value before the
// add. Rank 0's own claims take the same mutex without a round trip. The
// transport is host TCP for RCCL communicators too: a claim is 24 bytes, and
// there is no device atomic shared between processes that RCCL exposes.
struct ClaimService {
  std::mutex mu;
  std::map<int64_t, int64_t> counters;
  int listen_fd = -1;
  int wake[2] = {-1, -1};  // self-pipe: destroy wakes the server's poll
  std::vector<int> peers;  // rank 0: one socket per peer; others: [0] = to the root
  std::thread server;

  int64_t FetchAddLocal(int64_t key, int64_t delta) {
    std::lock_guard<std::mutex> lock(mu);
    int64_t& v = counters[key];
    const int64_t old = v;
    v += delta;
    return old;
  }

  void Serve() {
    std::vector<pollfd> fds;
    for (;;) {
      fds.clear();
      fds.push_back(pollfd{wake[0], POLLIN, 0});
      for (int fd : peers)
        if (fd >= 0) fds.push_back(pollfd{fd, POLLIN, 0});
      if (fds.size() == 1) return;  // every peer has gone
      if (::poll(fds.data(), fds.size(), -1) < 0) return;
      if (fds[0].revents) return;
      for (size_t k = 1; k < fds.size(); ++k) {
        if (!fds[k].revents) continue;
        int64_t req[2];
        if (!RecvAll(fds[k].fd, req, sizeof(req), kTcpTimeoutMs)) {
          for (int& fd : peers)
            if (fd == fds[k].fd) { ::close(fd); fd = -1; }
          continue;
        }
        const int64_t old = FetchAddLocal(req[0], req[1]);
        if (!SendAll(fds[k].fd, &old, sizeof(old))) {
          for (int& fd : peers)
            if (fd == fds[k].fd) { ::close(fd); fd = -1; }
        }
      }
    }
  }

  ~ClaimService() {
    if (wake[1] >= 0) {
      const char b = 1;
      (void)!::write(wake[1], &b, 1);
    }
    if (server.joinable()) server.join();
    for (int fd : peers)
      if (fd >= 0) ::close(fd);
    for (int fd : wake)
      if (fd >= 0) ::close(fd);
  }
};

int ClaimOpen(csm_comm* c, const char* host, int port) {
  auto svc = std::make_unique<ClaimService>();
  if (c->size > 1) {
    // The same rendezvous as the TCP transport, on its own port.
    csm_comm tmp;
    tmp.rank = c->rank;
    tmp.size = c->size;
    const int rc = TcpConnect(&tmp, host, port);
    if (rc) return rc;
    if (c->rank == 0) {
      svc->peers = tmp.peers;
      tmp.peers.clear();
      if (::pipe(svc->wake) != 0) return CSM_EINVAL;
      ClaimService* raw = svc.get();
      svc->server = std::thread([raw] { raw->Serve(); });
    } else {
      svc->peers.assign(1, tmp.root_fd);
      tmp.root_fd = -1;
    }
  }
  c->claims.reset(svc.release());
  return CSM_OK;
}

void DestroyClaims(ClaimService* s) { delete s; }

int ClaimFetchAdd(csm_comm* c, int64_t key, int64_t delta, int64_t* old) {
  ClaimService* s = c->claims.get();
  if (c->rank == 0 || c->size == 1) {
    *old = s->FetchAddLocal(key, delta);
    return CSM_OK;
  }
  // One request in flight per rank; callers on several threads take turns.
  std::lock_guard<std::mutex> lock(s->mu);
  const int64_t req[2] = {key, delta};
  if (!SendAll(s->peers[0], req, sizeof(req)) || !RecvAll(s->peers[0], old, sizeof(*old), DataTimeoutMs()))
    return CSM_EINVAL;
  return CSM_OK;
}

}  // namespace

extern "C" {

int csm_comm_get_unique_id(uint8_t* id) {
  if (!id) return CSM_EINVAL;
  RcclApi* R = Rccl();
  if (!R) return CSM_EHIP;
  UniqueId u;
  if (R->GetUniqueId(&u) != 0) return CSM_EHIP;
  std::memcpy(id, u.internal, kIdBytes);
  return CSM_OK;
}

int csm_comm_create_rccl(csm_context* ctx, int32_t rank, int32_t world_size, const uint8_t* id,
                         csm_comm** out) {
  if (!ctx || !id || !out || world_size < 1 || rank < 0 || rank >= world_size) return CSM_EINVAL;
  // The gather's count exchange uses a fixed buffer of kCountWords words
  // (world_size counts + 2 agreement words): refuse larger worlds here rather
  // than at the first gather.
  if (world_size > kCountWords - 2) return CSM_ERANGE;
  RcclApi* R = Rccl();
  if (!R) return CSM_EHIP;
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  auto c = std::make_unique<csm_comm>();
  c->rank = rank;
  c->size = world_size;
  c->rccl = true;
  c->ctx = ctx;
  UniqueId u;
  std::memcpy(u.internal, id, kIdBytes);
  // ncclCommInitRank(comm, nranks, ncclUniqueId (128 B by value), rank)
  using Init = int (*)(ncclComm_p*, int, UniqueId, int);
  if (c->d_counts.Reserve(sizeof(int64_t) * kCountWords)) return CSM_ENOMEM;
  if (reinterpret_cast<Init>(R->CommInitRank)(&c->nccl, world_size, u, rank) != 0)
    return CSM_EHIP;
  *out = c.release();
  return CSM_OK;
}

int csm_comm_create_tcp(int32_t rank, int32_t world_size, const char* root_host, int32_t port,
                        csm_comm** out) {
  if (!out || world_size < 1 || rank < 0 || rank >= world_size || port <= 0 || port > 65535 ||
      (rank != 0 && !root_host))
    return CSM_EINVAL;
  auto c = std::make_unique<csm_comm>();
  c->rank = rank;
  c->size = world_size;
  if (world_size > 1) {
    const int rc = TcpConnect(c.get(), root_host, port);
    if (rc) return rc;
  }
  *out = c.release();
  return CSM_OK;
}

void csm_comm_destroy(csm_comm* c) { delete c; }

int32_t csm_comm_rank(const csm_comm* c) { return c ? c->rank : -1; }
int32_t csm_comm_size(const csm_comm* c) { return c ? c->size : 0; }

int csm_comm_gather(csm_comm* c, const void* send, int64_t send_bytes, int64_t* total_bytes) {
  if (!c || send_bytes < 0 || (send_bytes > 0 && !send)) return CSM_EINVAL;
  int rc;
  if (c->size == 1) {
    c->sizes.assign(1, send_bytes);
    c->gathered.assign(static_cast<const char*>(send), static_cast<const char*>(send) + send_bytes);
    rc = CSM_OK;
  } else {
    c->gathered.clear();
    c->sizes.clear();
    rc = c->rccl ? RcclGather(c, send, send_bytes) : TcpGather(c, send, send_bytes);
  }
  if (total_bytes) *total_bytes = c->rank == 0 ? static_cast<int64_t>(c->gathered.size()) : 0;
  return rc;
}

int csm_comm_gathered(const csm_comm* c, void* out, int64_t capacity, int64_t* sizes) {
  if (!c) return CSM_EINVAL;
  if (c->rank != 0) return CSM_EINVAL;
  const int64_t total = static_cast<int64_t>(c->gathered.size());
  if (total > capacity || (total > 0 && !out)) return CSM_ERANGE;
  if (total > 0) std::memcpy(out, c->gathered.data(), static_cast<size_t>(total));
  if (sizes) std::copy(c->sizes.begin(), c->sizes.end(), sizes);
  return CSM_OK;
}

int csm_comm_allreduce_i64(csm_comm* c, int64_t* values, int32_t count, int32_t op) {
  if (!c || count < 0 || (count > 0 && !values) || (op != CSM_REDUCE_SUM && op != CSM_REDUCE_MAX))
    return CSM_EINVAL;
  if (c->size == 1 || count == 0) return CSM_OK;
  return c->rccl ? RcclAllreduce(c, values, count, op) : TcpAllreduce(c, values, count, op);
}

int csm_comm_barrier(csm_comm* c) {
  int64_t v = 0;
  return csm_comm_allreduce_i64(c, &v, 1, CSM_REDUCE_SUM);
}

int csm_comm_claim_open(csm_comm* c, const char* root_host, int32_t port) {
  if (!c || c->claims || (c->size > 1 && (port <= 0 || port > 65535 || (c->rank != 0 && !root_host))))
    return CSM_EINVAL;
  return ClaimOpen(c, root_host, port);
}

int csm_comm_fetch_add(csm_comm* c, int64_t key, int64_t delta, int64_t* old_value) {
  if (!c || !c->claims || !old_value) return CSM_EINVAL;
  return ClaimFetchAdd(c, key, delta, old_value);
}

}  // extern "C"
