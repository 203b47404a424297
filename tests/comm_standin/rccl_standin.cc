// Test-only stand-in for the RCCL entry points cartographer-1_amd/csrc/comm.cc
// loads (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclAllGather,
// ncclAllReduce, ncclSend, ncclRecv, ncclGroupStart, ncclGroupEnd), so that
// comm.cc's RCCL code paths — the count AllGather, the root's staging
// agreement, the grouped Send / Recv of exact sizes into d_recv and the
// chunked AllReduce — run with 2-3 ranks on a one-GPU box, where real RCCL
// cannot make a multi-rank world. Loaded only through CSM_RCCL_LIB by tests.
//
// Semantics follow RCCL's documented API for what comm.cc uses: device
// buffers, stream order (the stream is synchronised before a device buffer is
// read, and written buffers are complete on return), Send / Recv deferred
// inside a group and run at ncclGroupEnd. The transport is a TCP star around
// rank 0 with host staging: peers talk only to rank 0, which is all comm.cc
// asks for (payloads flow to the root; counts and reductions go through it).
#include <arpa/inet.h>
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

namespace {

constexpr int kSuccess = 0, kSystemError = 2, kInvalidArgument = 4, kInvalidUsage = 5;

struct Id {  // ncclUniqueId: 128 bytes
  char magic[16];
  int32_t port;
  char pad[108];
};
static_assert(sizeof(Id) == 128, "ncclUniqueId is 128 bytes");
constexpr char kMagic[16] = "csm-rccl-stdin";

struct Comm {
  int rank = 0, size = 1;
  int root_fd = -1;        // peers: the socket to rank 0
  std::vector<int> peers;  // rank 0: one socket per peer (index = rank)
  int Fd(int peer) const { return rank == 0 ? peers[peer] : root_fd; }
};

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

bool RecvAll(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

size_t TypeBytes(int dtype) {
  switch (dtype) {
    case 0: case 1: return 1;           // int8, uint8
    case 2: case 3: case 7: return 4;   // int32, uint32, float32
    case 4: case 5: case 8: return 8;   // int64, uint64, float64
    case 6: return 2;                   // float16
    default: return 0;
  }
}

// Device <-> host with the stream's earlier work complete.
bool ToHost(void* dst, const void* src, size_t n, hipStream_t st) {
  if (hipStreamSynchronize(st) != hipSuccess) return false;
  return n == 0 || hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess;
}
bool ToDevice(void* dst, const void* src, size_t n) {
  return n == 0 || hipMemcpy(dst, src, n, hipMemcpyHostToDevice) == hipSuccess;
}

thread_local int group_depth = 0;
thread_local std::vector<std::function<int()>> deferred;

int RunOrDefer(std::function<int()> op) {
  if (group_depth > 0) {
    deferred.push_back(std::move(op));
    return kSuccess;
  }
  return op();
}

}  // namespace

extern "C" {

int ncclGetUniqueId(void* out) {
  if (!out) return kInvalidArgument;
  // A free port on the loopback for rank 0 to listen on.
  const int s = ::socket(AF_INET, SOCK_STREAM, 0);
  if (s < 0) return kSystemError;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t len = sizeof(a);
  if (::bind(s, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 ||
      ::getsockname(s, reinterpret_cast<sockaddr*>(&a), &len) < 0) {
    ::close(s);
    return kSystemError;
  }
  ::close(s);
  Id id{};
  std::memcpy(id.magic, kMagic, sizeof(kMagic));
  id.port = ntohs(a.sin_port);
  std::memcpy(out, &id, sizeof(id));
  return kSuccess;
}

int ncclCommInitRank(void** out, int nranks, Id id, int rank) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks ||
      std::memcmp(id.magic, kMagic, sizeof(kMagic)) != 0)
    return kInvalidArgument;
  auto* c = new Comm;
  c->rank = rank;
  c->size = nranks;
  const int one = 1;
  if (rank == 0) {
    c->peers.assign(nranks, -1);
    if (nranks > 1) {
      const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
      ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons(static_cast<uint16_t>(id.port));
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      if (ls < 0 || ::bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 ||
          ::listen(ls, 64) < 0) {
        if (ls >= 0) ::close(ls);
        delete c;
        return kSystemError;
      }
      for (int k = 1; k < nranks; ++k) {
        pollfd pf{ls, POLLIN, 0};
        int32_t r = -1;
        const int fd = ::poll(&pf, 1, 120000) > 0 ? ::accept(ls, nullptr, nullptr) : -1;
        if (fd < 0 || !RecvAll(fd, &r, sizeof(r)) || r <= 0 || r >= nranks || c->peers[r] >= 0) {
          if (fd >= 0) ::close(fd);
          ::close(ls);
          for (int p : c->peers)
            if (p >= 0) ::close(p);
          delete c;
          return kSystemError;
        }
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        c->peers[r] = fd;
      }
      ::close(ls);
    }
  } else {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(id.port));
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    int fd = -1;
    while (std::chrono::steady_clock::now() < deadline) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) break;
      if (fd >= 0) ::close(fd);
      fd = -1;
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    const int32_t r = rank;
    if (fd < 0 || !SendAll(fd, &r, sizeof(r))) {
      if (fd >= 0) ::close(fd);
      delete c;
      return kSystemError;
    }
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    c->root_fd = fd;
  }
  *out = c;
  return kSuccess;
}

int ncclCommDestroy(void* comm) {
  auto* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  for (int fd : c->peers)
    if (fd >= 0) ::close(fd);
  if (c->root_fd >= 0) ::close(c->root_fd);
  delete c;
  return kSuccess;
}

int ncclAllGather(const void* send, void* recv, size_t count, int dtype, void* comm,
                  hipStream_t st) {
  auto* c = static_cast<Comm*>(comm);
  const size_t b = count * TypeBytes(dtype);
  if (!c || (b == 0 && count)) return kInvalidArgument;
  std::vector<char> all(b * c->size);
  if (!ToHost(all.data() + b * c->rank, send, b, st)) return kSystemError;
  if (c->rank == 0) {
    for (int r = 1; r < c->size; ++r)
      if (!RecvAll(c->peers[r], all.data() + b * r, b)) return kSystemError;
    for (int r = 1; r < c->size; ++r)
      if (!SendAll(c->peers[r], all.data(), all.size())) return kSystemError;
  } else {
    if (!SendAll(c->root_fd, all.data() + b * c->rank, b) ||
        !RecvAll(c->root_fd, all.data(), all.size()))
      return kSystemError;
  }
  return ToDevice(recv, all.data(), all.size()) ? kSuccess : kSystemError;
}

int ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm,
                  hipStream_t st) {
  auto* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  if (dtype != 4 || (op != 0 && op != 2)) return kInvalidUsage;  // int64 sum / max (comm.cc's)
  std::vector<int64_t> v(count), o(count);
  if (!ToHost(v.data(), send, sizeof(int64_t) * count, st)) return kSystemError;
  const size_t b = sizeof(int64_t) * count;
  if (c->rank == 0) {
    for (int r = 1; r < c->size; ++r) {
      if (!RecvAll(c->peers[r], o.data(), b)) return kSystemError;
      for (size_t i = 0; i < count; ++i) v[i] = op == 2 ? std::max(v[i], o[i]) : v[i] + o[i];
    }
    for (int r = 1; r < c->size; ++r)
      if (!SendAll(c->peers[r], v.data(), b)) return kSystemError;
  } else if (!SendAll(c->root_fd, v.data(), b) || !RecvAll(c->root_fd, v.data(), b)) {
    return kSystemError;
  }
  return ToDevice(recv, v.data(), b) ? kSuccess : kSystemError;
}

int ncclSend(const void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t st) {
  auto* c = static_cast<Comm*>(comm);
  if (!c || peer < 0 || peer >= c->size || peer == c->rank || (c->rank != 0 && peer != 0))
    return kInvalidUsage;  // the star carries root <-> peer traffic only
  const size_t b = count * TypeBytes(dtype);
  return RunOrDefer([=] {
    std::vector<char> h(b);
    if (!ToHost(h.data(), buf, b, st)) return kSystemError;
    return SendAll(c->Fd(peer), h.data(), b) ? kSuccess : kSystemError;
  });
}

int ncclRecv(void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t st) {
  auto* c = static_cast<Comm*>(comm);
  if (!c || peer < 0 || peer >= c->size || peer == c->rank || (c->rank != 0 && peer != 0))
    return kInvalidUsage;
  const size_t b = count * TypeBytes(dtype);
  return RunOrDefer([=] {
    std::vector<char> h(b);
    if (hipStreamSynchronize(st) != hipSuccess) return kSystemError;
    if (!RecvAll(c->Fd(peer), h.data(), b)) return kSystemError;
    return ToDevice(buf, h.data(), b) ? kSuccess : kSystemError;
  });
}

int ncclGroupStart() {
  ++group_depth;
  return kSuccess;
}

int ncclGroupEnd() {
  if (group_depth <= 0) return kInvalidUsage;
  if (--group_depth > 0) return kSuccess;
  std::vector<std::function<int()>> ops;
  ops.swap(deferred);
  for (auto& op : ops) {
    const int rc = op();
    if (rc != kSuccess) return rc;
  }
  return kSuccess;
}

}  // extern "C"
