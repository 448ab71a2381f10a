// Minimal blocking TCP socket helpers shared by the rendezvous store and the
// host (CPU) communicator. IPv4 only: rendezvous on this pool is 127.0.0.1 /
// a node-local address.
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <cerrno>
#include <string>
#include <thread>
#include <vector>

#include "../common.h"

namespace dcp {
namespace net {

inline void set_nodelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

inline void set_bufsizes(int fd, int bytes) {
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof(bytes));
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof(bytes));
}

inline void set_nonblocking(int fd, bool nb) {
  int flags = ::fcntl(fd, F_GETFL, 0);
  if (nb)
    flags |= O_NONBLOCK;
  else
    flags &= ~O_NONBLOCK;
  ::fcntl(fd, F_SETFL, flags);
}

inline std::string resolve_ipv4(const std::string& host) {
  if (host.empty() || host == "localhost") return "127.0.0.1";
  in_addr a{};
  if (::inet_pton(AF_INET, host.c_str(), &a) == 1) return host;
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  int rc = ::getaddrinfo(host.c_str(), nullptr, &hints, &res);
  DK_CHECK(rc == 0 && res != nullptr, "cannot resolve host '", host, "': ", gai_strerror(rc));
  char buf[INET_ADDRSTRLEN];
  ::inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr, buf, sizeof(buf));
  ::freeaddrinfo(res);
  return std::string(buf);
}

// Bind + listen on host:port (port 0 = ephemeral). Returns fd; *bound_port gets the port.
inline int listen_on(const std::string& host, int port, int* bound_port, int backlog = 512) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  DK_CHECK(fd >= 0, "socket() failed: ", std::strerror(errno));
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  std::string ip = host.empty() ? std::string("0.0.0.0") : resolve_ipv4(host);
  ::inet_pton(AF_INET, ip.c_str(), &addr.sin_addr);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    int e = errno;
    ::close(fd);
    throw Error(str_cat("bind(", ip, ":", port, ") failed: ", std::strerror(e)));
  }
  DK_CHECK(::listen(fd, backlog) == 0, "listen() failed: ", std::strerror(errno));
  socklen_t len = sizeof(addr);
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &len);
  if (bound_port) *bound_port = ntohs(addr.sin_port);
  return fd;
}

// Connect with retry until timeout_ms elapses (the server may not be up yet).
inline int connect_to(const std::string& host, int port, int64_t timeout_ms) {
  std::string ip = resolve_ipv4(host);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  ::inet_pton(AF_INET, ip.c_str(), &addr.sin_addr);
  const int64_t deadline = now_ms() + timeout_ms;
  int delay_ms = 2;
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    DK_CHECK(fd >= 0, "socket() failed: ", std::strerror(errno));
    if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    int e = errno;
    ::close(fd);
    if (now_ms() > deadline) {
      throw TimeoutError(str_cat("timed out connecting to ", ip, ":", port, " (", std::strerror(e), ")"));
    }
    std::this_thread::sleep_for(Millis(delay_ms));
    delay_ms = std::min(delay_ms * 2, 100);
  }
}

inline int accept_one(int listen_fd, int64_t timeout_ms) {
  pollfd p{listen_fd, POLLIN, 0};
  int rc = ::poll(&p, 1, timeout_ms < 0 ? -1 : static_cast<int>(timeout_ms));
  if (rc == 0) throw TimeoutError("timed out waiting for peer connection");
  DK_CHECK(rc > 0, "poll() failed: ", std::strerror(errno));
  int fd = ::accept(listen_fd, nullptr, nullptr);
  DK_CHECK(fd >= 0, "accept() failed: ", std::strerror(errno));
  set_nodelay(fd);
  return fd;
}

// Blocking full send / recv. Return false on orderly shutdown/EOF.
inline bool send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd, POLLOUT, 0};
        ::poll(&pf, 1, 1000);
        continue;
      }
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Receive exactly n bytes; timeout_ms < 0 blocks forever.
inline bool recv_all(int fd, void* buf, size_t n, int64_t timeout_ms = -1) {
  char* p = static_cast<char*>(buf);
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  while (n > 0) {
    if (deadline >= 0) {
      int64_t left = deadline - now_ms();
      if (left <= 0) throw TimeoutError("socket receive timed out");
      pollfd pf{fd, POLLIN, 0};
      int rc = ::poll(&pf, 1, static_cast<int>(std::min<int64_t>(left, 1 << 30)));
      if (rc == 0) throw TimeoutError("socket receive timed out");
      if (rc < 0 && errno == EINTR) continue;
    }
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd, POLLIN, 0};
        ::poll(&pf, 1, 1000);
        continue;
      }
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Full-duplex exchange: send `sn` bytes to send_fd while receiving `rn` bytes
// from recv_fd. Needed by ring collectives so two neighbours never deadlock on
// full kernel socket buffers.
inline void send_recv(int send_fd, const void* sbuf, size_t sn, int recv_fd, void* rbuf, size_t rn,
                      int64_t timeout_ms) {
  const char* sp = static_cast<const char*>(sbuf);
  char* rp = static_cast<char*>(rbuf);
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  while (sn > 0 || rn > 0) {
    pollfd pf[2];
    int np = 0;
    int si = -1, ri = -1;
    if (sn > 0) {
      pf[np] = {send_fd, POLLOUT, 0};
      si = np++;
    }
    if (rn > 0) {
      pf[np] = {recv_fd, POLLIN, 0};
      ri = np++;
    }
    int wait = 1000;
    if (deadline >= 0) {
      int64_t left = deadline - now_ms();
      if (left <= 0) throw TimeoutError("host collective timed out in send_recv");
      wait = static_cast<int>(std::min<int64_t>(left, 1000));
    }
    int rc = ::poll(pf, np, wait);
    if (rc < 0) {
      if (errno == EINTR) continue;
      throw Error(str_cat("poll failed: ", std::strerror(errno)));
    }
    if (rc == 0) continue;
    if (si >= 0 && (pf[si].revents & (POLLOUT | POLLERR | POLLHUP))) {
      ssize_t k = ::send(send_fd, sp, sn, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (k > 0) {
        sp += k;
        sn -= static_cast<size_t>(k);
      } else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
        throw Error(str_cat("peer send failed: ", std::strerror(errno)));
      }
    }
    if (ri >= 0 && (pf[ri].revents & (POLLIN | POLLERR | POLLHUP))) {
      ssize_t k = ::recv(recv_fd, rp, rn, MSG_DONTWAIT);
      if (k > 0) {
        rp += k;
        rn -= static_cast<size_t>(k);
      } else if (k == 0) {
        throw Error("peer closed connection during collective");
      } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
        throw Error(str_cat("peer recv failed: ", std::strerror(errno)));
      }
    }
  }
}

}  // namespace net
}  // namespace dcp
