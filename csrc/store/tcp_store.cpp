#include "tcp_store.h"

#include "../common.h"
#include "socket.h"

namespace dcp {

namespace {

enum Cmd : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, WAIT = 5, DEL = 6, NUM = 7, CAS = 8 };
enum Status : uint8_t { OK = 0, TIMEOUT = 1, FAIL = 2 };

bool read_args(int fd, std::vector<std::string>* args) {
  uint32_t n = 0;
  if (!net::recv_all(fd, &n, sizeof(n))) return false;
  if (n > 1u << 20) return false;
  args->resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t len = 0;
    if (!net::recv_all(fd, &len, sizeof(len))) return false;
    if (len > (1ull << 34)) return false;
    (*args)[i].resize(len);
    if (len && !net::recv_all(fd, &(*args)[i][0], len)) return false;
  }
  return true;
}

bool write_reply(int fd, uint8_t status, const std::string& payload) {
  std::string buf;
  buf.reserve(9 + payload.size());
  buf.push_back(static_cast<char>(status));
  uint64_t len = payload.size();
  buf.append(reinterpret_cast<const char*>(&len), sizeof(len));
  buf.append(payload);
  return net::send_all(fd, buf.data(), buf.size());
}

}  // namespace

// ---------------------------------------------------------------- server ---

TCPStoreServer::TCPStoreServer(const std::string& host, int port) {
  // Bind on all interfaces so both 127.0.0.1 and the node address reach us.
  (void)host;
  listen_fd_ = net::listen_on("0.0.0.0", port, &port_);
  acceptor_ = std::thread([this] { accept_loop(); });
}

TCPStoreServer::~TCPStoreServer() { stop(); }

void TCPStoreServer::stop() {
  if (stop_.exchange(true)) return;
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  {
    std::lock_guard<std::mutex> g(threads_mu_);
    for (int fd : client_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  cv_.notify_all();
  if (acceptor_.joinable()) acceptor_.join();
  std::vector<std::thread> ws;
  {
    std::lock_guard<std::mutex> g(threads_mu_);
    ws.swap(workers_);
  }
  for (auto& t : ws)
    if (t.joinable()) t.join();
}

void TCPStoreServer::accept_loop() {
  while (!stop_.load()) {
    pollfd p{listen_fd_, POLLIN, 0};
    int rc = ::poll(&p, 1, 200);
    if (rc <= 0) continue;
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    net::set_nodelay(fd);
    std::lock_guard<std::mutex> g(threads_mu_);
    client_fds_.push_back(fd);
    workers_.emplace_back([this, fd] { serve(fd); });
  }
}

void TCPStoreServer::serve(int fd) {
  std::vector<std::string> args;
  while (!stop_.load()) {
    uint8_t cmd = 0;
    if (!net::recv_all(fd, &cmd, 1)) break;
    if (!read_args(fd, &args)) break;
    std::string reply;
    uint8_t status = OK;
    try {
      switch (cmd) {
        case SET: {
          DK_CHECK(args.size() == 2, "SET arity");
          {
            std::lock_guard<std::mutex> g(mu_);
            kv_[args[0]] = args[1];
          }
          cv_.notify_all();
          break;
        }
        case GET:
        case WAIT: {
          DK_CHECK(!args.empty(), "GET/WAIT arity");
          const int64_t timeout_ms = std::stoll(args.back());
          const size_t nkeys = args.size() - 1;
          std::unique_lock<std::mutex> lk(mu_);
          auto ready = [&] {
            if (stop_.load()) return true;
            for (size_t i = 0; i < nkeys; ++i)
              if (!kv_.count(args[i])) return false;
            return true;
          };
          bool ok = timeout_ms < 0 ? (cv_.wait(lk, ready), true)
                                   : cv_.wait_for(lk, Millis(timeout_ms), ready);
          if (!ok || stop_.load()) {
            status = TIMEOUT;
          } else if (cmd == GET) {
            reply = kv_[args[0]];
          }
          break;
        }
        case ADD: {
          DK_CHECK(args.size() == 2, "ADD arity");
          int64_t v;
          {
            std::lock_guard<std::mutex> g(mu_);
            auto it = kv_.find(args[0]);
            int64_t cur = it == kv_.end() ? 0 : std::stoll(it->second);
            v = cur + std::stoll(args[1]);
            kv_[args[0]] = std::to_string(v);
          }
          cv_.notify_all();
          reply = std::to_string(v);
          break;
        }
        case CHECK: {
          std::lock_guard<std::mutex> g(mu_);
          bool all = true;
          for (auto& k : args) all = all && kv_.count(k);
          reply = all ? "1" : "0";
          break;
        }
        case DEL: {
          DK_CHECK(args.size() == 1, "DEL arity");
          std::lock_guard<std::mutex> g(mu_);
          reply = kv_.erase(args[0]) ? "1" : "0";
          break;
        }
        case NUM: {
          std::lock_guard<std::mutex> g(mu_);
          reply = std::to_string(kv_.size());
          break;
        }
        case CAS: {
          DK_CHECK(args.size() == 3, "CAS arity");
          {
            std::lock_guard<std::mutex> g(mu_);
            auto it = kv_.find(args[0]);
            if (it == kv_.end()) {
              if (args[1].empty()) kv_[args[0]] = args[2];
            } else if (it->second == args[1]) {
              it->second = args[2];
            }
            reply = kv_.count(args[0]) ? kv_[args[0]] : std::string();
          }
          cv_.notify_all();
          break;
        }
        default:
          status = FAIL;
          reply = "unknown command";
      }
    } catch (const std::exception& e) {
      status = FAIL;
      reply = e.what();
    }
    if (!write_reply(fd, status, reply)) break;
  }
  ::close(fd);
}

// ---------------------------------------------------------------- client ---

TCPStore::TCPStore(const std::string& host, int port, int world_size, bool is_master, int64_t timeout_ms,
                   bool wait_for_workers)
    : host_(host), port_(port), world_size_(world_size), timeout_ms_(timeout_ms) {
  if (is_master) {
    server_ = std::make_unique<TCPStoreServer>(host, port);
    port_ = server_->port();
  }
  fd_ = net::connect_to(is_master ? std::string("127.0.0.1") : host, port_, timeout_ms_);
  if (wait_for_workers && world_size_ > 0) {
    // Every participant checks in; the master waits for all of them so a
    // late worker cannot find the server already gone.
    add("__dcp/init/joined", 1);
    if (is_master) {
      const int64_t deadline = now_ms() + timeout_ms_;
      while (std::stoll(get("__dcp/init/joined")) < world_size_) {
        if (now_ms() > deadline) throw TimeoutError("store: timed out waiting for workers to join");
        std::this_thread::sleep_for(Millis(5));
      }
    }
  }
}

TCPStore::~TCPStore() {
  if (fd_ >= 0) ::close(fd_);
  if (server_) server_->stop();
}

std::string TCPStore::request(uint8_t cmd, const std::vector<std::string>& args, int64_t timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  std::string buf;
  buf.push_back(static_cast<char>(cmd));
  uint32_t n = static_cast<uint32_t>(args.size());
  buf.append(reinterpret_cast<const char*>(&n), sizeof(n));
  for (auto& a : args) {
    uint64_t len = a.size();
    buf.append(reinterpret_cast<const char*>(&len), sizeof(len));
    buf.append(a);
  }
  DK_CHECK(net::send_all(fd_, buf.data(), buf.size()), "store: connection to server lost (send)");
  uint8_t status = 0;
  // Allow the server side timeout to fire first, then a grace period.
  const int64_t wait = timeout_ms < 0 ? -1 : timeout_ms + 5000;
  DK_CHECK(net::recv_all(fd_, &status, 1, wait), "store: connection to server lost (recv)");
  uint64_t len = 0;
  DK_CHECK(net::recv_all(fd_, &len, sizeof(len), wait), "store: connection lost");
  std::string payload(len, '\0');
  if (len) DK_CHECK(net::recv_all(fd_, &payload[0], len, wait), "store: connection lost");
  if (status == TIMEOUT) throw TimeoutError("store: timed out waiting for key(s)");
  if (status != OK) throw Error("store: server error: " + payload);
  return payload;
}

std::string TCPStore::local_ip() const {
  sockaddr_in a{};
  socklen_t len = sizeof(a);
  if (::getsockname(fd_, reinterpret_cast<sockaddr*>(&a), &len) != 0) return "127.0.0.1";
  char buf[INET_ADDRSTRLEN];
  ::inet_ntop(AF_INET, &a.sin_addr, buf, sizeof(buf));
  return std::string(buf);
}

void TCPStore::set(const std::string& key, const std::string& value) { request(SET, {key, value}, -1); }

std::string TCPStore::get(const std::string& key) {
  return request(GET, {key, std::to_string(timeout_ms_)}, timeout_ms_);
}

int64_t TCPStore::add(const std::string& key, int64_t delta) {
  return std::stoll(request(ADD, {key, std::to_string(delta)}, -1));
}

bool TCPStore::check(const std::vector<std::string>& keys) { return request(CHECK, keys, -1) == "1"; }

void TCPStore::wait(const std::vector<std::string>& keys, int64_t timeout_ms) {
  std::vector<std::string> args(keys);
  const int64_t t = timeout_ms < 0 ? timeout_ms_ : timeout_ms;
  args.push_back(std::to_string(t));
  request(WAIT, args, t);
}

bool TCPStore::delete_key(const std::string& key) { return request(DEL, {key}, -1) == "1"; }

int64_t TCPStore::num_keys() { return std::stoll(request(NUM, {}, -1)); }

std::string TCPStore::compare_set(const std::string& key, const std::string& expected, const std::string& desired) {
  return request(CAS, {key, expected, desired}, -1);
}

void TCPStore::barrier(const std::string& tag) {
  const int64_t seq = barrier_seq_++;
  const std::string base = str_cat("__dcp/barrier/", tag, "/", seq);
  const int64_t arrived = add(base + "/count", 1);
  if (arrived == world_size_) set(base + "/done", "1");
  wait({base + "/done"}, timeout_ms_);
}

}  // namespace dcp
