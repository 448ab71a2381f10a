// TCP key-value rendezvous store (parity: the TCPStore that env:// rendezvous
// creates for the reference's init_process_group, main.py:47-50).
//
// One process (rank 0) hosts the server; every rank (server host included)
// talks to it through a client connection. The store carries the RCCL unique
// id, the host communicator's peer addresses, barrier counters and the
// bucket-order agreement of the Reducer.
#pragma once

#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dcp {

class TCPStoreServer {
 public:
  TCPStoreServer(const std::string& host, int port);
  ~TCPStoreServer();
  int port() const { return port_; }
  void stop();

 private:
  void accept_loop();
  void serve(int fd);

  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::mutex threads_mu_;
  std::vector<std::thread> workers_;
  std::vector<int> client_fds_;

  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
};

class TCPStore {
 public:
  // is_master: host the server in this process. port 0 + is_master picks a free port.
  TCPStore(const std::string& host, int port, int world_size, bool is_master, int64_t timeout_ms,
           bool wait_for_workers);
  ~TCPStore();

  void set(const std::string& key, const std::string& value);
  // Blocks until key exists (or timeout).
  std::string get(const std::string& key);
  int64_t add(const std::string& key, int64_t delta);
  bool check(const std::vector<std::string>& keys);
  void wait(const std::vector<std::string>& keys, int64_t timeout_ms);
  bool delete_key(const std::string& key);
  int64_t num_keys();
  // Atomic compare-and-set; returns the value after the operation.
  std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired);
  // Store-based barrier over world_size participants (used at init / teardown only).
  void barrier(const std::string& tag);

  int port() const { return port_; }
  const std::string& host() const { return host_; }
  int world_size() const { return world_size_; }
  // Local IPv4 address of the connection to the store server (the address
  // peers can reach this process on).
  std::string local_ip() const;
  int64_t timeout_ms() const { return timeout_ms_; }
  void set_timeout_ms(int64_t t) { timeout_ms_ = t; }

 private:
  std::string request(uint8_t cmd, const std::vector<std::string>& args, int64_t timeout_ms);

  std::unique_ptr<TCPStoreServer> server_;
  std::string host_;
  int port_;
  int world_size_;
  int64_t timeout_ms_;
  int fd_ = -1;
  std::mutex mu_;  // one request at a time per client connection
  int64_t barrier_seq_ = 0;
};

}  // namespace dcp
