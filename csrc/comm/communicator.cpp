#include "communicator.h"

#include "../common.h"

namespace dcp {

void Communicator::account(const char* op, const at::Tensor& t, int64_t extra) {
  ops_.fetch_add(1);
  bytes_.fetch_add(t.numel() * t.element_size());
  if (fingerprint_) check_fingerprint(op, t, extra);
}

void Communicator::check_fingerprint(const char* op, const at::Tensor& t, int64_t extra) {
  // All ranks publish their fingerprint for this sequence number, then each
  // compares against rank 0's. Debug only: costs two store round trips.
  const int64_t seq = seq_++;
  const std::string fp = str_cat(op, "|", c10::toString(t.scalar_type()), "|", t.numel(), "|", extra);
  const std::string base = str_cat(prefix_, "/fp/", seq, "/");
  store_->set(base + std::to_string(rank_), fp);
  const std::string ref = store_->get(base + "0");
  if (ref != fp) {
    throw Error(str_cat("collective mismatch at sequence ", seq, ": rank ", rank_, " issued [", fp,
                        "] but rank 0 issued [", ref, "]"));
  }
}

}  // namespace dcp
