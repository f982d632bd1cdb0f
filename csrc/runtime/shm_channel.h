// Single-producer / multi-consumer broadcast channel in POSIX shared memory.
//
// The TP leader publishes each step plan (a few KB) to its followers through
// this channel instead of a torch.distributed (gloo/TCP) broadcast: one memcpy
// into a mapped segment plus an atomic sequence bump, and followers poll the
// sequence ("shared-memory ring from the scheduler, not RCCL,
// so the GPU stream is never blocked").
//
// Layout: Header (cache-line separated seq / acks) + data[capacity].
// Protocol (one message in flight):
//   producer: wait until every reader acked seq, write size + bytes, seq += 1 (release)
//   reader r: wait until seq > last (acquire), copy bytes, acks[r] = seq (release)
// Waiting spins briefly, then yields, then sleeps with capped exponential backoff,
// so an idle follower does not burn a core. A timeout (seconds, < 0 = forever)
// turns a dead peer into an error instead of a hang.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace xgs {

constexpr int kShmMaxReaders = 16;

struct ShmHeader {
  alignas(64) std::atomic<uint64_t> seq;
  alignas(64) std::atomic<uint64_t> size;
  alignas(64) std::atomic<uint64_t> acks[kShmMaxReaders];
  alignas(64) uint64_t capacity;
  uint32_t num_readers;
  uint32_t magic;
};

class ShmChannel {
 public:
  // create=true: the producer creates (and later unlinks) the segment.
  ShmChannel(const std::string& name, uint64_t capacity, int num_readers, bool create);
  ~ShmChannel();
  ShmChannel(const ShmChannel&) = delete;
  ShmChannel& operator=(const ShmChannel&) = delete;

  // producer; returns false on timeout (a reader never acknowledged)
  bool publish(const void* data, uint64_t n, double timeout_s);
  // reader `rank` (0..num_readers-1): wait for the next message and return its
  // size (-1 on timeout); then consume() copies it out and acknowledges it.
  int64_t wait_message(int rank, double timeout_s);
  void consume(int rank, void* out);

  uint64_t capacity() const { return cap_; }
  uint64_t seq() const;
  const std::string& name() const { return name_; }
  void unlink();

 private:
  std::string name_;
  bool owner_ = false;
  int fd_ = -1;
  uint64_t cap_ = 0;
  size_t map_bytes_ = 0;
  ShmHeader* hdr_ = nullptr;
  uint8_t* data_ = nullptr;
};

}  // namespace xgs
