#include "shm_channel.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace xgs {

namespace {

constexpr uint32_t kMagic = 0x5847434Eu;  // "XGCN"

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Spin -> yield -> sleep (10 us doubling to 1 ms). Returns false once
// `timeout_s` (>= 0) has elapsed without `ready()` becoming true.
template <typename F>
bool wait_for(F ready, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int i = 0; i < 2000; ++i) {
    if (ready()) return true;
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  for (int i = 0; i < 200; ++i) {
    if (ready()) return true;
    sched_yield();
  }
  long sleep_us = 10;
  for (;;) {
    if (ready()) return true;
    if (timeout_s >= 0 &&
        std::chrono::duration<double>(clk::now() - t0).count() > timeout_s)
      return false;
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    if (sleep_us < 1000) sleep_us *= 2;
  }
}

}  // namespace

ShmChannel::ShmChannel(const std::string& name, uint64_t capacity, int num_readers,
                       bool create)
    : name_(name[0] == '/' ? name : "/" + name), owner_(create) {
  if (num_readers < 0 || num_readers > kShmMaxReaders)
    throw std::invalid_argument("ShmChannel: num_readers out of range");
  if (create) {
    ::shm_unlink(name_.c_str());  // stale segment from a crashed run
    fd_ = ::shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  } else {
    fd_ = ::shm_open(name_.c_str(), O_RDWR, 0600);
  }
  if (fd_ < 0) throw std::runtime_error("ShmChannel: shm_open failed for " + name_);

  if (create) {
    cap_ = round_up(capacity, 64);
    map_bytes_ = round_up(sizeof(ShmHeader), 4096) + cap_;
    if (::ftruncate(fd_, (off_t)map_bytes_) != 0) {
      ::close(fd_);
      ::shm_unlink(name_.c_str());
      throw std::runtime_error("ShmChannel: ftruncate failed");
    }
  } else {
    struct stat st;
    if (::fstat(fd_, &st) != 0 || (size_t)st.st_size < sizeof(ShmHeader)) {
      ::close(fd_);
      throw std::runtime_error("ShmChannel: segment not initialised: " + name_);
    }
    map_bytes_ = (size_t)st.st_size;
  }
  void* p = ::mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (p == MAP_FAILED) {
    ::close(fd_);
    if (create) ::shm_unlink(name_.c_str());
    throw std::runtime_error("ShmChannel: mmap failed");
  }
  hdr_ = static_cast<ShmHeader*>(p);
  data_ = static_cast<uint8_t*>(p) + round_up(sizeof(ShmHeader), 4096);
  if (create) {
    std::memset(p, 0, round_up(sizeof(ShmHeader), 4096));
    hdr_->capacity = cap_;
    hdr_->num_readers = (uint32_t)num_readers;
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    if (hdr_->magic != kMagic) {
      ::munmap(p, map_bytes_);
      ::close(fd_);
      throw std::runtime_error("ShmChannel: bad magic in " + name_);
    }
    cap_ = hdr_->capacity;
  }
}

ShmChannel::~ShmChannel() {
  if (hdr_) ::munmap(hdr_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
  if (owner_) ::shm_unlink(name_.c_str());
}

void ShmChannel::unlink() {
  if (owner_) {
    ::shm_unlink(name_.c_str());
    owner_ = false;
  }
}

uint64_t ShmChannel::seq() const { return hdr_->seq.load(std::memory_order_acquire); }

bool ShmChannel::publish(const void* data, uint64_t n, double timeout_s) {
  if (n > cap_) throw std::length_error("ShmChannel: message larger than capacity");
  const uint64_t cur = hdr_->seq.load(std::memory_order_relaxed);
  const uint32_t nr = hdr_->num_readers;
  bool ok = wait_for(
      [&] {
        for (uint32_t r = 0; r < nr; ++r)
          if (hdr_->acks[r].load(std::memory_order_acquire) < cur) return false;
        return true;
      },
      timeout_s);
  if (!ok) return false;
  std::memcpy(data_, data, n);
  hdr_->size.store(n, std::memory_order_relaxed);
  hdr_->seq.store(cur + 1, std::memory_order_release);
  return true;
}

int64_t ShmChannel::wait_message(int rank, double timeout_s) {
  if (rank < 0 || rank >= (int)hdr_->num_readers)
    throw std::out_of_range("ShmChannel: reader rank out of range");
  // acks[rank] is written only by this reader: it is the last message consumed,
  // so a reader attaching late still receives the message it has not acked.
  const uint64_t last = hdr_->acks[rank].load(std::memory_order_relaxed);
  bool ok = wait_for([&] { return hdr_->seq.load(std::memory_order_acquire) > last; },
                     timeout_s);
  if (!ok) return -1;
  return (int64_t)hdr_->size.load(std::memory_order_relaxed);
}

void ShmChannel::consume(int rank, void* out) {
  // size/data were published before seq (release) and observed after the
  // acquire load in wait_message, so they are stable until we ack.
  const uint64_t s = hdr_->seq.load(std::memory_order_acquire);
  std::memcpy(out, data_, hdr_->size.load(std::memory_order_relaxed));
  hdr_->acks[rank].store(s, std::memory_order_release);
}

}  // namespace xgs
