// Three-class priority queue with watermark hysteresis (backpressure).
//
// Behavioural parity with the reference `crates/core/src/queue.rs:74-250`:
//   * enqueue (queue.rs:103-126): reject when backpressure is active, or when
//     total >= max_queue_size; otherwise push to the class FIFO and THEN
//     recompute backpressure.
//   * backpressure (queue.rs:235-249): inactive -> active iff total >
//     high_watermark (strict); active -> inactive iff total < low_watermark
//     (strict). Recomputed only on mutation.
//   * dequeue_batch / dequeue_one (queue.rs:130-170): strict High > Normal > Low,
//     FIFO inside a class.
//   * remove_expired (queue.rs:198-226): elapsed > timeout (strict), order
//     preserved, High then Normal then Low.
// Additions (spec'd, not built in the reference): cancel(id) (design.md:215),
// optional aging (Req 3.5, requirements.md:61; off by default), injectable
// clock so timeouts are testable without sleeping.
//
// Thread-safety: every public method takes the object's mutex (the Rust type
// was `&mut self`, so its caller had to serialise; here the queue is shared by
// the HTTP threads and the engine driver).
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <deque>
#include <mutex>
#include <optional>
#include <string>
#include <utility>
#include <vector>

namespace xgs {

enum class Priority : uint8_t { Low = 0, Normal = 1, High = 2 };

struct QueueConfig {
  size_t high_watermark = 1000;
  size_t low_watermark = 500;
  double request_timeout_s = 30.0;
  size_t max_queue_size = 2000;
  // 0 = strict priority (reference behaviour). >0: a request is promoted one
  // class for every `aging_s` seconds it has waited (anti-starvation, Req 3.5).
  double aging_s = 0.0;
};

struct QueueDepth {
  size_t high = 0, normal = 0, low = 0, total = 0;
};

enum class EnqueueResult : uint8_t { Ok = 0, Full = 1 };

template <typename T>
struct QueuedRequest {
  std::string id;
  T data;
  Priority priority;
  double enqueued_at;  // seconds on the queue's clock
};

inline double steady_now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

template <typename T>
class PriorityQueueManager {
 public:
  using Item = QueuedRequest<T>;

  explicit PriorityQueueManager(QueueConfig cfg = QueueConfig()) : cfg_(cfg) {}

  // ---- clock ---------------------------------------------------------------
  void set_manual_clock(bool on, double t = 0.0) {
    std::lock_guard<std::mutex> g(mu_);
    manual_ = on;
    manual_t_ = t;
  }
  void advance_clock(double dt) {
    std::lock_guard<std::mutex> g(mu_);
    manual_t_ += dt;
  }
  double now() const {
    std::lock_guard<std::mutex> g(mu_);
    return now_locked();
  }

  // ---- mutation --------------------------------------------------------------
  EnqueueResult enqueue(std::string id, T data, Priority p) {
    std::lock_guard<std::mutex> g(mu_);
    if (backpressure_) return EnqueueResult::Full;
    if (total_locked() >= cfg_.max_queue_size) return EnqueueResult::Full;
    q_[idx(p)].push_back(Item{std::move(id), std::move(data), p, now_locked()});
    update_backpressure_locked();
    return EnqueueResult::Ok;
  }

  std::vector<Item> dequeue_batch(size_t max_count) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Item> out;
    out.reserve(std::min(max_count, total_locked()));
    if (cfg_.aging_s > 0.0) {
      while (out.size() < max_count) {
        int c = pick_aged_locked();
        if (c < 0) break;
        out.push_back(std::move(q_[c].front()));
        q_[c].pop_front();
      }
    } else {
      for (int c = 2; c >= 0 && out.size() < max_count; --c) {
        while (out.size() < max_count && !q_[c].empty()) {
          out.push_back(std::move(q_[c].front()));
          q_[c].pop_front();
        }
      }
    }
    update_backpressure_locked();
    return out;
  }

  std::optional<Item> dequeue_one() {
    std::lock_guard<std::mutex> g(mu_);
    std::optional<Item> r;
    int c = cfg_.aging_s > 0.0 ? pick_aged_locked() : pick_strict_locked();
    if (c >= 0) {
      r = std::move(q_[c].front());
      q_[c].pop_front();
    }
    update_backpressure_locked();
    return r;
  }

  // Peek the id of the request dequeue_one() would return (no mutation).
  std::optional<std::string> peek_id() const {
    std::lock_guard<std::mutex> g(mu_);
    int c = cfg_.aging_s > 0.0 ? pick_aged_locked() : pick_strict_locked();
    if (c < 0) return std::nullopt;
    return q_[c].front().id;
  }

  std::vector<Item> remove_expired() {
    std::lock_guard<std::mutex> g(mu_);
    const double t = now_locked();
    std::vector<Item> expired;
    for (int c = 2; c >= 0; --c) {  // High, Normal, Low (queue.rs:222-224)
      std::deque<Item> keep;
      for (auto& it : q_[c]) {
        if (t - it.enqueued_at > cfg_.request_timeout_s)
          expired.push_back(std::move(it));
        else
          keep.push_back(std::move(it));
      }
      q_[c].swap(keep);
    }
    update_backpressure_locked();
    return expired;
  }

  // Remove one request by id (design.md:215). nullopt == NotFound.
  std::optional<Item> cancel(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    for (int c = 2; c >= 0; --c) {
      for (auto it = q_[c].begin(); it != q_[c].end(); ++it) {
        if (it->id == id) {
          Item r = std::move(*it);
          q_[c].erase(it);
          update_backpressure_locked();
          return r;
        }
      }
    }
    return std::nullopt;
  }

  // Drain everything (shutdown / model swap).
  std::vector<Item> drain() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Item> out;
    for (int c = 2; c >= 0; --c) {
      for (auto& it : q_[c]) out.push_back(std::move(it));
      q_[c].clear();
    }
    update_backpressure_locked();
    return out;
  }

  // ---- queries ---------------------------------------------------------------
  QueueDepth queue_depth() const {
    std::lock_guard<std::mutex> g(mu_);
    QueueDepth d;
    d.high = q_[2].size();
    d.normal = q_[1].size();
    d.low = q_[0].size();
    d.total = d.high + d.normal + d.low;
    return d;
  }
  bool is_accepting() const {
    std::lock_guard<std::mutex> g(mu_);
    return !backpressure_;
  }
  size_t total_depth() const {
    std::lock_guard<std::mutex> g(mu_);
    return total_locked();
  }
  bool is_empty() const {
    std::lock_guard<std::mutex> g(mu_);
    return total_locked() == 0;
  }
  QueueConfig config() const {
    std::lock_guard<std::mutex> g(mu_);
    return cfg_;
  }
  // Hot-reload of thresholds (Req 10.5). Backpressure is re-evaluated.
  void set_config(const QueueConfig& c) {
    std::lock_guard<std::mutex> g(mu_);
    cfg_ = c;
    update_backpressure_locked();
  }
  // Oldest wait (seconds) in the queue, 0 if empty.
  double oldest_wait_s() const {
    std::lock_guard<std::mutex> g(mu_);
    double t = now_locked(), w = 0.0;
    for (int c = 0; c < 3; ++c)
      if (!q_[c].empty()) w = std::max(w, t - q_[c].front().enqueued_at);
    return w;
  }

 private:
  static int idx(Priority p) { return static_cast<int>(p); }
  size_t total_locked() const { return q_[0].size() + q_[1].size() + q_[2].size(); }
  double now_locked() const { return manual_ ? manual_t_ : steady_now_s(); }

  int pick_strict_locked() const {
    for (int c = 2; c >= 0; --c)
      if (!q_[c].empty()) return c;
    return -1;
  }
  // Effective class = base + floor(wait / aging_s), capped at High. Ties go
  // to the higher base class, then to the older request.
  int pick_aged_locked() const {
    const double t = now_locked();
    int best = -1;
    double best_eff = -1.0;
    for (int c = 2; c >= 0; --c) {
      if (q_[c].empty()) continue;
      double age = t - q_[c].front().enqueued_at;
      double eff = std::min(2.0, c + std::floor(age / cfg_.aging_s));
      if (eff > best_eff) {  // strict: ties keep the higher base class
        best = c;
        best_eff = eff;
      }
    }
    return best;
  }

  void update_backpressure_locked() {
    const size_t total = total_locked();
    if (backpressure_) {
      if (total < cfg_.low_watermark) backpressure_ = false;
    } else {
      if (total > cfg_.high_watermark) backpressure_ = true;
    }
  }

  QueueConfig cfg_;
  std::deque<Item> q_[3];  // index = Priority value: 0 Low, 1 Normal, 2 High
  bool backpressure_ = false;
  bool manual_ = false;
  double manual_t_ = 0.0;
  mutable std::mutex mu_;
};

}  // namespace xgs
