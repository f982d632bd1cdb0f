// Replica selection for the data-parallel router.
//
// Realises the reference's spec'd Adaptive Scheduler / Load Balancer
// (Req 6, requirements.md:88-98; design.md:269-308; Properties 16-19):
//   * strategies RoundRobin | LeastLoaded | MemoryAware (design.md:276-280),
//     switchable at run time (set_strategy, design.md:306);
//   * LeastLoaded picks a healthy worker with the minimum active load
//     (Property 16; ties -> lowest id);
//   * MemoryAware picks a healthy worker whose available memory >= the
//     request's estimate (Property 17), preferring the most free memory;
//     none -> -1 (reject);
//   * unhealthy workers are never selected (Property 18) and are eligible again
//     once marked healthy (Property 19).
// "Memory" for a replica = free KV-cache bytes in HBM reported by its engine.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <vector>

namespace xgs {

enum class Strategy : uint8_t { RoundRobin = 0, LeastLoaded = 1, MemoryAware = 2 };

struct WorkerStatus {
  int id = 0;
  int64_t active = 0;            // in-flight requests (active_batches)
  int64_t memory_used = 0;       // bytes
  int64_t memory_available = 0;  // bytes
  bool healthy = true;
  double last_health_check = 0.0;
};

class ReplicaRouter {
 public:
  explicit ReplicaRouter(Strategy s = Strategy::LeastLoaded) : strategy_(s) {}
  void register_worker(int id, int64_t memory_available);
  bool unregister_worker(int id);
  void set_strategy(Strategy s);
  Strategy strategy() const;
  void update(int id, int64_t active, int64_t memory_used, int64_t memory_available, double now);
  void set_healthy(int id, bool healthy, double now);
  void add_active(int id, int64_t delta);
  int select(int64_t estimated_memory);
  std::vector<WorkerStatus> statuses() const;
  int num_healthy() const;

 private:
  mutable std::mutex mu_;
  Strategy strategy_;
  std::map<int, WorkerStatus> workers_;
  uint64_t rr_ = 0;
};

}  // namespace xgs
