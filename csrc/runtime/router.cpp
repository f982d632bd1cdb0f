#include "router.h"

namespace xgs {

void ReplicaRouter::register_worker(int id, int64_t memory_available) {
  std::lock_guard<std::mutex> g(mu_);
  WorkerStatus w;
  w.id = id;
  w.memory_available = memory_available;
  workers_[id] = w;
}

bool ReplicaRouter::unregister_worker(int id) {
  std::lock_guard<std::mutex> g(mu_);
  return workers_.erase(id) > 0;
}

void ReplicaRouter::set_strategy(Strategy s) {
  std::lock_guard<std::mutex> g(mu_);
  strategy_ = s;
}

Strategy ReplicaRouter::strategy() const {
  std::lock_guard<std::mutex> g(mu_);
  return strategy_;
}

void ReplicaRouter::update(int id, int64_t active, int64_t memory_used, int64_t memory_available,
                           double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(id);
  if (it == workers_.end()) return;
  it->second.active = active;
  it->second.memory_used = memory_used;
  it->second.memory_available = memory_available;
  it->second.last_health_check = now;
}

void ReplicaRouter::set_healthy(int id, bool healthy, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(id);
  if (it == workers_.end()) return;
  it->second.healthy = healthy;
  it->second.last_health_check = now;
}

void ReplicaRouter::add_active(int id, int64_t delta) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(id);
  if (it != workers_.end()) it->second.active += delta;
}

int ReplicaRouter::select(int64_t est) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<const WorkerStatus*> ok;
  for (const auto& kv : workers_)
    if (kv.second.healthy) ok.push_back(&kv.second);
  if (ok.empty()) return -1;
  switch (strategy_) {
    case Strategy::RoundRobin:
      return ok[rr_++ % ok.size()]->id;
    case Strategy::LeastLoaded: {
      const WorkerStatus* best = ok[0];
      for (const auto* w : ok)
        if (w->active < best->active) best = w;
      return best->id;
    }
    case Strategy::MemoryAware: {
      const WorkerStatus* best = nullptr;
      for (const auto* w : ok)
        if (w->memory_available >= est &&
            (!best || w->memory_available > best->memory_available ||
             (w->memory_available == best->memory_available && w->active < best->active)))
          best = w;
      return best ? best->id : -1;
    }
  }
  return -1;
}

std::vector<WorkerStatus> ReplicaRouter::statuses() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<WorkerStatus> out;
  for (const auto& kv : workers_) out.push_back(kv.second);
  return out;
}

int ReplicaRouter::num_healthy() const {
  std::lock_guard<std::mutex> g(mu_);
  int n = 0;
  for (const auto& kv : workers_) n += kv.second.healthy ? 1 : 0;
  return n;
}

}  // namespace xgs
