// Native unit tests for the C++ runtime core (SURVEY.md 4.3 "Unit (C++)" and
// 5 "Race detection / sanitizers"): plain asserts, no framework, no GPU.
//
// Built three ways by tests/test_native_runtime.py: plain -O1, with
// -fsanitize=address,undefined, and with -fsanitize=thread. The concurrent
// sections (queue producers/consumers, router updates vs selects, the shm plan
// channel with reader threads) are what ThreadSanitizer checks.
//
//   g++ -std=c++17 -O1 -g -Icsrc/runtime csrc/tests/test_runtime.cpp \
//       csrc/runtime/{kv_blocks,scheduler,router,validator,shm_channel}.cpp -o /tmp/t -lpthread -lrt
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "kv_blocks.h"
#include "queue.h"
#include "router.h"
#include "scheduler.h"
#include "shm_channel.h"
#include "validator.h"

using namespace xgs;

static int g_checks = 0;
#define CHECK(cond)                                                                      \
  do {                                                                                   \
    ++g_checks;                                                                          \
    if (!(cond)) {                                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      std::abort();                                                                      \
    }                                                                                    \
  } while (0)

// ---------------------------------------------------------------- queue
static void test_queue_hysteresis_and_timeouts() {
  QueueConfig c;  // 1000 / 500 / 2000, 30 s
  PriorityQueueManager<int> q(c);
  q.set_manual_clock(true, 0.0);
  // queue.rs:235-249: active iff total > high (strict), inactive iff total < low (strict)
  for (int i = 0; i < 1000; ++i) CHECK(q.enqueue("r" + std::to_string(i), i, Priority::Normal) == EnqueueResult::Ok);
  CHECK(q.is_accepting());  // exactly at the high watermark
  CHECK(q.enqueue("r1000", 0, Priority::Normal) == EnqueueResult::Ok);
  CHECK(!q.is_accepting());
  CHECK(q.enqueue("x", 0, Priority::High) == EnqueueResult::Full);
  q.dequeue_batch(501);
  CHECK(q.total_depth() == 500 && !q.is_accepting());  // 500 is not < 500
  q.dequeue_batch(1);
  CHECK(q.total_depth() == 499 && q.is_accepting());
  // strict priority + FIFO inside a class
  PriorityQueueManager<int> p(c);
  p.set_manual_clock(true, 0.0);
  p.enqueue("l", 0, Priority::Low);
  p.enqueue("n1", 1, Priority::Normal);
  p.enqueue("h", 2, Priority::High);
  p.enqueue("n2", 3, Priority::Normal);
  auto b = p.dequeue_batch(4);
  CHECK(b.size() == 4 && b[0].id == "h" && b[1].id == "n1" && b[2].id == "n2" && b[3].id == "l");
  // timeouts with the injected clock (no sleeping)
  p.enqueue("old", 0, Priority::Normal);
  p.advance_clock(20.0);
  p.enqueue("young", 1, Priority::Normal);
  p.advance_clock(10.5);
  auto ex = p.remove_expired();
  CHECK(ex.size() == 1 && ex[0].id == "old");
  CHECK(p.total_depth() == 1 && p.peek_id().value() == "young");
  CHECK(p.cancel("young").has_value() && p.is_empty());
}

static void test_queue_concurrent() {
  QueueConfig c;
  c.high_watermark = 1 << 20;
  c.low_watermark = 1 << 19;
  c.max_queue_size = 1 << 21;
  PriorityQueueManager<int> q(c);
  constexpr int kProducers = 4, kPer = 5000;
  std::atomic<int> consumed{0};
  std::atomic<bool> done{false};
  std::vector<std::thread> th;
  for (int t = 0; t < kProducers; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < kPer; ++i)
        q.enqueue("p" + std::to_string(t) + "_" + std::to_string(i), i, static_cast<Priority>(i % 3));
    });
  std::thread cons([&] {
    while (!done.load() || !q.is_empty()) {
      consumed += static_cast<int>(q.dequeue_batch(64).size());
      (void)q.queue_depth();
      (void)q.remove_expired();
    }
  });
  for (auto& t : th) t.join();
  done = true;
  cons.join();
  CHECK(consumed.load() == kProducers * kPer);
}

// ---------------------------------------------------------------- validator
static void test_validator() {
  RequestValidator v;
  CHECK(v.token_count("") == 0 && v.token_count("abcd") == 1 && v.token_count("abcde") == 2);
  CHECK(v.validate_generate("hello", 16, 1.0f, 1.0f).ok());
  CHECK(v.validate_generate("   ", 16, 1.0f, 1.0f).kind == ValidationKind::EmptyPrompt);
  CHECK(v.validate_generate("hi", 16, 2.5f, 1.0f).kind == ValidationKind::InvalidParameter);
  CHECK(v.validate_generate("hi", 16, 1.0f, 1.5f).kind == ValidationKind::InvalidParameter);
  CHECK(v.validate_generate(std::string(40000, 'a'), 16, 1.0f, 1.0f).kind == ValidationKind::TokenLimitExceeded);
}

// ---------------------------------------------------------------- KV pages + prefix cache
static void test_blocks_and_prefix_cache() {
  BlockAllocator a(8);
  std::vector<int> got;
  for (int i = 0; i < 8; ++i) got.push_back(a.alloc());
  CHECK(a.alloc() == -1 && a.num_free() == 0);
  a.incref(got[0]);
  a.decref(got[0]);
  CHECK(a.refcount(got[0]) == 1);
  for (int b : got) a.decref(b);
  CHECK(a.num_free() == 8);

  BlockAllocator a2(16);
  PrefixCache pc(&a2, 4, 16);
  std::vector<int32_t> toks = {1, 2, 3, 4, 5, 6, 7, 8, 9};
  int b0 = a2.alloc(), b1 = a2.alloc();
  int blocks[2] = {b0, b1};
  pc.insert(toks.data(), 8, blocks, 2);
  a2.decref(b0);
  a2.decref(b1);  // the cache holds the only references now
  auto m = pc.match(toks.data(), 9, 8);
  CHECK(m.size() == 2 && m[0] == b0 && m[1] == b1);
  std::vector<int32_t> other = {1, 2, 3, 4, 9, 9, 9, 9};
  CHECK(pc.match(other.data(), 8, 8).size() == 1);
  CHECK(pc.evict(16) == 2 && a2.num_free() == 16);
}

// ---------------------------------------------------------------- step scheduler
static void test_scheduler_decode_prefill_preempt() {
  SchedulerConfig c;
  c.block_size = 4;
  c.num_blocks = 12;
  c.max_num_seqs = 4;
  c.max_num_batched_tokens = 16;
  c.max_model_len = 64;
  c.eos_ids = {2};
  StepScheduler s(c);
  std::vector<int32_t> p1(10, 7), p2(6, 9);
  CHECK(s.add(1, p1, 8, 1, true, false, {}));
  CHECK(s.add(2, p2, 8, 1, true, false, {}));
  CHECK(!s.add(1, p1, 8, 1, true, false, {}));  // duplicate id
  const StepPlan& a = s.schedule();
  CHECK(a.num_seqs == 2 && a.num_tokens == 16 && a.num_decodes == 0);  // 10 + 6 (budget 16)
  CHECK(a.num_sample == 2);
  int32_t toks[2] = {11, 12}, cnt[2] = {1, 1};
  CHECK(s.update(toks, cnt, 2).empty());
  const StepPlan& b = s.schedule();
  CHECK(b.num_decodes == 2 && b.num_tokens == 2);
  CHECK(b.input_ids[0] == 11 && b.input_ids[1] == 12);
  // run to completion: max_tokens 8 -> finished with Length
  int finished = 0;
  for (int step = 0; step < 20 && s.has_work(); ++step) {
    const StepPlan& p = s.schedule();
    std::vector<int32_t> t(p.num_sample, 5), k(p.num_sample, 1);
    finished += static_cast<int>(s.update(t.data(), k.data(), p.num_sample).size());
  }
  CHECK(finished == 2 && s.num_free_blocks() + s.num_evictable_blocks() == c.num_blocks);
  // preemption: 3 long prompts over a tiny pool
  SchedulerConfig c2 = c;
  c2.num_blocks = 6;
  c2.enable_prefix_cache = false;
  StepScheduler s2(c2);
  for (int i = 0; i < 3; ++i) CHECK(s2.add(10 + i, std::vector<int32_t>(7, 3 + i), 12, 1, true, false, {}));
  int done = 0;
  for (int step = 0; step < 200 && s2.has_work(); ++step) {
    const StepPlan& p = s2.schedule();
    std::vector<int32_t> t(p.num_sample, 4), k(p.num_sample, 1);
    done += static_cast<int>(s2.update(t.data(), k.data(), p.num_sample).size());
  }
  CHECK(done == 3 && s2.total_preemptions() > 0 && s2.num_free_blocks() == 6);
}

// ---------------------------------------------------------------- router (concurrent)
static void test_router_concurrent() {
  ReplicaRouter r(Strategy::LeastLoaded);
  for (int i = 0; i < 4; ++i) r.register_worker(i, 1 << 30);
  std::atomic<bool> stop{false};
  std::thread upd([&] {
    for (int it = 0; it < 20000; ++it) {
      int id = it % 4;
      r.update(id, it % 7, 1000, (1 << 30) - 1000, it * 1e-3);
      r.set_healthy(id, it % 13 != 0, it * 1e-3);
    }
    stop = true;
  });
  int picks = 0;
  while (!stop.load() || picks < 100) {
    int w = r.select(0);
    if (w >= 0) {
      r.add_active(w, 1);
      r.add_active(w, -1);
      ++picks;
    }
    (void)r.statuses();
  }
  upd.join();
  for (int i = 0; i < 4; ++i) r.set_healthy(i, true, 0.0);
  r.set_strategy(Strategy::RoundRobin);
  int a = r.select(0), b = r.select(0);
  CHECK(a >= 0 && b >= 0 && a != b && picks > 0);
  r.set_strategy(Strategy::MemoryAware);
  CHECK(r.select(int64_t(1) << 40) == -1);  // nobody has 1 TiB free
}

// ---------------------------------------------------------------- shm plan channel (threads)
static void test_shm_channel_threads() {
  const std::string name = "xgs_ut_" + std::to_string(getpid());
  ShmChannel w(name, 1 << 14, 3, true);
  constexpr int kMsgs = 3000;
  std::atomic<int> bad{0};
  std::vector<std::thread> rd;
  for (int r = 0; r < 3; ++r)
    rd.emplace_back([&, r] {
      ShmChannel c(name, 0, 3, false);
      std::vector<char> buf(c.capacity());
      for (int i = 0; i < kMsgs; ++i) {
        int64_t n = c.wait_message(r, 10.0);
        if (n < 0) { ++bad; return; }
        c.consume(r, buf.data());
        int v = 0;
        std::memcpy(&v, buf.data(), sizeof v);
        if (v != i || n != static_cast<int64_t>(sizeof(int) + (i % 100))) ++bad;
      }
    });
  std::vector<char> msg(sizeof(int) + 100);
  for (int i = 0; i < kMsgs; ++i) {
    std::memcpy(msg.data(), &i, sizeof i);
    CHECK(w.publish(msg.data(), sizeof(int) + (i % 100), 10.0));
  }
  for (auto& t : rd) t.join();
  CHECK(bad.load() == 0 && w.seq() == kMsgs);
}

int main() {
  test_queue_hysteresis_and_timeouts();
  test_queue_concurrent();
  test_validator();
  test_blocks_and_prefix_cache();
  test_scheduler_decode_prefill_preempt();
  test_router_concurrent();
  test_shm_channel_threads();
  std::printf("runtime unit tests: %d checks passed\n", g_checks);
  return 0;
}
