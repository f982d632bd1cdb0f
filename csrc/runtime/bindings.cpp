// pybind11 bindings for the native runtime core (module xgserve._runtime).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kv_blocks.h"
#include "queue.h"
#include "router.h"
#include "scheduler.h"
#include "shm_channel.h"
#include "validator.h"

namespace py = pybind11;
using namespace xgs;

namespace {

using PyQueue = PriorityQueueManager<py::object>;

py::tuple item_tuple(QueuedRequest<py::object>& it) {
  return py::make_tuple(it.id, it.data, static_cast<int>(it.priority), it.enqueued_at);
}

py::object vres(const ValidationResult& r) {
  if (r.ok()) return py::none();
  py::dict d;
  static const char* kinds[] = {"ok", "invalid_json", "missing_field", "token_limit_exceeded",
                                "invalid_parameter", "empty_prompt"};
  d["kind"] = kinds[static_cast<int>(r.kind)];
  d["message"] = r.message;
  d["field"] = r.field;
  d["reason"] = r.reason;
  d["actual"] = r.actual;
  d["limit"] = r.limit;
  return d;
}

template <typename T>
py::array_t<T> arr(const std::vector<T>& v) {
  py::array_t<T> a(v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

py::dict plan_dict(const StepPlan& p) {
  py::dict d;
  d["num_seqs"] = p.num_seqs;
  d["num_decodes"] = p.num_decodes;
  d["num_tokens"] = p.num_tokens;
  d["num_sample"] = p.num_sample;
  d["max_q_len"] = p.max_q_len;
  d["max_seq_len"] = p.max_seq_len;
  d["bt_width"] = p.bt_width;
  d["seq_ids"] = arr(p.seq_ids);
  d["slots"] = arr(p.slots);
  d["q_lens"] = arr(p.q_lens);
  d["ctx_lens"] = arr(p.ctx_lens);
  d["seq_lens"] = arr(p.seq_lens);
  d["is_prefill"] = arr(p.is_prefill);
  d["do_sample"] = arr(p.do_sample);
  d["is_embed"] = arr(p.is_embed);
  d["input_ids"] = arr(p.input_ids);
  d["positions"] = arr(p.positions);
  d["slot_mapping"] = arr(p.slot_mapping);
  d["query_start_loc"] = arr(p.query_start_loc);
  d["block_tables"] = arr(p.block_tables);
  d["logits_indices"] = arr(p.logits_indices);
  d["sample_seq_index"] = arr(p.sample_seq_index);
  d["preempted"] = arr(p.preempted);
  return d;
}

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "xgserve native runtime core: queue, validator, KV pages, prefix cache, step scheduler, router";

  // ---------------------------------------------------------------- queue
  py::class_<QueueConfig>(m, "QueueConfig")
      .def(py::init<>())
      .def_readwrite("high_watermark", &QueueConfig::high_watermark)
      .def_readwrite("low_watermark", &QueueConfig::low_watermark)
      .def_readwrite("request_timeout_s", &QueueConfig::request_timeout_s)
      .def_readwrite("max_queue_size", &QueueConfig::max_queue_size)
      .def_readwrite("aging_s", &QueueConfig::aging_s);

  py::class_<PyQueue>(m, "PriorityQueueManager")
      .def(py::init<QueueConfig>(), py::arg("config") = QueueConfig())
      .def("enqueue",
           [](PyQueue& q, std::string id, py::object data, int prio) {
             if (prio < 0 || prio > 2) throw py::value_error("priority must be 0..2");
             return q.enqueue(std::move(id), std::move(data), static_cast<Priority>(prio)) ==
                    EnqueueResult::Ok;
           })
      .def("dequeue_batch",
           [](PyQueue& q, size_t n) {
             auto v = q.dequeue_batch(n);
             py::list out;
             for (auto& it : v) out.append(item_tuple(it));
             return out;
           })
      .def("dequeue_one",
           [](PyQueue& q) -> py::object {
             auto r = q.dequeue_one();
             if (!r) return py::none();
             return item_tuple(*r);
           })
      .def("peek_id", [](PyQueue& q) -> py::object {
        auto r = q.peek_id();
        if (!r) return py::none();
        return py::str(*r);
      })
      .def("remove_expired",
           [](PyQueue& q) {
             auto v = q.remove_expired();
             py::list out;
             for (auto& it : v) out.append(item_tuple(it));
             return out;
           })
      .def("cancel",
           [](PyQueue& q, const std::string& id) -> py::object {
             auto r = q.cancel(id);
             if (!r) return py::none();
             return item_tuple(*r);
           })
      .def("drain",
           [](PyQueue& q) {
             auto v = q.drain();
             py::list out;
             for (auto& it : v) out.append(item_tuple(it));
             return out;
           })
      .def("queue_depth",
           [](const PyQueue& q) {
             auto d = q.queue_depth();
             return py::make_tuple(d.high, d.normal, d.low, d.total);
           })
      .def("is_accepting", &PyQueue::is_accepting)
      .def("total_depth", &PyQueue::total_depth)
      .def("is_empty", &PyQueue::is_empty)
      .def("config", &PyQueue::config)
      .def("set_config", &PyQueue::set_config)
      .def("oldest_wait_s", &PyQueue::oldest_wait_s)
      .def("set_manual_clock", &PyQueue::set_manual_clock, py::arg("on"), py::arg("t") = 0.0)
      .def("advance_clock", &PyQueue::advance_clock)
      .def("now", &PyQueue::now);

  // ---------------------------------------------------------------- validator
  py::class_<ValidatorConfig>(m, "ValidatorConfig")
      .def(py::init<>())
      .def_readwrite("max_context_tokens", &ValidatorConfig::max_context_tokens)
      .def_readwrite("max_output_tokens", &ValidatorConfig::max_output_tokens)
      .def_readwrite("min_temperature", &ValidatorConfig::min_temperature)
      .def_readwrite("max_temperature", &ValidatorConfig::max_temperature)
      .def_readwrite("min_top_p", &ValidatorConfig::min_top_p)
      .def_readwrite("max_top_p", &ValidatorConfig::max_top_p)
      .def_readwrite("reject_nan", &ValidatorConfig::reject_nan);

  py::class_<RequestValidator>(m, "RequestValidator")
      .def(py::init<ValidatorConfig>(), py::arg("config") = ValidatorConfig())
      .def("token_count", &RequestValidator::token_count)
      .def("validate_generate",
           [](const RequestValidator& v, const std::string& p, size_t mt, float t, float tp) {
             return vres(v.validate_generate(p, mt, t, tp));
           })
      .def("validate_chat",
           [](const RequestValidator& v, const std::vector<std::string>& c, size_t mt, float t,
              float tp) { return vres(v.validate_chat(c, mt, t, tp)); })
      .def("validate_embeddings",
           [](const RequestValidator& v, const std::vector<std::string>& in) {
             return vres(v.validate_embeddings(in));
           })
      .def("config", &RequestValidator::config)
      .def("set_config", &RequestValidator::set_config);

  m.def("rust_f32_display", &rust_f32_display);
  m.def("is_blank_utf8", &is_blank_utf8);

  // ---------------------------------------------------------------- KV pages
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int>())
      .def("alloc", &BlockAllocator::alloc)
      .def("incref", &BlockAllocator::incref)
      .def("decref", &BlockAllocator::decref)
      .def("refcount", &BlockAllocator::refcount)
      .def("num_free", &BlockAllocator::num_free)
      .def("num_blocks", &BlockAllocator::num_blocks);

  py::class_<PrefixCache>(m, "PrefixCache")
      .def(py::init([](BlockAllocator& a, int bs, int maxb) { return new PrefixCache(&a, bs, maxb); }),
           py::keep_alive<1, 2>())
      .def("match",
           [](PrefixCache& c, const std::vector<int32_t>& t, int max_tokens, bool count) {
             return c.match(t.data(), static_cast<int>(t.size()), max_tokens, count);
           },
           py::arg("tokens"), py::arg("max_tokens"), py::arg("count") = true)
      .def("insert",
           [](PrefixCache& c, const std::vector<int32_t>& t, const std::vector<int>& b) {
             return c.insert(t.data(), static_cast<int>(t.size()), b.data(), static_cast<int>(b.size()));
           })
      .def("evict", &PrefixCache::evict)
      .def("evictable", &PrefixCache::evictable)
      .def("clear", &PrefixCache::clear)
      .def("reset_stats", &PrefixCache::reset_stats)
      .def("last_access_of", &PrefixCache::last_access_of)
      .def("tick", &PrefixCache::tick)
      .def("max_cached_blocks", &PrefixCache::max_cached_blocks)
      .def("set_max_cached_blocks", &PrefixCache::set_max_cached_blocks)
      .def("stats", [](const PrefixCache& c) {
        const auto& s = c.stats();
        py::dict d;
        d["entries"] = s.entries;
        d["hit_tokens"] = s.hit_tokens;
        d["miss_tokens"] = s.miss_tokens;
        d["hit_count"] = s.hit_count;
        d["miss_count"] = s.miss_count;
        d["eviction_count"] = s.eviction_count;
        return d;
      });

  // ---------------------------------------------------------------- scheduler
  py::class_<SchedulerConfig>(m, "SchedulerConfig")
      .def(py::init<>())
      .def_readwrite("block_size", &SchedulerConfig::block_size)
      .def_readwrite("num_blocks", &SchedulerConfig::num_blocks)
      .def_readwrite("max_num_seqs", &SchedulerConfig::max_num_seqs)
      .def_readwrite("max_num_batched_tokens", &SchedulerConfig::max_num_batched_tokens)
      .def_readwrite("max_model_len", &SchedulerConfig::max_model_len)
      .def_readwrite("enable_prefix_cache", &SchedulerConfig::enable_prefix_cache)
      .def_readwrite("chunked_prefill", &SchedulerConfig::chunked_prefill)
      .def_readwrite("cache_threshold", &SchedulerConfig::cache_threshold)
      .def_readwrite("admit_watermark", &SchedulerConfig::admit_watermark)
      .def_readwrite("max_prefill_seqs", &SchedulerConfig::max_prefill_seqs)
      .def_readwrite("decode_prefill_cap", &SchedulerConfig::decode_prefill_cap)
      .def_readwrite("decode_prefill_seqs", &SchedulerConfig::decode_prefill_seqs)
      .def_readwrite("coalesce_prompts", &SchedulerConfig::coalesce_prompts)
      .def_readwrite("coalesce_max_wait", &SchedulerConfig::coalesce_max_wait)
      .def_readwrite("lookahead_mixed", &SchedulerConfig::lookahead_mixed)
      .def_readwrite("early_release", &SchedulerConfig::early_release)
      .def_readwrite("eos_ids", &SchedulerConfig::eos_ids);

  py::class_<StepScheduler>(m, "StepScheduler")
      .def(py::init<const SchedulerConfig&>())
      .def("add", &StepScheduler::add, py::arg("id"), py::arg("prompt"), py::arg("max_tokens"),
           py::arg("priority") = 1, py::arg("ignore_eos") = false, py::arg("embed") = false,
           py::arg("stop_seqs") = std::vector<std::vector<int32_t>>{}, py::arg("min_tokens") = 0)
      .def("abort", &StepScheduler::abort)
      .def("set_draft", &StepScheduler::set_draft)
      .def("schedule", [](StepScheduler& s) { return plan_dict(s.schedule()); })
      .def("update",
           [](StepScheduler& s, py::array_t<int32_t, py::array::c_style | py::array::forcecast> tok,
              py::array_t<int32_t, py::array::c_style | py::array::forcecast> cnt) {
             auto fin = s.update(tok.data(), cnt.data(), static_cast<int>(cnt.size()));
             py::list out;
             for (const auto& f : fin)
               out.append(py::make_tuple(f.id, static_cast<int>(f.reason), f.prompt_len, f.num_generated,
                                         f.num_cached));
             return out;
           })
      .def("lookahead", &StepScheduler::lookahead, py::arg("across_length_finish") = false)
      .def("commit",
           [](StepScheduler& s, py::array_t<int32_t, py::array::c_style | py::array::forcecast> tok) {
             auto fin = s.commit(tok.data(), static_cast<int>(tok.size()));
             py::list out;
             for (const auto& f : fin)
               out.append(py::make_tuple(f.id, static_cast<int>(f.reason), f.prompt_len, f.num_generated,
                                         f.num_cached));
             return out;
           })
      .def("num_inflight", &StepScheduler::num_inflight)
      .def("num_waiting", &StepScheduler::num_waiting)
      .def("num_running", &StepScheduler::num_running)
      .def("has_work", &StepScheduler::has_work)
      .def("num_free_blocks", &StepScheduler::num_free_blocks)
      .def("num_blocks", &StepScheduler::num_blocks)
      .def("num_used_blocks", &StepScheduler::num_used_blocks)
      .def("num_evictable_blocks", &StepScheduler::num_evictable_blocks)
      .def("total_preemptions", &StepScheduler::total_preemptions)
      .def("set_limits", &StepScheduler::set_limits)
      .def("set_decode_prefill", &StepScheduler::set_decode_prefill)
      .def("clear_prefix_cache", &StepScheduler::clear_prefix_cache)
      .def("cached_prefix", &StepScheduler::cached_prefix)
      .def("install_prefix", &StepScheduler::install_prefix)
      .def("seq_info",
           [](const StepScheduler& s, int64_t id) -> py::object {
             const Sequence* q = s.get(id);
             if (!q) return py::none();
             py::dict d;
             d["tokens"] = q->tokens;
             d["prompt_len"] = q->prompt_len;
             d["num_computed"] = q->num_computed;
             d["num_cached"] = q->num_cached;
             d["blocks"] = q->blocks;
             d["status"] = static_cast<int>(q->status);
             d["slot"] = q->slot;
             d["num_preemptions"] = q->num_preemptions;
             return d;
           })
      .def("cache_stats", [](StepScheduler& s) {
        const auto& st = s.cache().stats();
        py::dict d;
        d["entries"] = st.entries;
        d["hit_tokens"] = st.hit_tokens;
        d["miss_tokens"] = st.miss_tokens;
        d["hit_count"] = st.hit_count;
        d["miss_count"] = st.miss_count;
        d["eviction_count"] = st.eviction_count;
        return d;
      });

  // ---------------------------------------------------------------- router
  py::enum_<Strategy>(m, "Strategy")
      .value("RoundRobin", Strategy::RoundRobin)
      .value("LeastLoaded", Strategy::LeastLoaded)
      .value("MemoryAware", Strategy::MemoryAware);

  py::class_<ReplicaRouter>(m, "ReplicaRouter")
      .def(py::init<Strategy>(), py::arg("strategy") = Strategy::LeastLoaded)
      .def("register_worker", &ReplicaRouter::register_worker)
      .def("unregister_worker", &ReplicaRouter::unregister_worker)
      .def("set_strategy", &ReplicaRouter::set_strategy)
      .def("strategy", &ReplicaRouter::strategy)
      .def("update", &ReplicaRouter::update)
      .def("set_healthy", &ReplicaRouter::set_healthy)
      .def("add_active", &ReplicaRouter::add_active)
      .def("select", &ReplicaRouter::select, py::arg("estimated_memory") = 0)
      .def("num_healthy", &ReplicaRouter::num_healthy)
      .def("statuses", [](const ReplicaRouter& r) {
        py::list out;
        for (const auto& w : r.statuses()) {
          py::dict d;
          d["id"] = w.id;
          d["active"] = w.active;
          d["memory_used"] = w.memory_used;
          d["memory_available"] = w.memory_available;
          d["healthy"] = w.healthy;
          d["last_health_check"] = w.last_health_check;
          out.append(d);
        }
        return out;
      });

  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, uint64_t, int, bool>(), py::arg("name"),
           py::arg("capacity"), py::arg("num_readers"), py::arg("create"))
      .def("publish",
           [](ShmChannel& c, py::bytes b, double timeout_s) {
             std::string_view v = b;
             py::gil_scoped_release nogil;
             return c.publish(v.data(), v.size(), timeout_s);
           },
           py::arg("data"), py::arg("timeout_s") = -1.0)
      .def("receive",
           [](ShmChannel& c, int rank, double timeout_s) -> py::object {
             int64_t n;
             {
               py::gil_scoped_release nogil;
               n = c.wait_message(rank, timeout_s);
             }
             if (n < 0) return py::none();
             PyObject* b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)n);
             if (!b) throw py::error_already_set();
             c.consume(rank, PyBytes_AS_STRING(b));
             return py::reinterpret_steal<py::object>(b);
           },
           py::arg("rank"), py::arg("timeout_s") = -1.0)
      .def_property_readonly("capacity", &ShmChannel::capacity)
      .def_property_readonly("seq", &ShmChannel::seq)
      .def_property_readonly("name", &ShmChannel::name)
      .def("unlink", &ShmChannel::unlink);
}
