// Continuous-batching step scheduler (iteration-level batching over paged KV).
//
// Realises the reference's spec'd Request Batcher + worker-side batching
// (Req 2, requirements.md:39-49; design.md:227-267) the MI355X way: there is no
// padded static batch. Every engine step the scheduler packs
//   [decode tokens of running sequences] ++ [prefill chunks]
// under a token budget (max_num_batched_tokens) and a sequence cap
// (max_num_seqs), allocating KV pages as it goes. Ragged attention kernels
// consume the packed layout directly, so padding overhead is always zero.
//
// Responsibilities:
//   * admission from the engine-local waiting list (priority, then arrival),
//     prefix-cache matching (PrefixCache), chunked prefill;
//   * page allocation; on exhaustion: evict prefix cache, then preempt the
//     lowest-priority / newest running sequence (recompute mode: its computed
//     full pages are first published to the prefix cache, so re-admission is
//     mostly a cache hit);
//   * building the step's flat metadata (token ids, positions, slot mapping,
//     block tables, query_start_loc, logits indices);
//   * applying sampled tokens, stop checks (EOS, token stop-sequences,
//     max_tokens, max_model_len) and releasing finished sequences;
//   * speculative decoding: a decode sequence may carry draft tokens, scheduled
//     as q_len = 1 + len(draft); update() appends the accepted prefix + bonus.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <unordered_map>
#include <vector>

#include "kv_blocks.h"

namespace xgs {

enum class SeqStatus : uint8_t { Waiting = 0, Running = 1, Finished = 2 };
enum class SeqFinish : uint8_t { None = 0, Stop = 1, Length = 2, StopSequence = 3, Aborted = 4, Embedded = 5 };

struct SchedulerConfig {
  int block_size = 16;
  int num_blocks = 1024;
  int max_num_seqs = 256;
  int max_num_batched_tokens = 8192;
  int max_model_len = 8192;
  bool enable_prefix_cache = true;
  bool chunked_prefill = true;
  float cache_threshold = 0.8f;   // max share of the pool the prefix cache may hold
  float admit_watermark = 0.01f;  // keep this share of pages free when admitting
  int max_prefill_seqs = 1 << 30; // cap on prefill sequences per step
  // cap on prefill tokens in a step that also carries decode rows (0: no cap).
  // Stall-free batching: prompt chunks ride on the decode step's weight reads
  // instead of stalling every running stream behind one large prefill step.
  int decode_prefill_cap = 0;
  // cap on prefill sequences in a step that also carries decode rows (0: max_prefill_seqs
  // only). 1 keeps every stall-free mixed step at ONE prompt chunk (the runner's
  // mixed-step graphs take exactly that shape).
  int decode_prefill_seqs = 0;
  // Admission window for continuous batching (Req 2.1/2.2 batching window, applied to
  // prompt admission): while decode rows are running, new prompts are held until
  // coalesce_prompts of them are waiting or the oldest has been passed over by
  // coalesce_max_wait plans, then admitted together into one mixed step (one larger
  // prefill GEMM instead of several M ~ 575 ones). With no decode rows running a
  // prompt is admitted at once. coalesce_prompts <= 1: off (every prompt admitted
  // at the first plan that has room).
  int coalesce_prompts = 1;
  int coalesce_max_wait = 4;
  // lookahead() over prompt steps (1) or pure-decode plans only (0)
  int lookahead_mixed = 1;
  // a length-finishing row: released at lookahead() so the next plan can admit into
  // its slot (1), or the plan stays synchronous so a request that arrives when it
  // finishes is admitted in the very next step (0: the TTFT-preserving default)
  int early_release = 0;
  std::vector<int32_t> eos_ids;
};

struct Sequence {
  int64_t id = 0;
  int slot = -1;
  int priority = 1;
  int64_t arrival = 0;
  std::vector<int32_t> tokens;
  int prompt_len = 0;
  int num_computed = 0;
  int num_cached = 0;  // prefix-cache hit tokens at (first) admission
  int max_tokens = 256;
  int min_tokens = 0;
  bool ignore_eos = false;
  bool embed = false;  // prefill-only (embeddings endpoint)
  bool released_early = false;  // length-finishing row released at lookahead(); reported at commit()
  int wait_plans = 0;            // plans that passed this waiting prompt over (admission window)
  std::vector<std::vector<int32_t>> stop_seqs;
  std::vector<int> blocks;
  std::vector<int32_t> draft;  // speculative tokens for the next step
  SeqStatus status = SeqStatus::Waiting;
  SeqFinish finish = SeqFinish::None;
  int num_preemptions = 0;
  int num_generated() const { return static_cast<int>(tokens.size()) - prompt_len; }
};

struct StepPlan {
  int num_seqs = 0;
  int num_decodes = 0;   // the first num_decodes sequences have q_len == 1 (no draft)
  int num_tokens = 0;
  int num_sample = 0;
  int max_q_len = 0;
  int max_seq_len = 0;
  int bt_width = 0;
  std::vector<int64_t> seq_ids;
  std::vector<int32_t> slots, q_lens, ctx_lens, seq_lens;
  std::vector<uint8_t> is_prefill, do_sample, is_embed;
  std::vector<int32_t> input_ids, positions, slot_mapping, query_start_loc;
  std::vector<int32_t> block_tables;  // [num_seqs, bt_width]
  std::vector<int32_t> logits_indices, sample_seq_index;
  std::vector<int64_t> preempted;
};

struct FinishedSeq {
  int64_t id;
  SeqFinish reason;
  int prompt_len;
  int num_generated;
  int num_cached;
};

class StepScheduler {
 public:
  explicit StepScheduler(const SchedulerConfig& cfg);

  // returns false if the id is already known or the prompt is too long.
  bool add(int64_t id, const std::vector<int32_t>& prompt, int max_tokens, int priority,
           bool ignore_eos, bool embed, const std::vector<std::vector<int32_t>>& stop_seqs,
           int min_tokens = 0);
  bool abort(int64_t id);
  bool set_draft(int64_t id, const std::vector<int32_t>& draft);

  const StepPlan& schedule();
  // tokens: concatenated accepted tokens per sampled sequence; counts[i]: how
  // many belong to sampled sequence i (1 for plain decode). Returns finished.
  std::vector<FinishedSeq> update(const int32_t* tokens, const int32_t* counts, int num_sample);

  // Asynchronous scheduling (one step of lookahead): for a plan whose tokens are
  // still being sampled on the GPU, append a placeholder token (kPlaceholder) to
  // every sampled sequence (decode rows and prompts completing this step; prompt
  // chunks that do not complete just advance) so schedule() can plan the NEXT step
  // before this one finishes -- the runner substitutes the placeholders on the
  // device from this step's sampled-token buffer. commit() later resolves the
  // oldest lookahead plan with its real tokens (one per sampled row, sample order)
  // and runs the stop checks; a sequence that stopped there may already be in the
  // next plan, whose row for it is then ignored. A row that reaches its length
  // limit with this token is released at once (unless across_length_finish), so
  // the next plan can admit into its slot; commit() reports it. Returns false (and
  // does nothing) for verify / embedding plans.
  static constexpr int32_t kPlaceholder = -1;
  bool lookahead(bool across_length_finish = false);
  std::vector<FinishedSeq> commit(const int32_t* tokens, int num_sample);
  int num_inflight() const { return static_cast<int>(inflight_.size()); }

  // queries
  int num_waiting() const { return static_cast<int>(waiting_.size()); }
  int num_running() const { return static_cast<int>(running_.size()); }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  int num_free_blocks() const { return alloc_.num_free(); }
  int num_blocks() const { return alloc_.num_blocks(); }
  int num_used_blocks() const;
  int num_evictable_blocks() const { return cache_.evictable(); }
  const Sequence* get(int64_t id) const;
  const SchedulerConfig& config() const { return cfg_; }
  PrefixCache& cache() { return cache_; }
  BlockAllocator& allocator() { return alloc_; }
  int64_t total_preemptions() const { return total_preemptions_; }
  void set_limits(int max_num_seqs, int max_num_batched_tokens);
  // stall-free batching limits of decoding steps (SchedulerConfig::decode_prefill_*);
  // 0 lifts them
  void set_decode_prefill(int cap, int seqs) {
    cfg_.decode_prefill_cap = std::max(0, cap);
    cfg_.decode_prefill_seqs = std::max(0, seqs);
  }
  void clear_prefix_cache() { cache_.clear(); }
  // KV export/import (cache entry serialisation, design.md:400-401):
  // pages currently caching the page-aligned prefix of tokens (no stats, no incref)
  std::vector<int> cached_prefix(const std::vector<int32_t>& tokens);
  // make the first n_pages pages of tokens resident in the prefix cache; returns
  // {#pages that were already cached, page ids...}. Empty on allocation failure.
  std::vector<int> install_prefix(const std::vector<int32_t>& tokens, int n_pages);

 private:
  bool ensure_blocks(Sequence& s, int total_tokens);
  void release(Sequence& s, bool publish);
  void preempt(Sequence& s);
  void insert_waiting(Sequence* s);
  void emit(Sequence& s, int q_len, bool prefill, bool sample);
  int check_stop(Sequence& s);
  void forget(Sequence* s);  // drop s from the plan / lookahead records

  struct Inflight {
    std::vector<Sequence*> seqs;  // the plan's sampled rows, in sample order
    std::vector<int> pos;         // index of the placeholder in seqs[i]->tokens, -1 = none
  };
  std::deque<Inflight> inflight_;

  SchedulerConfig cfg_;
  BlockAllocator alloc_;
  PrefixCache cache_;
  std::unordered_map<int64_t, std::unique_ptr<Sequence>> seqs_;
  std::deque<Sequence*> waiting_;
  std::vector<Sequence*> running_;
  std::vector<int> free_slots_;
  int slots_created_ = 0;  // slot ids [0, slots_created_) exist (free or in use)
  StepPlan plan_;
  std::vector<Sequence*> plan_seqs_;
  int64_t arrival_counter_ = 0;
  int64_t total_preemptions_ = 0;
  int max_blocks_per_seq_;
};

}  // namespace xgs
