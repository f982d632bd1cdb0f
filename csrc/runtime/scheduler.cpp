#include "scheduler.h"

#include <algorithm>
#include <stdexcept>

namespace xgs {

StepScheduler::StepScheduler(const SchedulerConfig& cfg)
    : cfg_(cfg),
      alloc_(cfg.num_blocks),
      cache_(&alloc_, cfg.block_size,
             cfg.enable_prefix_cache ? static_cast<int>(cfg.cache_threshold * cfg.num_blocks) : 0) {
  if (cfg_.block_size <= 0 || cfg_.num_blocks <= 0) throw std::invalid_argument("bad scheduler config");
  max_blocks_per_seq_ = (cfg_.max_model_len + cfg_.block_size - 1) / cfg_.block_size + 1;
  free_slots_.reserve(cfg_.max_num_seqs);
  for (int i = cfg_.max_num_seqs - 1; i >= 0; --i) free_slots_.push_back(i);
  slots_created_ = cfg_.max_num_seqs;
}

void StepScheduler::set_limits(int max_num_seqs, int max_num_batched_tokens) {
  // The slot pool only grows: ids below the high-water mark already exist (free or
  // held by a running sequence); a shrink just lowers the admission limit, which
  // the running_.size() < max_num_seqs check enforces.
  for (int i = slots_created_; i < max_num_seqs; ++i) free_slots_.insert(free_slots_.begin(), i);
  slots_created_ = std::max(slots_created_, max_num_seqs);
  cfg_.max_num_seqs = std::max(1, max_num_seqs);
  cfg_.max_num_batched_tokens = std::max(1, max_num_batched_tokens);
}

int StepScheduler::num_used_blocks() const { return alloc_.num_blocks() - alloc_.num_free(); }

std::vector<int> StepScheduler::cached_prefix(const std::vector<int32_t>& tokens) {
  return cache_.match(tokens.data(), static_cast<int>(tokens.size()), static_cast<int>(tokens.size()), false);
}

std::vector<int> StepScheduler::install_prefix(const std::vector<int32_t>& tokens, int n_pages) {
  const int bs = cfg_.block_size;
  n_pages = std::min<int>(n_pages, static_cast<int>(tokens.size()) / bs);
  std::vector<int> have = cached_prefix(tokens);
  const int before = std::min<int>(static_cast<int>(have.size()), n_pages);
  have.resize(before);
  std::vector<int> fresh;
  for (int i = before; i < n_pages; ++i) {
    int b = alloc_.alloc();
    if (b < 0 && cache_.evict(1) > 0) b = alloc_.alloc();
    if (b < 0) {
      for (int f : fresh) alloc_.decref(f);
      return {};
    }
    fresh.push_back(b);
    have.push_back(b);
  }
  cache_.insert(tokens.data(), n_pages * bs, have.data(), n_pages);
  for (int f : fresh) alloc_.decref(f);  // the cache now holds the only reference
  std::vector<int> out;
  out.reserve(have.size() + 1);
  out.push_back(before);
  out.insert(out.end(), have.begin(), have.end());
  return out;
}

const Sequence* StepScheduler::get(int64_t id) const {
  auto it = seqs_.find(id);
  return it == seqs_.end() ? nullptr : it->second.get();
}

bool StepScheduler::add(int64_t id, const std::vector<int32_t>& prompt, int max_tokens, int priority,
                        bool ignore_eos, bool embed,
                        const std::vector<std::vector<int32_t>>& stop_seqs, int min_tokens) {
  if (seqs_.count(id) || prompt.empty()) return false;
  const int limit = embed ? cfg_.max_model_len : cfg_.max_model_len - 1;
  if (static_cast<int>(prompt.size()) > limit) return false;
  auto s = std::make_unique<Sequence>();
  s->id = id;
  s->priority = priority;
  s->arrival = arrival_counter_++;
  s->tokens = prompt;
  s->prompt_len = static_cast<int>(prompt.size());
  s->max_tokens = max_tokens;
  s->min_tokens = min_tokens;
  s->ignore_eos = ignore_eos;
  s->embed = embed;
  for (const auto& ss : stop_seqs)
    if (!ss.empty()) s->stop_seqs.push_back(ss);
  Sequence* raw = s.get();
  seqs_.emplace(id, std::move(s));
  insert_waiting(raw);
  return true;
}

void StepScheduler::insert_waiting(Sequence* s) {
  auto it = waiting_.begin();
  for (; it != waiting_.end(); ++it) {
    Sequence* w = *it;
    if (w->priority < s->priority || (w->priority == s->priority && w->arrival > s->arrival)) break;
  }
  waiting_.insert(it, s);
}

bool StepScheduler::ensure_blocks(Sequence& s, int total_tokens) {
  const int bs = cfg_.block_size;
  const int need = (total_tokens + bs - 1) / bs;
  while (static_cast<int>(s.blocks.size()) < need) {
    int b = alloc_.alloc();
    if (b < 0) {
      int want = need - static_cast<int>(s.blocks.size());
      if (cache_.evict(std::max(want, 16)) == 0) return false;
      b = alloc_.alloc();
      if (b < 0) return false;
    }
    s.blocks.push_back(b);
  }
  return true;
}

void StepScheduler::release(Sequence& s, bool publish) {
  if (publish && cfg_.enable_prefix_cache && !s.blocks.empty()) {
    int n = std::min(s.num_computed, static_cast<int>(s.tokens.size()));
    cache_.insert(s.tokens.data(), n, s.blocks.data(), static_cast<int>(s.blocks.size()));
  }
  for (int b : s.blocks) alloc_.decref(b);
  s.blocks.clear();
  if (s.slot >= 0) {
    free_slots_.push_back(s.slot);
    s.slot = -1;
  }
}

void StepScheduler::preempt(Sequence& s) {
  release(s, /*publish=*/true);
  s.num_computed = 0;
  s.draft.clear();
  s.status = SeqStatus::Waiting;
  ++s.num_preemptions;
  ++total_preemptions_;
  insert_waiting(&s);
  plan_.preempted.push_back(s.id);
}

bool StepScheduler::abort(int64_t id) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  Sequence* s = it->second.get();
  if (s->status == SeqStatus::Running) {
    release(*s, /*publish=*/true);
    running_.erase(std::remove(running_.begin(), running_.end(), s), running_.end());
  } else {
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), s), waiting_.end());
    release(*s, false);
  }
  forget(s);
  seqs_.erase(it);
  return true;
}

void StepScheduler::forget(Sequence* s) {
  for (auto& p : plan_seqs_)
    if (p == s) p = nullptr;
  for (auto& r : inflight_)
    for (auto& p : r.seqs)
      if (p == s) p = nullptr;
}

bool StepScheduler::set_draft(int64_t id, const std::vector<int32_t>& draft) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  Sequence* s = it->second.get();
  int room = cfg_.max_model_len - static_cast<int>(s->tokens.size()) - 1;
  int left = s->max_tokens - s->num_generated() - 1;
  int n = std::max(0, std::min<int>({static_cast<int>(draft.size()), room, left}));
  s->draft.assign(draft.begin(), draft.begin() + n);
  return true;
}

void StepScheduler::emit(Sequence& s, int q, bool prefill, bool sample) {
  const int bs = cfg_.block_size;
  StepPlan& p = plan_;
  p.seq_ids.push_back(s.id);
  p.slots.push_back(s.slot);
  p.q_lens.push_back(q);
  p.ctx_lens.push_back(s.num_computed);
  p.seq_lens.push_back(s.num_computed + q);
  p.is_prefill.push_back(prefill ? 1 : 0);
  p.do_sample.push_back(sample ? 1 : 0);
  p.is_embed.push_back(s.embed ? 1 : 0);
  const int n_tok = static_cast<int>(s.tokens.size());
  for (int t = 0; t < q; ++t) {
    int pos = s.num_computed + t;
    int tok = pos < n_tok ? s.tokens[pos] : s.draft[pos - n_tok];
    p.input_ids.push_back(tok);
    p.positions.push_back(pos);
    p.slot_mapping.push_back(s.blocks[pos / bs] * bs + pos % bs);
  }
  if (sample) {
    int first = s.draft.empty() ? q - 1 : 0;  // verify steps need every row
    for (int t = first; t < q; ++t) p.logits_indices.push_back(p.num_tokens + t);
    p.sample_seq_index.push_back(p.num_seqs);
    ++p.num_sample;
  }
  p.num_tokens += q;
  p.query_start_loc.push_back(p.num_tokens);
  p.max_q_len = std::max(p.max_q_len, q);
  p.max_seq_len = std::max(p.max_seq_len, s.num_computed + q);
  ++p.num_seqs;
  plan_seqs_.push_back(&s);
}

const StepPlan& StepScheduler::schedule() {
  plan_ = StepPlan{};
  plan_.query_start_loc.push_back(0);
  plan_seqs_.clear();
  int budget = cfg_.max_num_batched_tokens;

  std::stable_sort(running_.begin(), running_.end(), [](const Sequence* a, const Sequence* b) {
    if (a->priority != b->priority) return a->priority > b->priority;
    return a->arrival < b->arrival;
  });
  std::vector<uint8_t> scheduled(running_.size(), 0);
  auto pick_victim = [&](size_t self) -> int {
    for (int j = static_cast<int>(running_.size()) - 1; j >= 0; --j)
      if (static_cast<size_t>(j) != self && !scheduled[j] && running_[j]->status == SeqStatus::Running)
        return j;
    return -1;
  };

  // Pass 1: pure decodes (q_len 1, no draft) -- they come first in the batch.
  for (size_t i = 0; i < running_.size() && budget > 0; ++i) {
    Sequence* s = running_[i];
    if (s->status != SeqStatus::Running) continue;
    int remaining = static_cast<int>(s->tokens.size()) - s->num_computed;
    if (remaining != 1 || !s->draft.empty() || s->embed) continue;
    bool ok = true;
    while (!ensure_blocks(*s, s->num_computed + 1)) {
      int v = pick_victim(i);
      if (v < 0) { ok = false; break; }
      preempt(*running_[v]);
    }
    if (!ok) { preempt(*s); continue; }
    scheduled[i] = 1;
    emit(*s, 1, false, true);
    --budget;
  }
  plan_.num_decodes = plan_.num_seqs;
  if (cfg_.decode_prefill_cap > 0 && plan_.num_decodes > 0) budget = std::min(budget, cfg_.decode_prefill_cap);
  int max_pf = cfg_.max_prefill_seqs;
  if (cfg_.decode_prefill_seqs > 0 && plan_.num_decodes > 0) max_pf = std::min(max_pf, cfg_.decode_prefill_seqs);

  // Pass 2: verify steps (decode + draft) and continuing prefill chunks.
  int n_prefill = 0;
  for (size_t i = 0; i < running_.size() && budget > 0; ++i) {
    Sequence* s = running_[i];
    if (s->status != SeqStatus::Running || scheduled[i]) continue;
    int remaining = static_cast<int>(s->tokens.size()) - s->num_computed;
    bool verify = remaining == 1 && !s->draft.empty();
    int q = verify ? 1 + static_cast<int>(s->draft.size()) : std::min(remaining, budget);
    if (verify && q > budget) continue;
    if (!verify && q < remaining && !cfg_.chunked_prefill && plan_.num_seqs > 0) continue;
    if (!verify && n_prefill >= max_pf) continue;
    bool ok = true;
    while (!ensure_blocks(*s, s->num_computed + q)) {
      int v = plan_.num_seqs == 0 ? pick_victim(i) : -1;
      if (v < 0) { ok = false; break; }
      preempt(*running_[v]);
    }
    if (!ok) {
      if (verify) {  // fall back to a plain decode next step
        s->draft.clear();
      }
      continue;
    }
    scheduled[i] = 1;
    bool completes = s->num_computed + q >= static_cast<int>(s->tokens.size());
    emit(*s, q, !verify, completes && !s->embed);
    if (!verify) ++n_prefill;
    budget -= q;
  }
  running_.erase(std::remove_if(running_.begin(), running_.end(),
                                [](Sequence* s) { return s->status != SeqStatus::Running; }),
                 running_.end());

  // Pass 3: admissions (behind the admission window, see SchedulerConfig).
  const int reserve_pages = static_cast<int>(cfg_.admit_watermark * cfg_.num_blocks);
  bool hold = false;
  if (cfg_.coalesce_prompts > 1 && plan_.num_decodes > 0 && n_prefill == 0 && !waiting_.empty()) {
    int ready = 0;
    for (const Sequence* s : waiting_) {
      if (s->tokens.back() == kPlaceholder) break;
      if (++ready >= cfg_.coalesce_prompts) break;
    }
    // (free slots can be fewer than coalesce_prompts: rows finishing meanwhile make
    // room, and the wait bound caps the hold either way)
    hold = ready < cfg_.coalesce_prompts && waiting_.front()->wait_plans < cfg_.coalesce_max_wait;
  }
  while (!hold && !waiting_.empty() && budget > 0 && static_cast<int>(running_.size()) < cfg_.max_num_seqs &&
         n_prefill < max_pf) {
    Sequence* s = waiting_.front();
    if (s->tokens.back() == kPlaceholder) break;  // preempted by a lookahead plan: wait for commit()
    int matched_pages = 0;
    bool looked_up = false;
    if (cfg_.enable_prefix_cache && s->blocks.empty() && s->num_computed == 0) {
      looked_up = true;
      const int n = static_cast<int>(s->tokens.size());
      std::vector<int> pages = cache_.match(s->tokens.data(), n, n - 1, /*count=*/false);
      for (int b : pages) {
        alloc_.incref(b);
        s->blocks.push_back(b);
      }
      matched_pages = static_cast<int>(pages.size());
      s->num_computed = matched_pages * cfg_.block_size;
      if (s->num_preemptions == 0) s->num_cached = s->num_computed;
    }
    int remaining = static_cast<int>(s->tokens.size()) - s->num_computed;
    int q = std::min(remaining, budget);
    auto undo = [&]() {
      for (int b : s->blocks) alloc_.decref(b);
      s->blocks.clear();
      s->num_computed = 0;
    };
    if (q < remaining && !cfg_.chunked_prefill && plan_.num_seqs > 0) { undo(); break; }
    const int bs = cfg_.block_size;
    int need = (s->num_computed + q + bs - 1) / bs - static_cast<int>(s->blocks.size());
    int reserve = running_.empty() ? 0 : reserve_pages;
    if (alloc_.num_free() - need < reserve) cache_.evict(need + reserve - alloc_.num_free());
    if (alloc_.num_free() - need < reserve || !ensure_blocks(*s, s->num_computed + q)) {
      undo();
      break;
    }
    waiting_.pop_front();
    if (looked_up && s->num_preemptions == 0)  // count the lookup once, when it is used
      cache_.record_lookup(static_cast<int>(s->tokens.size()), matched_pages);
    s->status = SeqStatus::Running;
    if (free_slots_.empty()) throw std::runtime_error("scheduler: slot pool exhausted");
    s->slot = free_slots_.back();
    free_slots_.pop_back();
    running_.push_back(s);
    bool completes = s->num_computed + q >= static_cast<int>(s->tokens.size());
    emit(*s, q, true, completes && !s->embed);
    ++n_prefill;
    budget -= q;
  }
  for (Sequence* s : waiting_) ++s->wait_plans;

  // Block tables.
  int w = 1;
  for (Sequence* s : plan_seqs_) w = std::max<int>(w, static_cast<int>(s->blocks.size()));
  plan_.bt_width = w;
  plan_.block_tables.assign(static_cast<size_t>(plan_.num_seqs) * w, 0);
  for (int i = 0; i < plan_.num_seqs; ++i) {
    const auto& b = plan_seqs_[i]->blocks;
    std::copy(b.begin(), b.end(), plan_.block_tables.begin() + static_cast<size_t>(i) * w);
  }
  return plan_;
}

int StepScheduler::check_stop(Sequence& s) {
  const int32_t last = s.tokens.back();
  const int gen = s.num_generated();
  if (!s.ignore_eos && gen >= std::max(1, s.min_tokens)) {
    for (int32_t e : cfg_.eos_ids)
      if (e == last) return static_cast<int>(SeqFinish::Stop);
  }
  for (const auto& ss : s.stop_seqs) {
    if (static_cast<int>(ss.size()) > gen) continue;
    if (std::equal(ss.begin(), ss.end(), s.tokens.end() - ss.size()))
      return static_cast<int>(SeqFinish::StopSequence);
  }
  if (gen >= s.max_tokens) return static_cast<int>(SeqFinish::Length);
  if (static_cast<int>(s.tokens.size()) >= cfg_.max_model_len) return static_cast<int>(SeqFinish::Length);
  return 0;
}

std::vector<FinishedSeq> StepScheduler::update(const int32_t* tokens, const int32_t* counts,
                                               int num_sample) {
  std::vector<FinishedSeq> done;
  if (!inflight_.empty()) throw std::logic_error("update: lookahead plans must be committed first");
  if (num_sample != plan_.num_sample) throw std::invalid_argument("update: num_sample mismatch");
  int k = 0, si = 0;
  std::vector<Sequence*> finished;
  for (int i = 0; i < plan_.num_seqs; ++i) {
    Sequence* s = plan_seqs_[i];
    const bool sample = plan_.do_sample[i] != 0;
    int c = 0;
    if (sample) c = counts[si++];
    if (!s || s->status != SeqStatus::Running) { k += c; continue; }
    int reason = 0;
    if (sample) {
      const bool first_sample = s->num_generated() == 0;
      s->draft.clear();
      for (int t = 0; t < c && !reason; ++t) {
        s->tokens.push_back(tokens[k + t]);
        reason = check_stop(*s);
      }
      k += c;
      s->num_computed = static_cast<int>(s->tokens.size()) - 1;
      if (first_sample && cfg_.enable_prefix_cache)  // publish the prompt pages early
        cache_.insert(s->tokens.data(), s->num_computed, s->blocks.data(),
                      static_cast<int>(s->blocks.size()));
    } else {
      s->num_computed += plan_.q_lens[i];
      if (s->embed && s->num_computed >= static_cast<int>(s->tokens.size()))
        reason = static_cast<int>(SeqFinish::Embedded);
    }
    if (reason) {
      s->finish = static_cast<SeqFinish>(reason);
      finished.push_back(s);
    }
  }
  for (Sequence* s : finished) {
    release(*s, /*publish=*/true);
    s->status = SeqStatus::Finished;
    running_.erase(std::remove(running_.begin(), running_.end(), s), running_.end());
    done.push_back(FinishedSeq{s->id, s->finish, s->prompt_len, s->num_generated(), s->num_cached});
    forget(s);
    seqs_.erase(s->id);
  }
  return done;
}

bool StepScheduler::lookahead(bool across_length_finish) {
  const StepPlan& p = plan_;
  if (p.num_seqs == 0 || p.num_sample == 0) return false;
  if (!cfg_.lookahead_mixed && (p.num_decodes != p.num_seqs || p.num_sample != p.num_seqs)) return false;
  for (int i = 0; i < p.num_seqs; ++i) {
    const Sequence* s = plan_seqs_[i];
    if (s == nullptr) continue;
    if (!s->draft.empty() || p.is_embed[i]) return false;  // verify / embedding steps stay synchronous
    // a sampled row that reaches its length limit with this token: either released
    // early below, or (the default) this plan stays synchronous
    const int i_sampled = p.do_sample[i];
    if (i_sampled && !cfg_.early_release && !across_length_finish && s->status == SeqStatus::Running &&
        (s->num_generated() + 1 >= s->max_tokens || static_cast<int>(s->tokens.size()) + 1 >= cfg_.max_model_len))
      return false;
  }
  // Every sampled row (decodes and prompts completing this step) gets a placeholder
  // token in sample order; prompt chunks that do not complete advance as update()
  // would advance them. A sampled row that reaches its length limit with this token
  // finishes at commit whatever the token is: unless across_length_finish, its slot
  // and pages are released NOW (published to the prefix cache without the
  // placeholder), so the plan made next can admit a waiting request into them
  // (admission latency = TTFT) while this step is still on the GPU -- the GPU
  // stream orders this step's reads of those pages before the next step's writes.
  Inflight r;
  r.seqs.reserve(p.num_sample);
  r.pos.reserve(p.num_sample);
  std::vector<uint8_t> sampled(p.num_seqs, 0);
  for (int j = 0; j < p.num_sample; ++j) {
    const int i = p.sample_seq_index[j];
    sampled[i] = 1;
    Sequence* s = plan_seqs_[i];
    r.seqs.push_back(s);
    if (s == nullptr || s->status != SeqStatus::Running) {
      r.pos.push_back(-1);
      continue;
    }
    const bool first_sample = s->num_generated() == 0;
    r.pos.push_back(static_cast<int>(s->tokens.size()));
    s->tokens.push_back(kPlaceholder);
    s->num_computed = static_cast<int>(s->tokens.size()) - 1;
    if (first_sample && cfg_.enable_prefix_cache)  // publish the prompt pages early (as update())
      cache_.insert(s->tokens.data(), s->num_computed, s->blocks.data(), static_cast<int>(s->blocks.size()));
    const bool length_end = s->num_generated() >= s->max_tokens ||
                            static_cast<int>(s->tokens.size()) >= cfg_.max_model_len;
    if (length_end && !across_length_finish && cfg_.early_release) {
      release(*s, /*publish=*/true);
      running_.erase(std::remove(running_.begin(), running_.end(), s), running_.end());
      s->status = SeqStatus::Finished;
      s->released_early = true;
    }
  }
  for (int i = 0; i < p.num_seqs; ++i) {
    Sequence* s = plan_seqs_[i];
    if (s == nullptr || sampled[i] || s->status != SeqStatus::Running) continue;
    s->num_computed += p.q_lens[i];
  }
  inflight_.push_back(std::move(r));
  for (auto& q : plan_seqs_) q = nullptr;  // the plan is now owned by the record
  return true;
}

std::vector<FinishedSeq> StepScheduler::commit(const int32_t* tokens, int num_sample) {
  if (inflight_.empty()) throw std::logic_error("commit: no lookahead plan in flight");
  Inflight r = std::move(inflight_.front());
  inflight_.pop_front();
  if (num_sample != static_cast<int>(r.seqs.size())) throw std::invalid_argument("commit: num_sample mismatch");
  std::vector<Sequence*> finished;
  for (int i = 0; i < num_sample; ++i) {
    Sequence* s = r.seqs[i];
    const int pos = r.pos[i];
    if (s == nullptr || pos < 0 || (s->status == SeqStatus::Finished && !s->released_early)) continue;
    if (pos != static_cast<int>(s->tokens.size()) - 1 || s->tokens[pos] != kPlaceholder)
      throw std::logic_error("commit: placeholder bookkeeping out of order");
    s->tokens[pos] = tokens[i];
    int reason = check_stop(*s);
    if (s->released_early && !reason) reason = static_cast<int>(SeqFinish::Length);
    if (reason) {
      s->finish = static_cast<SeqFinish>(reason);
      finished.push_back(s);
    }
  }
  std::vector<FinishedSeq> done;
  for (Sequence* s : finished) {
    if (s->status == SeqStatus::Running) {
      release(*s, /*publish=*/true);
      running_.erase(std::remove(running_.begin(), running_.end(), s), running_.end());
    } else {  // preempted by the lookahead schedule(): waiting, holds no pages
      waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), s), waiting_.end());
      release(*s, false);
    }
    s->status = SeqStatus::Finished;
    done.push_back(FinishedSeq{s->id, s->finish, s->prompt_len, s->num_generated(), s->num_cached});
    forget(s);
    seqs_.erase(s->id);
  }
  return done;
}

}  // namespace xgs
