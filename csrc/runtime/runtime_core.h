// Core of the native host runtime (no Python dependency): the paged-KV block allocator, the
// continuous-batching scheduler and the UTF-8 edit distance.  runtime.cpp binds it as `_lsa_runtime`;
// csrc/tests/runtime_selftest.cpp drives it under AddressSanitizer + UBSan (tests/test_native_sanitizers.py).
#pragma once
#include <algorithm>
#include <deque>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

// ------------------------------------------------------------------------------------------ utf-8
inline std::u32string utf8_to_u32(const std::string& s) {
  std::u32string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = s[i];
    char32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 0x6) { cp = c & 0x1f; n = 2; }
    else if ((c >> 4) == 0xe) { cp = c & 0x0f; n = 3; }
    else { cp = c & 0x07; n = 4; }
    for (int k = 1; k < n && i + k < s.size(); ++k) cp = (cp << 6) | (s[i + k] & 0x3f);
    out.push_back(cp);
    i += n;
  }
  return out;
}

inline int levenshtein_u32(const std::u32string& a, const std::u32string& b) {
  const std::u32string& s = a.size() < b.size() ? b : a;  // longer
  const std::u32string& t = a.size() < b.size() ? a : b;  // shorter: O(|t|) memory
  std::vector<int> prev(t.size() + 1), cur(t.size() + 1);
  for (size_t j = 0; j <= t.size(); ++j) prev[j] = (int)j;
  for (size_t i = 1; i <= s.size(); ++i) {
    cur[0] = (int)i;
    for (size_t j = 1; j <= t.size(); ++j) {
      const int sub = prev[j - 1] + (s[i - 1] == t[j - 1] ? 0 : 1);
      cur[j] = std::min({prev[j] + 1, cur[j - 1] + 1, sub});
    }
    std::swap(prev, cur);
  }
  return prev[t.size()];
}

inline int levenshtein(const std::string& a, const std::string& b) { return levenshtein_u32(utf8_to_u32(a), utf8_to_u32(b)); }

// ------------------------------------------------------------------------------------- allocator
class BlockAllocator {
 public:
  BlockAllocator(int num_blocks, int block_size) : num_blocks_(num_blocks), block_size_(block_size) {
    if (num_blocks < 2) throw std::invalid_argument("need at least 2 KV blocks (block 0 is scratch)");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 1; --b) free_.push_back(b);
    owned_.assign(num_blocks, 0);
  }
  int blocks_for(int tokens) const { return (tokens + block_size_ - 1) / block_size_; }
  bool can_alloc(int n) const { return (int)free_.size() >= n; }
  std::vector<int> alloc(int n) {
    if (!can_alloc(n)) throw std::runtime_error("KV cache exhausted");
    if (n < 0) throw std::invalid_argument("negative block count");
    std::vector<int> out(free_.end() - n, free_.end());
    free_.resize(free_.size() - n);
    std::reverse(out.begin(), out.end());
    for (int b : out) owned_[b] = 1;
    return out;
  }
  void release(const std::vector<int>& blocks) {
    for (int b : blocks)  // validate everything first: a bad list releases nothing
      if (b <= 0 || b >= num_blocks_ || !owned_[b]) throw std::invalid_argument("bad or already-free block id");
    std::vector<int> sorted(blocks);
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      throw std::invalid_argument("block listed twice");
    for (int b : blocks) {
      owned_[b] = 0;
      free_.push_back(b);
    }
  }
  int num_free() const { return (int)free_.size(); }
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }

 private:
  int num_blocks_, block_size_;
  std::vector<int> free_;
  std::vector<unsigned char> owned_;  // 1 while a block is handed out (double-free / foreign-id guard)
};

// ------------------------------------------------------------------------------------- scheduler
// KV reservation is lazy: admission reserves the prompt plus at most `reserve_tokens` generated tokens (one 64-token
// block by default; < 0 = the whole prompt + max_new up front, the pre-round-4 behaviour), and the engine grows a
// running request's table before each decode run (grow) as its context crosses block boundaries.  When the arena is
// exhausted the engine preempts (preempt): the request's blocks and slot are released and it is re-queued at the
// FRONT of the waiting queue with its generated tokens folded into its prompt (recompute on re-admission).  Without
// this, Ollama's generate-until-EOS default (max_new = the whole remaining window) pinned a full-window KV reservation
// per request for a ~30-token SQL answer.
struct Req {
  long long id;
  int prompt_len;
  int max_new;
  int slot = -1;
  long long admit_seq = -1;  // admission order (preemption picks the youngest)
  std::vector<int> blocks;
};

class Scheduler {
 public:
  Scheduler(int num_blocks, int block_size, int max_slots, int max_prefill_tokens, int max_blocks_per_seq,
            int reserve_tokens = 64)
      : alloc_(num_blocks, block_size), max_slots_(max_slots), max_prefill_tokens_(max_prefill_tokens),
        max_blocks_per_seq_(max_blocks_per_seq), reserve_tokens_(reserve_tokens), slots_(max_slots, -1) {}

  void add(long long id, int prompt_len, int max_new) {
    if (reqs_.count(id)) throw std::invalid_argument("duplicate request id");
    if (prompt_len < 1 || max_new < 1) throw std::invalid_argument("empty prompt or max_new < 1");
    const int need = alloc_.blocks_for(prompt_len + max_new);
    if (need > max_blocks_per_seq_) throw std::invalid_argument("request exceeds max model length");
    if (need > alloc_.num_blocks() - 1) throw std::invalid_argument("request larger than the whole KV cache");
    reqs_[id] = Req{id, prompt_len, max_new};
    waiting_.push_back(id);
  }

  // blocks reserved when a request is admitted
  int admit_blocks(const Req& r) const {
    const int gen = reserve_tokens_ < 0 ? r.max_new : std::min(r.max_new, reserve_tokens_);
    return alloc_.blocks_for(r.prompt_len + gen);
  }

  // Admit waiting requests (FCFS) while a slot, the prefill budget and KV blocks allow.
  // Returns the ids admitted this step (to be prefilled) — each now owns a slot and its blocks.
  std::vector<long long> admit() {
    std::vector<long long> out;
    int budget = max_prefill_tokens_;
    while (!waiting_.empty()) {
      Req& r = reqs_.at(waiting_.front());
      if (!out.empty() && r.prompt_len > budget) break;  // always admit at least one if it fits
      const int need = admit_blocks(r);
      if (!alloc_.can_alloc(need)) break;
      int slot = -1;
      for (int s = 0; s < max_slots_; ++s)
        if (slots_[s] < 0) { slot = s; break; }
      if (slot < 0) break;
      r.blocks = alloc_.alloc(need);
      r.slot = slot;
      r.admit_seq = ++admit_counter_;
      slots_[slot] = r.id;
      budget -= r.prompt_len;
      out.push_back(r.id);
      waiting_.pop_front();
    }
    return out;
  }

  // Make a running request own the blocks for its first `tokens` cache positions (capped at prompt + max_new).
  // Returns the number of blocks added (0 if it already had them), or -1 when the arena cannot supply them
  // (nothing is allocated then).
  int grow(long long id, int tokens) {
    Req& r = reqs_.at(id);
    if (r.slot < 0) throw std::invalid_argument("grow: request is not running");
    const int want = std::min(alloc_.blocks_for(std::min(tokens, r.prompt_len + r.max_new)), max_blocks_per_seq_);
    const int add = want - (int)r.blocks.size();
    if (add <= 0) return 0;
    if (!alloc_.can_alloc(add)) return -1;
    const std::vector<int> nb = alloc_.alloc(add);
    r.blocks.insert(r.blocks.end(), nb.begin(), nb.end());
    return add;
  }

  // Release a running request's slot and blocks and put it back at the front of the waiting queue with a new
  // (prompt, max_new): the engine folds the tokens generated so far into the prompt and re-prefills them.
  void preempt(long long id, int prompt_len, int max_new) {
    Req& r = reqs_.at(id);
    if (r.slot < 0) throw std::invalid_argument("preempt: request is not running");
    if (prompt_len < 1 || max_new < 1 || alloc_.blocks_for(prompt_len + max_new) > max_blocks_per_seq_)
      throw std::invalid_argument("preempt: bad resumed lengths");
    slots_[r.slot] = -1;
    r.slot = -1;
    r.admit_seq = -1;
    alloc_.release(r.blocks);
    r.blocks.clear();
    r.prompt_len = prompt_len;
    r.max_new = max_new;
    waiting_.push_front(id);
  }

  // running requests, youngest admission first (the engine's preemption order)
  std::vector<long long> youngest_first() const {
    std::vector<std::pair<long long, long long>> v;
    for (long long s : slots_)
      if (s >= 0) v.emplace_back(-reqs_.at(s).admit_seq, s);
    std::sort(v.begin(), v.end());
    std::vector<long long> out;
    for (auto& p : v) out.push_back(p.second);
    return out;
  }

  void finish(long long id) {
    auto it = reqs_.find(id);
    if (it == reqs_.end()) return;
    Req& r = it->second;
    if (r.slot >= 0) slots_[r.slot] = -1;
    if (!r.blocks.empty()) alloc_.release(r.blocks);
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    reqs_.erase(it);
  }

  std::vector<int> block_table(long long id) const { return reqs_.at(id).blocks; }
  int slot(long long id) const { return reqs_.at(id).slot; }
  std::vector<long long> slot_owners() const { return slots_; }
  std::vector<long long> running() const {
    std::vector<long long> out;
    for (long long s : slots_)
      if (s >= 0) out.push_back(s);
    return out;
  }
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const {
    int n = 0;
    for (long long s : slots_) n += s >= 0;
    return n;
  }
  int highest_slot() const {
    for (int s = max_slots_ - 1; s >= 0; --s)
      if (slots_[s] >= 0) return s;
    return -1;
  }
  double kv_usage() const {
    return 1.0 - (double)alloc_.num_free() / (double)(alloc_.num_blocks() - 1);
  }
  int free_blocks() const { return alloc_.num_free(); }
  int reserve_tokens() const { return reserve_tokens_; }

 private:
  BlockAllocator alloc_;
  int max_slots_, max_prefill_tokens_, max_blocks_per_seq_, reserve_tokens_;
  long long admit_counter_ = 0;
  std::vector<long long> slots_;
  std::deque<long long> waiting_;
  std::unordered_map<long long, Req> reqs_;
};
