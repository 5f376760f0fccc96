// Randomised self-test of the native host runtime (csrc/runtime/runtime_core.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py (host code only;
// GPU sanitizers are not available on the MI355X pool).  Exits non-zero on the first broken invariant.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>

#include "../runtime/runtime_core.h"

#define REQUIRE(c)                                                       \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "%s:%d: invariant failed: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

template <typename F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

static void test_allocator(std::mt19937& rng) {
  BlockAllocator a(257, 64);
  REQUIRE(a.num_free() == 256);
  REQUIRE(a.blocks_for(1) == 1 && a.blocks_for(64) == 1 && a.blocks_for(65) == 2);
  std::vector<std::vector<int>> held;
  std::set<int> live;
  for (int step = 0; step < 20000; ++step) {
    if (held.empty() || rng() % 2) {
      const int n = rng() % 9;
      if (!a.can_alloc(n)) {
        REQUIRE(throws([&] { a.alloc(n); }));
        continue;
      }
      auto b = a.alloc(n);
      REQUIRE((int)b.size() == n);
      for (int x : b) {
        REQUIRE(x >= 1 && x < 257);
        REQUIRE(live.insert(x).second);  // never handed out twice
      }
      held.push_back(b);
    } else {
      const size_t i = rng() % held.size();
      a.release(held[i]);
      for (int x : held[i]) live.erase(x);
      if (!held[i].empty()) REQUIRE(throws([&] { a.release(held[i]); }));  // double free rejected
      held.erase(held.begin() + i);
    }
    REQUIRE(a.num_free() + (int)live.size() == 256);
  }
  REQUIRE(throws([&] { a.release({0}); }));   // scratch block
  REQUIRE(throws([&] { a.release({999}); })); // foreign id
  auto two = a.can_alloc(1) ? a.alloc(1) : std::vector<int>{};
  if (!two.empty()) REQUIRE(throws([&] { a.release({two[0], two[0]}); }));
}

static void test_scheduler(std::mt19937& rng) {
  const int blocks = 65, bs = 64, slots = 8, maxb = 16;
  Scheduler s(blocks, bs, slots, 512, maxb);
  long long next = 1;
  std::set<long long> known;
  for (int step = 0; step < 5000; ++step) {
    const int op = rng() % 5;
    if (op == 3 && s.num_running() > 0) {  // lazy growth of a random running request
      const auto run = s.running();
      const long long id = run[rng() % run.size()];
      const int before = (int)s.block_table(id).size(), free0 = s.free_blocks();
      const int got = s.grow(id, 1 + rng() % (bs * maxb + 100));
      REQUIRE(got == -1 ? ((int)s.block_table(id).size() == before && s.free_blocks() == free0)
                        : ((int)s.block_table(id).size() == before + got && s.free_blocks() == free0 - got));
      REQUIRE((int)s.block_table(id).size() <= maxb);
    } else if (op == 4 && s.num_running() > 0) {  // preempt the youngest, re-queued first
      const long long id = s.youngest_first().front();
      const int p = 1 + rng() % 300, m = 1 + rng() % 200;
      if ((p + m + bs - 1) / bs > maxb) {
        REQUIRE(throws([&] { s.preempt(id, p, m); }));
      } else {
        const int w0 = s.num_waiting();
        s.preempt(id, p, m);
        REQUIRE(s.slot(id) == -1 && s.block_table(id).empty() && s.num_waiting() == w0 + 1);
      }
    } else if (op == 0) {
      const int p = 1 + rng() % 300, m = 1 + rng() % 400;
      if ((p + m + bs - 1) / bs > maxb) {
        REQUIRE(throws([&] { s.add(next, p, m); }));
      } else {
        s.add(next, p, m);
        known.insert(next);
      }
      ++next;
    } else if (op == 1) {
      for (long long id : s.admit()) {
        REQUIRE(known.count(id));
        const int sl = s.slot(id);
        REQUIRE(sl >= 0 && sl < slots && s.slot_owners()[sl] == id);
      }
    } else if (op == 2 && !known.empty()) {
      auto it = known.begin();
      std::advance(it, rng() % known.size());
      s.finish(*it);
      known.erase(it);
    }
    // every running request's blocks are distinct and within the pool
    std::set<int> seen;
    int owned = 0;
    for (long long id : s.running())
      for (int b : s.block_table(id)) {
        REQUIRE(b >= 1 && b < blocks && seen.insert(b).second);
        ++owned;
      }
    REQUIRE(owned + s.free_blocks() == blocks - 1);
    REQUIRE(s.num_running() <= slots);
    REQUIRE(s.kv_usage() >= 0.0 && s.kv_usage() <= 1.0);
  }
  for (long long id : known) s.finish(id);
  REQUIRE(s.free_blocks() == blocks - 1 && s.num_running() == 0 && s.num_waiting() == 0);
}

static void test_levenshtein(std::mt19937& rng) {
  REQUIRE(levenshtein("kitten", "sitting") == 3);
  REQUIRE(levenshtein("", "abc") == 3 && levenshtein("abc", "") == 3);
  REQUIRE(levenshtein("h\xC3\xA9" "llo", "hello") == 1);  // one code point, not two bytes
  // malformed UTF-8 (truncated sequences, stray continuation bytes) must never read out of bounds
  const char* bad[] = {"\xE2\x82", "\xF0", "\x80\x80" "abc", "ab\xC3"};
  for (const char* b : bad) REQUIRE(levenshtein(b, "abc") >= 0);
  for (int i = 0; i < 2000; ++i) {
    std::string a(rng() % 40, 'x'), b(rng() % 40, 'y');
    for (auto& c : a) c = (char)(rng() & 0xff);
    for (auto& c : b) c = (char)(rng() & 0xff);
    const int d = levenshtein(a, b);
    REQUIRE(d == levenshtein(b, a));
    REQUIRE(d <= (int)std::max(a.size(), b.size()));
    REQUIRE(levenshtein(a, a) == 0);
  }
}

int main() {
  std::mt19937 rng(1234);
  test_allocator(rng);
  test_scheduler(rng);
  test_levenshtein(rng);
  std::puts("runtime selftest ok");
  return 0;
}
