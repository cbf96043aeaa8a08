// Standalone stress test of the native host runtime (ai_agent_kubectl_amd/runtime/runtime.h),
// built by tests/test_native_sanitizers.py with -fsanitize=address,undefined.
//
// It drives the block manager the way the engine does — shared-prefix prompts, sub-block reuse,
// decode growth, frees in random order, LRU eviction under memory pressure, prefix-cache resets —
// and checks the allocator's invariants after every operation:
//   * refcounts never go negative, num_used == blocks referenced by live tables (+ pins);
//   * a prompt's cached prefix returns exactly the blocks that were published for it;
//   * the sibling index stays bounded by the number of blocks (no growth with distinct prompts).
// Any out-of-bounds access, use-after-free or UB aborts the process under the sanitizers.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>

#include "../../ai_agent_kubectl_amd/runtime/runtime.h"

#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

struct Live {
  std::vector<int> table, toks;
  std::vector<uint64_t> hashes;
  int pin = -1;
};

static void check_refs(const ka::BlockManager& bm, const std::vector<Live>& live, int nblocks) {
  std::vector<int> want(nblocks, 0);
  for (const auto& l : live) {
    for (int b : l.table) ++want[b];
    if (l.pin >= 0) ++want[l.pin];
  }
  int used = 0;
  for (int b = 0; b < nblocks; ++b) {
    CHECK(bm.ref(b) == want[b]);
    used += want[b] > 0;
  }
  CHECK(bm.num_used() == used);
  CHECK(bm.num_index_keys() <= (size_t)nblocks);
}

static void test_trie() {
  ka::Trie t;
  for (int c = 0; c < 256; ++c) t.add(std::string(1, (char)c), c);
  t.add("kubectl", 300);
  t.add("kube", 301);
  t.add(" get", 302);
  auto ids = t.encode("kubectl get pods");
  CHECK(ids.size() == 7 && ids[0] == 300 && ids[1] == 302 && ids[2] == ' ');
  ids = t.encode("kubex");
  CHECK(ids.size() == 2 && ids[0] == 301 && ids[1] == 'x');
  CHECK(t.encode("").empty());
  std::mt19937 rng(7);
  for (int it = 0; it < 2000; ++it) {   // random bytes, including NUL and high bytes
    std::string s(rng() % 64, '\0');
    for (auto& ch : s) ch = (char)(rng() & 255);
    size_t total = 0;
    for (int id : t.encode(s)) total += id == 300 ? 7 : id == 301 ? 4 : id == 302 ? 4 : 1;
    CHECK(total == s.size());
  }
  ka::Trie empty;
  bool threw = false;
  try {
    empty.encode("a");
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_block_manager(uint32_t seed, bool prefix) {
  const int nblocks = 96, bs = 4;
  ka::BlockManager bm(nblocks, bs, prefix);
  std::mt19937 rng(seed);
  std::vector<Live> live;
  std::vector<int> instr = {11, 12, 13, 14, 15, 16, 17, 18, 19};   // shared "instruction" prefix
  for (int step = 0; step < 6000; ++step) {
    const int op = rng() % 10;
    if (op < 5) {   // new prompt: shared prefix + unique tail (sometimes sharing a sibling's head)
      Live l;
      l.toks = instr;
      const int tail = 1 + rng() % 14;
      const int fam = rng() % 6;
      for (int i = 0; i < tail; ++i) l.toks.push_back(i < 3 ? 100 + fam * 3 + i : 1000 + (int)(rng() % 50000));
      try {
        auto r = bm.allocate_prompt(l.toks);
        l.table = std::get<0>(r);
        l.hashes = std::get<2>(r);
        const int cached = std::get<1>(r);
        CHECK(cached % bs == 0 && cached < (int)l.toks.size());
        CHECK((int)l.table.size() == bm.blocks_needed((int)l.toks.size()));
        auto pr = bm.reuse_partial(l.toks, cached, l.hashes);
        if (pr.second > 0) {
          CHECK(pr.first >= 0 && pr.first < nblocks && pr.second <= bs);
          l.pin = pr.first;
        }
        l.hashes = bm.register_computed(l.table, l.toks, l.hashes);
        CHECK(l.hashes.size() == l.toks.size() / bs || !prefix);
        if (l.pin >= 0) {   // the engine unpins after the block copy
          bm.unpin(l.pin);
          l.pin = -1;
        }
        live.push_back(std::move(l));
      } catch (const std::runtime_error& e) {
        CHECK(std::string(e.what()) == "NoFreeBlocks");
      }
    } else if (op < 7 && !live.empty()) {   // decode growth
      Live& l = live[rng() % live.size()];
      const int grow = 1 + rng() % 9;
      try {
        l.table = bm.ensure_capacity(l.table, (int)l.toks.size() + grow);
        for (int i = 0; i < grow; ++i) l.toks.push_back(2000 + (int)(rng() % 1000));
      } catch (const std::runtime_error& e) {
        CHECK(std::string(e.what()) == "NoFreeBlocks");
      }
    } else if (!live.empty()) {   // finish a random sequence
      const size_t i = rng() % live.size();
      bm.free_table(live[i].table);
      live.erase(live.begin() + (long)i);
    }
    if (step % 997 == 0) bm.reset_prefix_cache();
    check_refs(bm, live, nblocks);
  }
  // re-querying a live prompt walks the same hash chain and hits at least the shared prefix
  if (prefix) {
    for (const auto& l : live) {
      if (l.hashes.size() < 2) continue;
      try {
        auto r = bm.allocate_prompt(l.toks);
        const auto& hs = std::get<2>(r);
        CHECK(std::get<1>(r) >= 2 * bs);
        for (size_t i = 0; i < hs.size() && i < l.hashes.size(); ++i) CHECK(hs[i] == l.hashes[i]);
        bm.free_table(std::get<0>(r));
      } catch (const std::runtime_error& e) {
        CHECK(std::string(e.what()) == "NoFreeBlocks");
      }
    }
  }
  for (auto& l : live) bm.free_table(l.table);
  live.clear();
  check_refs(bm, live, nblocks);
  CHECK(bm.num_free() == nblocks);
  bool threw = false;
  try {
    bm.free_table({0});
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

int main() {
  test_trie();
  for (uint32_t seed = 1; seed <= 8; ++seed) {
    test_block_manager(seed, true);
    test_block_manager(seed, false);
  }
  std::printf("native runtime OK\n");
  return 0;
}
