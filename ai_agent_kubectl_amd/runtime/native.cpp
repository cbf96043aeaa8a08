// Native host runtime for the kubectl-agent engine (pybind11 module `_native`).
//
//  * Trie: greedy longest-match byte tokenizer (engine/tokenizer.py semantics) — the per-request
//    encode of the query runs on the API thread, so it is kept off the Python interpreter.
//  * BlockManager: the paged-KV block allocator with reference counts and hash-chained automatic
//    prefix caching (engine/block_manager.py semantics, including LRU eviction of unreferenced
//    cached blocks and "always recompute the last prompt token").  It is the engine's KV memory
//    manager; the Python class is the reference implementation and the tests check both agree.
//  * SharedState: the response cache + rate-limit windows in POSIX shared memory, shared by the
//    API worker processes of one service (runtime/shared_state.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"
#include "shared_state.h"

namespace py = pybind11;
using ka::BlockManager;
using ka::SharedState;
using ka::Trie;

static void split_key(py::bytes k, uint64_t& k0, uint64_t& k1) {
  std::string s(k);
  if (s.size() != 16) throw std::invalid_argument("shared-state keys are 16-byte digests");
  std::memcpy(&k0, s.data(), 8);
  std::memcpy(&k1, s.data() + 8, 8);
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "kubectl-agent native host runtime (tokenizer trie, paged-KV block manager)";
  py::class_<Trie>(m, "Trie")
      .def(py::init<>())
      .def("add", [](Trie& t, py::bytes b, int id) { t.add(std::string(b), id); })
      .def("encode", [](const Trie& t, py::bytes b) {
        std::string s(b);
        py::gil_scoped_release rel;
        return t.encode(s);
      })
      .def("size", &Trie::size);
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>())
      .def("allocate_prompt", &BlockManager::allocate_prompt)
      .def("register_computed", &BlockManager::register_computed)
      .def("ensure_capacity", &BlockManager::ensure_capacity)
      .def("free_table", &BlockManager::free_table)
      .def("num_free", &BlockManager::num_free)
      .def("num_used", &BlockManager::num_used)
      .def("ref", &BlockManager::ref)
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("reuse_partial", &BlockManager::reuse_partial)
      .def("unpin", &BlockManager::unpin)
      .def("partial_tokens", &BlockManager::partial_tokens)
      .def("hits", &BlockManager::hits)
      .def("queries", &BlockManager::queries)
      .def("num_index_keys", &BlockManager::num_index_keys)
      .def_static("chain_hash", &BlockManager::chain_hash);
  py::class_<SharedState>(m, "SharedState")
      .def(py::init([](const std::string& name, uint32_t cache_cap, uint32_t value_max, uint32_t lim_cap) {
             return SharedState::open(name, cache_cap, value_max, lim_cap);
           }),
           py::arg("name"), py::arg("cache_cap"), py::arg("value_max") = 4096, py::arg("lim_cap") = 65536)
      .def_static("unlink", &SharedState::unlink)
      .def_property_readonly("name", &SharedState::name)
      .def_property_readonly("cache_capacity", &SharedState::cache_capacity)
      .def_property_readonly("value_max", &SharedState::value_max)
      .def("cache_get",
           [](SharedState& s, py::bytes k, double now) -> py::object {
             uint64_t k0, k1;
             split_key(k, k0, k1);
             std::string v;
             bool hit;
             {
               py::gil_scoped_release rel;
               hit = s.cache_get(k0, k1, now, &v);
             }
             if (!hit) return py::none();
             return py::bytes(v);
           })
      .def("cache_contains",
           [](SharedState& s, py::bytes k, double now) {
             uint64_t k0, k1;
             split_key(k, k0, k1);
             return s.cache_get(k0, k1, now, nullptr, false);
           })
      .def("cache_set",
           [](SharedState& s, py::bytes k, py::bytes v, double now, double ttl, uint32_t maxsize) {
             uint64_t k0, k1;
             split_key(k, k0, k1);
             std::string vs(v);
             py::gil_scoped_release rel;
             return s.cache_set(k0, k1, vs, now, ttl, maxsize);
           })
      .def("cache_delete",
           [](SharedState& s, py::bytes k) {
             uint64_t k0, k1;
             split_key(k, k0, k1);
             return s.cache_delete(k0, k1);
           })
      .def("cache_len", &SharedState::cache_len)
      .def("cache_clear", &SharedState::cache_clear)
      .def("debug_die_locked", &SharedState::debug_die_locked)
      .def("stats",
           [](SharedState& s) {
             uint64_t o[7];
             s.stats(o);
             py::dict d;
             d["hits"] = o[0];
             d["misses"] = o[1];
             d["sets"] = o[2];
             d["evictions"] = o[3];
             d["size"] = o[4];
             d["limiter_keys"] = o[5];
             d["owner_deaths"] = o[6];
             return d;
           })
      .def("limiter_hit",
           [](SharedState& s, py::bytes k, uint32_t amount, double expiry, double now) {
             uint64_t k0, k1;
             split_key(k, k0, k1);
             py::gil_scoped_release rel;
             return s.limiter_hit(k0, k1, amount, expiry, now);
           })
      .def("limiter_reset", &SharedState::limiter_reset)
      .def("load_set", &SharedState::load_set)
      .def("load_clear_worker", &SharedState::load_clear_worker)
      .def("load_total", &SharedState::load_total)
      .def("load_pick", &SharedState::load_pick);
}
