// Native host runtime for the kubectl-agent engine (pybind11 module `_native`).
//
//  * Trie: greedy longest-match byte tokenizer (engine/tokenizer.py semantics) — the per-request
//    encode of the query runs on the API thread, so it is kept off the Python interpreter.
//  * BlockManager: the paged-KV block allocator with reference counts and hash-chained automatic
//    prefix caching (engine/block_manager.py semantics, including LRU eviction of unreferenced
//    cached blocks and "always recompute the last prompt token").  It is the engine's KV memory
//    manager; the Python class is the reference implementation and the tests check both agree.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace py = pybind11;
using ka::BlockManager;
using ka::Trie;

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
}
