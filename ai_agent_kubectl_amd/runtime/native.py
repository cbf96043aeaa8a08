"""Python face of the C++ host runtime (`runtime/native.cpp`, built by `build.build_runtime()`).

`make_tokenizer(tok)` returns a native trie encoder for a SyntheticTokenizer; `NativeBlockManager`
wraps the C++ paged-KV allocator behind the exact interface of `engine.block_manager.BlockManager`
(block tables stay Python lists owned by the sequences and are updated in place).
Set `KA_NATIVE=0` to force the pure-Python implementations.
"""
from __future__ import annotations

import os
from typing import List, Sequence

from ..engine.block_manager import NoFreeBlocks

try:
    if os.environ.get("KA_NATIVE", "1") == "0":
        raise ImportError("disabled by KA_NATIVE=0")
    from . import _native  # type: ignore
except ImportError:  # not built (CPU-only dev tree) -> pure Python fallbacks are used
    _native = None


def available() -> bool:
    return _native is not None


class _NativeTok:
    def __init__(self, trie):
        self.trie = trie

    def encode(self, data: bytes) -> List[int]:
        return self.trie.encode(data)


def make_tokenizer(tok):
    if _native is None:
        raise ImportError("native runtime not built")
    t = _native.Trie()
    for tid, p in enumerate(tok.id_to_bytes):
        if p is not None:
            t.add(p, tid)
    return _NativeTok(t)


class NativeBlockManager:
    """C++ block manager with the BlockManager interface."""

    def __init__(self, num_blocks: int, block_size: int = 16, enable_prefix_caching: bool = True):
        if _native is None:
            raise ImportError("native runtime not built")
        self._m = _native.BlockManager(num_blocks, block_size, enable_prefix_caching)
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.prefix_caching = enable_prefix_caching

    @property
    def num_free(self) -> int:
        return self._m.num_free()

    @property
    def num_used(self) -> int:
        return self._m.num_used()

    @property
    def hits(self) -> int:
        return self._m.hits()

    @property
    def queries(self) -> int:
        return self._m.queries()

    def ref_count(self, b: int) -> int:
        return self._m.ref(b)

    @property
    def num_index_keys(self) -> int:
        return self._m.num_index_keys()

    def blocks_needed(self, n: int) -> int:
        return (n + self.block_size - 1) // self.block_size

    def can_allocate(self, n: int) -> bool:
        return self.blocks_needed(n) <= self.num_free

    def allocate_prompt(self, tokens: Sequence[int]):
        try:
            table, cached, hashes = self._m.allocate_prompt(list(tokens))
        except RuntimeError as e:
            if "NoFreeBlocks" in str(e):
                raise NoFreeBlocks() from None
            raise
        return table, cached, hashes

    def register_computed(self, table: List[int], tokens: Sequence[int], hashes: List[int]) -> None:
        new = self._m.register_computed(table, list(tokens), hashes)
        hashes[:] = new

    def ensure_capacity(self, table: List[int], num_tokens: int) -> None:
        if len(table) * self.block_size >= num_tokens:
            return
        try:
            table[:] = self._m.ensure_capacity(table, num_tokens)
        except RuntimeError as e:
            if "NoFreeBlocks" in str(e):
                raise NoFreeBlocks() from None
            raise

    def free_table(self, table: List[int]) -> None:
        self._m.free_table(table)
        table.clear()

    def reset_prefix_cache(self) -> None:
        self._m.reset_prefix_cache()

    def reuse_partial(self, table: List[int], tokens: Sequence[int], cached: int, hashes: List[int]):
        src, r = self._m.reuse_partial(list(tokens), cached, hashes)
        return (src, r) if r > 0 else None

    def unpin(self, b: int) -> None:
        self._m.unpin(b)

    @property
    def partial_tokens(self) -> int:
        return self._m.partial_tokens()
