"""Paged-KV block manager with automatic prefix caching.

KV memory is a pool of fixed-size blocks (16 tokens; `[NB, Hkv, 16, D]` K and `[NB, Hkv, D, 16]` V
per layer, engine/runner.py).  A sequence owns a block table (list of block ids).  Full blocks are
content-addressed by a hash chained over (parent hash, 16 token ids), so every request that starts
with the reference's fixed instruction prompt (`/root/reference/app.py:50-57`, ~65 tokens with the
chat header) shares those KV blocks and only its own query tokens are prefilled.

Invariants:
* ref_count[b] = number of live sequences whose table contains b;
* a block with ref 0 that carries a hash stays cached (evictable, LRU) until the free list runs
  dry; a block with ref 0 and no hash goes straight back to the free list;
* at least one prompt token is always recomputed so the prefill produces logits.

Sub-block reuse (`reuse_partial`): the instruction prompt rarely ends on a block boundary (72
tokens with the Llama-3 chat header = 4 full blocks + 8 tokens), so block-granular caching would
recompute its tail in every request.  Each published block is also indexed under its PARENT hash
with its 16 tokens; a new prompt whose next block shares a token prefix of length r with such a
sibling pins the sibling and copies its KV into its own fresh block before the prefill (the copy
is exact: causal attention makes the first r rows depend only on the shared chain), so only the
tokens after r are computed.

The C++ runtime (`runtime/native.cpp`, `make_block_manager`) implements the same structure for the scheduler hot
path when the native module is built; this Python class is the reference and the fallback.
"""
from __future__ import annotations

import collections
from typing import Dict, List, Optional, Sequence


class NoFreeBlocks(RuntimeError):
    pass


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int = 16, enable_prefix_caching: bool = True):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.prefix_caching = enable_prefix_caching
        self.ref = [0] * num_blocks
        self.block_hash: List[Optional[int]] = [None] * num_blocks
        self.free: collections.deque = collections.deque(range(num_blocks))
        self.cached: Dict[int, int] = {}                         # hash -> block
        self.evictable: "collections.OrderedDict[int, None]" = collections.OrderedDict()  # LRU of ref-0 cached
        self.hits = 0
        self.queries = 0
        self.partial_tokens = 0
        self.children: Dict[int, "collections.deque[int]"] = {}   # parent hash -> recent child blocks
        self.parent_of: List[Optional[int]] = [None] * num_blocks
        self.block_toks: List[Optional[tuple]] = [None] * num_blocks

    # ------------------------------------------------------------------------------------------
    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.evictable)

    @property
    def num_used(self) -> int:
        return self.num_blocks - self.num_free

    @staticmethod
    def chain_hash(parent: int, tokens: Sequence[int]) -> int:
        return hash((parent, tuple(tokens)))

    def _pop_free(self) -> int:
        if self.free:
            return self.free.popleft()
        if self.evictable:
            b, _ = self.evictable.popitem(last=False)
            h = self.block_hash[b]
            if h is not None and self.cached.get(h) == b:
                del self.cached[h]
            self._unhash(b)
            return b
        raise NoFreeBlocks()

    def _acquire(self, b: int) -> None:
        if self.ref[b] == 0 and b in self.evictable:
            del self.evictable[b]
        self.ref[b] += 1

    def _release(self, b: int) -> None:
        self.ref[b] -= 1
        assert self.ref[b] >= 0
        if self.ref[b] == 0:
            if self.block_hash[b] is not None and self.cached.get(self.block_hash[b]) == b:
                self.evictable[b] = None
            else:
                self._unhash(b)
                self.free.append(b)

    def _unhash(self, b: int) -> None:
        """Drop b's prefix-cache identity and its entry in the sibling index (so the index keeps
        one key per parent with a live published child, however many prompts pass through)."""
        if self.block_hash[b] is None:
            return
        self.block_hash[b] = None
        par = self.parent_of[b]
        kids = self.children.get(par)
        if kids is not None:
            try:
                kids.remove(b)
            except ValueError:
                pass   # already pushed out of the 4-deep deque
            if not kids:
                del self.children[par]
        self.parent_of[b] = None
        self.block_toks[b] = None

    # ------------------------------------------------------------------------------------------
    def ref_count(self, b: int) -> int:
        return self.ref[b]

    @property
    def num_index_keys(self) -> int:
        return len(self.children)

    def blocks_needed(self, num_tokens: int) -> int:
        return (num_tokens + self.block_size - 1) // self.block_size

    def can_allocate(self, num_tokens: int) -> bool:
        return self.blocks_needed(num_tokens) <= self.num_free

    def allocate_prompt(self, tokens: Sequence[int]):
        """Build a block table for a new prompt.  Returns (table, num_cached_tokens, hashes)."""
        bs = self.block_size
        table: List[int] = []
        hashes: List[int] = []
        cached_tokens = 0
        parent = 0
        n_full = (len(tokens) - 1) // bs if self.prefix_caching else 0
        self.queries += 1
        for i in range(n_full):
            h = self.chain_hash(parent, tokens[i * bs:(i + 1) * bs])
            b = self.cached.get(h)
            if b is None:
                break
            self._acquire(b)
            table.append(b)
            hashes.append(h)
            parent = h
            cached_tokens += bs
        if cached_tokens:
            self.hits += 1
        need = self.blocks_needed(len(tokens)) - len(table)
        if need > self.num_free:
            for b in table:
                self._release(b)
            raise NoFreeBlocks()
        for _ in range(need):
            b = self._pop_free()
            self._acquire(b)
            table.append(b)
        return table, cached_tokens, hashes

    def register_computed(self, table: List[int], tokens: Sequence[int], hashes: List[int]) -> None:
        """After a prefill, publish the sequence's newly completed full blocks to the prefix cache."""
        if not self.prefix_caching:
            return
        bs = self.block_size
        parent = hashes[-1] if hashes else 0
        for i in range(len(hashes), len(tokens) // bs):
            h = self.chain_hash(parent, tokens[i * bs:(i + 1) * bs])
            b = table[i]
            hashes.append(h)
            parent = h
            if h not in self.cached and self.block_hash[b] is None:
                self.cached[h] = b
                self.block_hash[b] = h
                self.parent_of[b] = hashes[-2] if len(hashes) > 1 else 0
                self.block_toks[b] = tuple(tokens[i * bs:(i + 1) * bs])
                self.children.setdefault(self.parent_of[b], collections.deque(maxlen=4)).append(b)

    def reuse_partial(self, table: List[int], tokens: Sequence[int], cached: int,
                      hashes: List[int]) -> Optional[tuple]:
        """Find a published sibling of the first uncached block sharing a token prefix with it.

        Returns (src_block, r): the caller copies src's KV into table[cached // bs] and treats the
        first r tokens of that block as computed; src is pinned until `unpin(src)`."""
        if not self.prefix_caching:
            return None
        bs = self.block_size
        maxr = min(bs, len(tokens) - 1 - cached)
        if maxr <= 0:
            return None
        parent = hashes[-1] if hashes else 0
        want = tokens[cached:cached + maxr]
        best, best_r = -1, 0
        for b in self.children.get(parent, ()):
            if self.block_hash[b] is None or self.parent_of[b] != parent:
                continue   # evicted (or re-published elsewhere) since it was indexed
            bt = self.block_toks[b]
            r = 0
            while r < maxr and bt[r] == want[r]:
                r += 1
            if r > best_r:
                best, best_r = b, r
        if best_r == 0:
            return None
        self._acquire(best)
        self.partial_tokens += best_r
        return best, best_r

    def unpin(self, b: int) -> None:
        self._release(b)

    def ensure_capacity(self, table: List[int], num_tokens: int) -> None:
        """Grow a table so that it can hold `num_tokens` tokens (decode appends); all or nothing."""
        if self.blocks_needed(num_tokens) - len(table) > self.num_free:
            raise NoFreeBlocks()
        while len(table) * self.block_size < num_tokens:
            b = self._pop_free()
            self._acquire(b)
            table.append(b)

    def free_table(self, table: List[int]) -> None:
        for b in table:
            self._release(b)
        table.clear()

    def reset_prefix_cache(self) -> None:
        for b in list(self.evictable):
            self._unhash(b)
            self.free.append(b)
        self.evictable.clear()
        self.cached = {h: b for h, b in self.cached.items() if self.ref[b] > 0}


def make_block_manager(num_blocks: int, block_size: int = 16, enable_prefix_caching: bool = True):
    """The C++ allocator (runtime/native.cpp) when built, else this Python reference."""
    try:
        from ..runtime.native import NativeBlockManager, available
        if available():
            return NativeBlockManager(num_blocks, block_size, enable_prefix_caching)
    except ImportError:
        pass
    return BlockManager(num_blocks, block_size, enable_prefix_caching)
