"""Host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The native runtime core (`ai_agent_kubectl_amd/runtime/runtime.h`: tokenizer trie, paged-KV block
manager) is compiled into a standalone stress driver (`tests/native/test_runtime.cpp`) with
`-fsanitize=address,undefined -fno-sanitize-recover=all` and run on the CPU.  The pybind11 module
is not loaded into an instrumented interpreter (that needs libasan preloaded into python); the
driver exercises the same classes directly.  GPU sanitizers are not available on this pool.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_native_runtime_asan_ubsan(tmp_path):
    exe = tmp_path / "test_runtime"
    src = os.path.join(ROOT, "tests", "native", "test_runtime.cpp")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", src, "-o", str(exe)], check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native runtime OK" in r.stdout


def _churn(bm, n_prompts=3000, bs=4):
    """Distinct prompts sharing an instruction prefix, each finished right after its prefill."""
    instr = list(range(11, 20))
    for i in range(n_prompts):
        toks = instr + [1000 + i * 7 + k for k in range(9)]
        table, cached, hashes = bm.allocate_prompt(toks)
        bm.register_computed(table, toks, hashes)
        bm.free_table(table)
    return bm


@pytest.mark.parametrize("native", [False, True])
def test_sibling_index_bounded(native):
    """The sub-block-reuse sibling index drops evicted blocks: it cannot grow with the number of
    distinct prompts served (it did before: one key per distinct parent hash, forever)."""
    from ai_agent_kubectl_amd.engine.block_manager import BlockManager
    if native:
        from ai_agent_kubectl_amd.runtime.native import NativeBlockManager, available
        if not available():
            pytest.skip("native runtime not built")
        bm = NativeBlockManager(num_blocks=32, block_size=4)
    else:
        bm = BlockManager(num_blocks=32, block_size=4)
    _churn(bm)
    assert bm.num_index_keys <= 32
    assert bm.num_free == 32
    bm.reset_prefix_cache()
    assert bm.num_index_keys == 0


@pytest.mark.parametrize("native", [False, True])
def test_ensure_capacity_all_or_nothing(native):
    from ai_agent_kubectl_amd.engine.block_manager import BlockManager, NoFreeBlocks
    if native:
        from ai_agent_kubectl_amd.runtime.native import NativeBlockManager, available
        if not available():
            pytest.skip("native runtime not built")
        bm = NativeBlockManager(num_blocks=4, block_size=4, enable_prefix_caching=False)
    else:
        bm = BlockManager(num_blocks=4, block_size=4, enable_prefix_caching=False)
    table, _, _ = bm.allocate_prompt(list(range(6)))     # 2 blocks
    with pytest.raises(NoFreeBlocks):
        bm.ensure_capacity(table, 4 * 5)                  # needs 3 more, 2 free
    assert len(table) == 2 and bm.num_free == 2           # nothing taken by the failed grow
    bm.free_table(table)
    assert bm.num_free == 4
