"""CPU contracts of the op layer's dispatch helpers (the GPU kernels are in test_kernels_gpu.py)."""
import torch

from ai_agent_kubectl_amd import ops
from ai_agent_kubectl_amd.ops import reference as ref


def test_linear_swiglu_cpu_is_reference():
    torch.manual_seed(0)
    x = torch.randn(9, 256, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * 128, 256) / 16).to(torch.bfloat16)
    y = ops.linear_swiglu(x, w13)
    torch.testing.assert_close(y.float(), ref.silu_mul(ref.linear(x, w13)).float())
    assert not ops.use_prefill_swiglu(x, w13)   # CPU tensors never take the HIP path


def test_linear_gm_swiglu_cpu_is_reference():
    torch.manual_seed(0)
    x = torch.randn(40, 256, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * 64, 256) / 16).to(torch.bfloat16)
    torch.testing.assert_close(ops.linear_gm_swiglu(x, w13, 2).float(), ref.silu_mul(ref.linear(x, w13)).float())
    saved = dict(ops.DECODE_SWIGLU_CFG)
    ops.DECODE_SWIGLU_CFG[40] = 2
    try:
        assert ops.decode_swiglu_cfg(x, w13) == 0   # CPU tensors never take the HIP path
    finally:
        ops.DECODE_SWIGLU_CFG.clear()
        ops.DECODE_SWIGLU_CFG.update(saved)
    assert ops.decode_swiglu_ok(x, w13)
    assert ops.decode_swiglu_ok(x[:16], w13) and ops.decode_swiglu_ok(x[:4], w13)   # M < 8: tune_swiglu decides
    assert not ops.decode_swiglu_ok(x, torch.zeros(2 * 56, 256, dtype=torch.bfloat16))   # I % 16


def test_gemv_rows_rules_and_cpu_reference():
    assert ops.rows_ok(1, 4096, 1) and ops.rows_ok(4, 14336, 4) and ops.rows_ok(1, 14336, 1)
    assert ops.rows_ok(5, 4096, 1) and ops.rows_ok(16, 4096, 2)   # 8 / 16 staged rows
    assert not ops.rows_ok(16, 4096, 1)           # 16 x 4096 x 2 B: over the 64 KB LDS budget
    assert not ops.rows_ok(17, 4096, 4)           # M > 16: tiled kernels
    assert not ops.rows_ok(4, 14336, 1)           # X slice over the 64 KB LDS budget
    assert not ops.rows_ok(1, 4096, 3)            # K % (512 * split)
    x = torch.randn(2, 1024, dtype=torch.bfloat16)
    w = (torch.randn(96, 1024) / 32).to(torch.bfloat16)
    torch.testing.assert_close(ops.linear_rows(x, w, 2, 4).float(), ref.linear(x, w).float())


def test_swiglu_gemm_shape_rules():
    x = torch.zeros(2048, 4096, dtype=torch.bfloat16)
    assert ops.swiglu_gemm_ok(x, torch.zeros(2 * 14336, 4096, dtype=torch.bfloat16))
    assert not ops.swiglu_gemm_ok(x, torch.zeros(2 * 14336 + 128, 4096, dtype=torch.bfloat16))
    assert not ops.swiglu_gemm_ok(x[:, :4000], torch.zeros(256, 4000, dtype=torch.bfloat16))


def test_argmax_combine_reference_ties_lowest_id():
    """TP vocab-parallel combine (A3): the largest gathered value wins, the lowest global id on ties."""
    vals = torch.tensor([[1.0, 5.0, 2.0], [3.0, 5.0, 2.0], [3.0, 1.0, 7.0]])
    idxs = torch.tensor([[10, 11, 12], [1000, 1001, 1002], [2000, 2001, 2002]], dtype=torch.int32)
    assert ops.argmax_combine(vals, idxs).tolist() == [1000, 11, 2002]


def test_shared_prefix_len():
    """engine/runner.py shared_prefix_len: the leading block-table columns every row shares, capped."""
    import numpy as np
    from ai_agent_kubectl_amd.engine.runner import shared_prefix_len
    bt = np.array([[1, 2, 3, 9, 0], [1, 2, 3, 7, 8], [1, 2, 4, 5, 6]], dtype=np.int32)
    assert shared_prefix_len(bt, 5) == 2
    assert shared_prefix_len(bt[:2], 5) == 3
    assert shared_prefix_len(bt[:2], 2) == 2
    assert shared_prefix_len(bt[:1], 4) == 4
    assert shared_prefix_len(bt, 0) == 0
    assert shared_prefix_len(np.array([[5, 1], [6, 1]], dtype=np.int32), 2) == 0


def test_plan_for_takes_the_next_bucket_up():
    """ops.plan_for: exact (M, N, K) entries first; an un-timed row count (a mixed step of 300 rows)
    takes the smallest planned bucket above it; none past the largest bucket; a batch-1..4 GEMV
    plan ("rows") only where its row rule holds."""
    saved = dict(ops.GEMM_PLAN)
    try:
        ops.GEMM_PLAN.clear()
        ops.GEMM_PLAN[(256, 64, 128)] = ("gm", 4, 12)
        ops.GEMM_PLAN[(320, 64, 128)] = ("blas", 0, 0)
        ops.GEMM_PLAN[(512, 64, 128)] = ("gm", 2, 3)
        ops.GEMM_PLAN[(4, 64, 4096)] = ("rows", 2, 4)
        assert ops.plan_for(256, 64, 128) == ("gm", 4, 12)
        assert ops.plan_for(200, 64, 128) == ("gm", 4, 12)
        assert ops.plan_for(300, 64, 128) == ("blas", 0, 0)
        assert ops.plan_for(321, 64, 128) == ("gm", 2, 3)
        assert ops.plan_for(513, 64, 128) is None
        assert ops.plan_for(300, 96, 128) is None
        assert ops.plan_for(3, 64, 4096) == (("rows", 2, 4) if ops.rows_ok(3, 4096, 2) else None)
        ops.GEMM_PLAN[(384, 64, 128)] = ("gm", 4, 3)   # the lookup table follows new entries
        assert ops.plan_for(321, 64, 128) == ("gm", 4, 3)
    finally:
        ops.GEMM_PLAN.clear()
        ops.GEMM_PLAN.update(saved)


def test_lgkm_window_checker_flags_compiler_lgkm_ops():
    """build.py re-verifies that no compiler-issued LGKM operation sits between the
    k-loop's asm fragment reads and their counted lgkmcnt wait (gemm_mfma KA_GM_PIPE 2, gemm_big)."""
    from ai_agent_kubectl_amd.build import lgkm_window_violations
    ok = """_ZN2gm11gemm_kernelI1EEvNS_4ArgsE:
\t;;#ASMSTART
\tds_read_b128 v[0:3], v10 offset:0
\t;;#ASMEND
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(4)
\t;;#ASMEND
\ts_load_dword s4, s[0:1], 0x10
\tds_write_b32 v1, v2
"""
    n, bad = lgkm_window_violations(ok, "gemm_kernel")
    assert n == 1 and bad == []
    broken = ok.replace("\tv_mfma", "\ts_load_dwordx2 s[6:7], s[0:1], 0x8\n\tv_mfma")
    n, bad = lgkm_window_violations(broken, "gemm_kernel")
    assert n == 1 and len(bad) == 1 and "s_load_dwordx2" in bad[0][2]
    assert lgkm_window_violations(broken, "other_kernel") == (0, [])


def test_plan_ladder_anomalies_flags_slower_smaller_bucket():
    """a bucket whose planned GEMM time exceeds the next larger bucket's (whose
    plan also runs the smaller M) is a tuning miss; ladder_anomalies finds it per (N, K, consumer)."""
    from ai_agent_kubectl_amd.ops.autotune import ladder_anomalies
    plans = {"4,28672,4096,plain": ["skinny", 1, 0, 47.8, 49.2], "8,28672,4096,plain": ["gm", 1, 5, 42.2, 50.0],
             "16,28672,4096,plain": ["gm", 1, 5, 42.4, 49.6], "8,4096,4096,norm": ["gm", 8, 5, 13.8, 31.9],
             "16,4096,4096,norm": ["gm", 8, 5, 13.5, 27.5]}
    bad = ladder_anomalies(plans)
    assert [b[0] for b in bad] == ["4,28672,4096,plain"]
    assert ladder_anomalies(plans, tol=0.2) == []


def test_repair_ladder_takes_the_larger_buckets_plan():
    """Entries left by an earlier run with another bucket subset: a bucket slower than the next larger
    one takes its plan (chained from the largest down); a hipBLASLt plan is never propagated."""
    from ai_agent_kubectl_amd.ops.autotune import ladder_anomalies, repair_ladder
    plans = {"32,32000,4096,plain": ["gm", 2, 4, 45.8, 52.6, 45.8], "48,32000,4096,plain": ["gm", 1, 4, 44.9, 53.0, 44.9],
             "64,32000,4096,plain": ["gm", 1, 5, 40.0, 55.7, 40.0], "1,4096,4096,norm": ["skinny", 4, 0, 9.0, 20.0, 9.0],
             "2,4096,4096,norm": ["rows", 1, 2, 7.0, 20.0, 7.0], "16,4096,4096,norm": ["rows", 1, 1, 7.5, 20.0, 7.5],
             "32,4096,4096,norm": ["blas", 0, 0, 5.0, 5.0, 9.0]}
    changed = repair_ladder(plans)
    assert sorted(changed) == ["1,4096,4096,norm", "32,32000,4096,plain", "48,32000,4096,plain"]
    assert plans["32,32000,4096,plain"][:4] == ["gm", 1, 5, 40.0] and plans["32,32000,4096,plain"][4] == 52.6
    assert plans["2,4096,4096,norm"][0] == "rows" and plans["1,4096,4096,norm"][:3] == ["rows", 1, 2]
    assert [a[0] for a in ladder_anomalies(plans)] == ["16,4096,4096,norm"]   # blas above: left alone


def test_mfma_span_valu_checker():
    """build.py refuses a gemm_big build whose all-asm k-loop got a compiler VALU instruction between
    asm MFMAs (a WAR hazard on operands hipcc cannot see being read)."""
    from ai_agent_kubectl_amd.build import mfma_span_valu
    ok = """_ZN2gb14gemm256_kernelILi3ELi8EEEvNS_4ArgsE:
\tv_mov_b32 v1, 0
\t;;#ASMSTART
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[56:59], v[4:7], a[0:3]
\t;;#ASMEND
\ts_and_b64 vcc, exec, s[4:5]
\t;;#ASMSTART
\tv_mfma_f32_16x16x32_bf16 a[4:7], v[56:59], v[8:11], a[4:7]
\t;;#ASMEND
\tv_add_u32 v2, v1, v3
"""
    assert mfma_span_valu(ok, "gemm256_kernel") == []
    bad = ok.replace("\ts_and_b64", "\tv_cndmask_b32_e64 v56, 0, 1, s[58:59]\n\ts_and_b64")
    got = mfma_span_valu(bad, "gemm256_kernel")
    assert len(got) == 1 and "v_cndmask" in got[0][2]


def test_prefill_gemm_plan_buckets():
    """ops.PREFILL_GEMM auto: a prefill row count takes the decision of the smallest timed bucket at or
    above it (the largest one beyond); CPU tensors always run the fp32 reference."""
    import torch
    from ai_agent_kubectl_amd import ops
    assert ops.prefill_bucket(600) == 1024 and ops.prefill_bucket(4080) == 4096
    assert ops.prefill_bucket(4097) == 6144 and ops.prefill_bucket(20000) == 8192
    x = torch.zeros(4096, 256, dtype=torch.bfloat16)
    w = torch.zeros(512, 256, dtype=torch.bfloat16)
    ops.PREFILL_PLAN[(4096, 512, 256)] = True
    try:
        assert not ops.use_big_gemm(x, w)   # CPU: reference path
    finally:
        ops.PREFILL_PLAN.pop((4096, 512, 256))


def test_hip_lib_override_needs_the_diag_flag():
    """an experimental kernel library (KA_HIP_LIB) is loaded only for an explicit
    diagnostic run; a stray KA_HIP_LIB alone makes the import fail loudly instead of switching builds."""
    import os
    import subprocess
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import ai_agent_kubectl_amd.ops._hip as h; print(h.LIB_PATH)"
    env = dict(os.environ, KA_HIP_LIB="/tmp/elsewhere/libkagent_hip.so")
    env.pop("KA_HIP_LIB_DIAG", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT)
    assert r.returncode != 0 and "KA_HIP_LIB_DIAG" in r.stderr
    env["KA_HIP_LIB_DIAG"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip() == "/tmp/elsewhere/libkagent_hip.so"
    env = dict(os.environ)
    env.pop("KA_HIP_LIB", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().endswith("ops/lib/libkagent_hip.so")
