"""HIP kernel numerics vs plain-PyTorch fp32 references (SURVEY.md §4.3 'kernel (GPU)' row).

Every test asserts the HIP library is the code that ran (ops dispatch CUDA tensors to it and raises
if it is missing).  Shapes cover the real head geometry (D=128, block 16), GQA 4 and 8, varlen
prefill with cached context, and padding rows.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU with -m "not gpu" deselected anyway
    pytest.skip("no GPU", allow_module_level=True)

from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.ops import _hip, reference as ref  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


@pytest.fixture(autouse=True, scope="module")
def _lib():
    _hip.require()
    torch.manual_seed(0)


def close(a, b, atol, rtol=0.02):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


@pytest.mark.parametrize("rows,hidden", [(1, 4096), (37, 4096), (5, 8192), (3, 256)])
def test_rmsnorm(rows, hidden):
    x = torch.randn(rows, hidden, device=DEV, dtype=BF)
    w = (1 + 0.1 * torch.randn(hidden, device=DEV)).to(BF)
    close(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x, w, 1e-5), atol=2e-2)
    res = torch.randn(rows, hidden, device=DEV, dtype=BF)
    res2 = res.clone()
    y = ops.rmsnorm(x, w, 1e-5, residual=res)
    y2 = ref.rmsnorm(x, w, 1e-5, residual=res2)
    close(res, res2, atol=1e-2)
    close(y, y2, atol=3e-2)


def _cache(nb, hkv, bs=16, d=128):
    k = torch.randn(nb, hkv, bs, d, device=DEV, dtype=BF)
    v = torch.randn(nb, hkv, d, bs, device=DEV, dtype=BF)
    return k, v


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 1), (48, 12)])
@pytest.mark.parametrize("T", [23, 301])
def test_rope_kv_write(hq, hkv, T):
    """T >= 64 takes the 16-token window kernel (V transposed through LDS, one kv head at a time)."""
    d = 128
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=DEV, dtype=BF)
    cs = ref.rope_cos_sin(4096, d, 5e5, device=DEV)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    perm = torch.randperm(64 * 16)
    if T > 64:   # unique slots with a run of 100 consecutive ones (straddling blocks) at rows 40..139
        run = torch.arange(333, 433)
        rest = perm[~torch.isin(perm, run)]
        perm = torch.cat([rest[:40], run, rest[40:]])
    slots = perm[:T].to(DEV, torch.int32)
    slots[3] = -1
    k1, v1 = _cache(64, hkv)
    k2, v2 = k1.clone(), v1.clone()
    q1 = ops.rope_kv_write(qkv, pos, cs, slots, k1, v1, hq, hkv, d)
    q2 = ref.rope_kv_write(qkv, pos, cs, slots, k2, v2, hq, hkv, d)
    close(q1, q2, atol=2e-2)
    close(k1, k2, atol=2e-2)
    assert torch.equal(v1, v2)


def _tables(S, ctx_lens, nb_total, max_blocks, bs=16):
    perm = torch.randperm(nb_total).tolist()
    bt = torch.zeros(S, max_blocks, dtype=torch.int32)
    k = 0
    for s, c in enumerate(ctx_lens):
        n = (c + bs - 1) // bs
        bt[s, :n] = torch.tensor(perm[k:k + n], dtype=torch.int32)
        k += n
    return bt.to(DEV)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (4, 1)])
@pytest.mark.parametrize("ctx_lens", [[1, 17, 100, 129], [2048], [31, 32, 33]])
def test_paged_decode(hq, hkv, ctx_lens):
    S = len(ctx_lens)
    kc, vc = _cache(400, hkv)
    bt = _tables(S, ctx_lens, 400, 160)
    q = torch.randn(S, hq, 128, device=DEV, dtype=BF)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)
    scale = 128 ** -0.5
    close(ops.attention_decode(q, kc, vc, bt, ctx, scale), ref.attention_decode(q, kc, vc, bt, ctx, scale), atol=2e-2)


@pytest.mark.parametrize("S,hq", [(80, 32), (160, 32), (160, 64)])
def test_paged_decode_large_batch_mixed_lengths(S, hq):
    """S sequences of mixed lengths, a padding row (ctx 0 -> zeros) and a 1000-token context whose
    chunks each wave walks in several passes; S * hkv > 1024 takes the 2-wave workgroups."""
    import random
    rng = random.Random(0)
    hkv = 8
    ctx_lens = [rng.randint(1, 300) for _ in range(S)]
    ctx_lens[5] = 0
    ctx_lens[7] = 1000
    nb = 2000
    kc, vc = _cache(nb, hkv)
    bt = _tables(S, ctx_lens, nb, 64)
    q = torch.randn(S, hq, 128, device=DEV, dtype=BF)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)
    got = ops.attention_decode(q, kc, vc, bt, ctx, 128 ** -0.5)
    want = ref.attention_decode(q, kc, vc, bt, ctx, 128 ** -0.5)
    close(got, want, atol=2e-2)
    assert got[5].abs().max().item() == 0


def test_paged_decode_padding_rows_zero():
    kc, vc = _cache(8, 8)
    bt = torch.zeros(2, 4, dtype=torch.int32, device=DEV)
    q = torch.randn(2, 32, 128, device=DEV, dtype=BF)
    ctx = torch.tensor([5, 0], dtype=torch.int32, device=DEV)
    out = ops.attention_decode(q, kc, vc, bt, ctx, 0.088)
    assert torch.isfinite(out.float()).all()
    assert out[1].abs().max().item() == 0


@pytest.mark.parametrize("hq,hkv,reps", [(32, 8, 1), (64, 8, 1), (4, 1, 1), (32, 8, 23), (64, 8, 23)])
@pytest.mark.parametrize("split", [0, 1, 4, 6, -1, -4, -6])
@pytest.mark.parametrize("tight", [False, True])
def test_decode_attention_rope_fused(hq, hkv, reps, split, tight):
    """RoPE + KV append + paged decode in one kernel == rope_kv_write then attention_decode (fp32
    torch references), on bf16 qkv and on split-K partials (6: past the prologue's 4 unrolled
    slices); cache contents identical to the unfused kernels'; a padding row (slot -1, ctx 0) writes
    nothing and returns zeros.  reps = 23: 162 rows x 8 kv heads > 1024 workgroups, the 2-wave
    variant.  tight: the block table is exactly as wide as the longest context needs (9
    blocks for 137 tokens), so the 137-token rows' last chunk, which ends in its first block, reads
    its clamped second table entry inside the row."""
    d, nb = 128, 400 * reps
    ctx_lens = [1, 2, 17, 100, 129, 33, 137] * reps + [0]
    S = len(ctx_lens)
    bt = _tables(S, ctx_lens, nb, (max(ctx_lens) + 15) // 16 if tight else 16)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)
    btc = bt.cpu()
    slots = torch.tensor([int(btc[s, (c - 1) // 16]) * 16 + (c - 1) % 16 if c > 0 else -1
                          for s, c in enumerate(ctx_lens)], dtype=torch.int32, device=DEV)
    pos = (ctx - 1).clamp(min=0)
    cs = ref.rope_cos_sin(4096, d, 5e5, device=DEV)
    width = (hq + 2 * hkv) * d
    if split:   # split < 0: bf16 partials (gemm_mfma EPI_P16), summed in fp32 by the prologue
        sp = abs(split)
        P = torch.randn(sp, S, width, device=DEV)
        qkv = ops.SplitK(P.to(BF) if split < 0 else P, sp)
        P0 = qkv.P[0].float().clone()
        for k in range(1, sp):
            P0 += qkv.P[k].float()
        qkv_bf = P0.to(BF)                                   # the kernels' summation order
    else:
        qkv = qkv_bf = torch.randn(S, width, device=DEV, dtype=BF)
    k1, v1 = _cache(nb, hkv)
    k2, v2 = k1.clone(), v1.clone()
    scale = d ** -0.5
    got = ops.decode_attention_rope(qkv, pos, cs, slots, k1, v1, bt, ctx, hq, hkv, d, scale)
    q = ops.rope_kv_write(qkv_bf, pos, cs, slots, k2, v2, hq, hkv, d)
    want = ref.attention_decode(q, k2, v2, bt, ctx, scale)
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    close(got, want, atol=2e-2)
    assert got[-1].abs().max().item() == 0


@pytest.mark.parametrize("hq,hkv,ns", [(32, 8, 5), (32, 8, 1), (32, 8, 0), (64, 8, 6), (8, 8, 4), (16, 8, 3)])
@pytest.mark.parametrize("S", [33, 256])
def test_decode_attention_rope_cascade(hq, hkv, ns, S):
    """Cascade decode attention (the first ns blocks of every row's table are the same physical
    blocks, attended once by cascade_prefix_kernel and merged) == the plain fused kernel == the fp32
    reference, including rows whose own part is only the new token, a padding row, and ns = 0 (the
    second kernel returns at once)."""
    import random
    rng = random.Random(ns * 7 + S)
    d, nb = 128, 5000
    k1, v1 = _cache(nb, hkv)
    k2, v2 = k1.clone(), v1.clone()
    shared = list(range(1, ns + 1))                       # physical blocks 1 .. ns
    ctx_lens, rows = [], []
    free = ns + 1
    for s in range(S - 1):
        own_tok = rng.choice([1, 1, 2, 16, 17, 40, 100])     # incl. the new token
        c = ns * 16 + own_tok
        n_own = (c + 15) // 16 - ns
        rows.append(shared + list(range(free, free + n_own)))
        free += n_own
        ctx_lens.append(c)
    rows.append([0])                                      # padding row
    ctx_lens.append(0)
    mb = max(len(r) for r in rows)
    bt = torch.zeros(S, mb, dtype=torch.int32)
    for i, r in enumerate(rows):
        bt[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
    bt = bt.to(DEV)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)
    btc = bt.cpu()
    slots = torch.tensor([int(btc[s, (c - 1) // 16]) * 16 + (c - 1) % 16 if c > 0 else -1
                          for s, c in enumerate(ctx_lens)], dtype=torch.int32, device=DEV)
    pos = (ctx - 1).clamp(min=0)
    cs = ref.rope_cos_sin(4096, d, 5e5, device=DEV)
    qkv = torch.randn(S, (hq + 2 * hkv) * d, device=DEV, dtype=BF)
    nsh = torch.tensor([ns], dtype=torch.int32, device=DEV)
    scale = d ** -0.5
    got = ops.decode_attention_rope(qkv, pos, cs, slots, k1, v1, bt, ctx, hq, hkv, d, scale, shared_blocks=nsh)
    plain = ops.decode_attention_rope(qkv, pos, cs, slots, k2, v2, bt, ctx, hq, hkv, d, scale)
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    q = ops.rope_kv_write(qkv, pos, cs, slots, k2.clone(), v2.clone(), hq, hkv, d)
    want = ref.attention_decode(q, k2, v2, bt, ctx, scale)
    close(got[:-1], want[:-1], atol=2e-2)
    close(got[:-1], plain[:-1], atol=2e-2)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 8)])
@pytest.mark.parametrize("qlens,ctxs", [([90], [90]), ([7, 1, 33, 20], [71, 130, 33, 84]), ([130, 1], [130, 5])])
def test_paged_prefill(hq, hkv, qlens, ctxs):
    """Varlen paged prefill attention with cached context (prefix hits / chunked prefill)."""
    S = len(qlens)
    kc, vc = _cache(200, hkv)
    bt = _tables(S, ctxs, 200, 16)
    T = sum(qlens)
    q = torch.randn(T, hq, 128, device=DEV, dtype=BF)
    starts = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    scale = 128 ** -0.5
    got = ops.attention_prefill(q, kc, vc, bt, starts, ctx, max(qlens), scale)
    want = ref.attention_prefill(q, kc, vc, bt, starts, ctx, scale)
    close(got, want, atol=2e-2)


def test_mixed_step_split_attention():
    """Mixed step: leading 1-token decode rows through the decode kernel, prompt rows through the
    varlen prefill kernel (subset metadata, absolute q_starts, shared output) == reference."""
    hq, hkv = 32, 8
    qlens, ctxs = [1, 1, 1, 30, 17], [40, 93, 7, 30, 81]
    S, nd = len(qlens), 3
    kc, vc = _cache(200, hkv)
    bt = _tables(S, ctxs, 200, 16)
    T = sum(qlens)
    q = torch.randn(T, hq, 128, device=DEV, dtype=BF)
    starts = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    scale = 128 ** -0.5
    out = ops.attention_prefill(q, kc, vc, bt[nd:], starts[nd:], ctx[nd:], max(qlens), scale,
                                out=torch.empty_like(q))
    ops.attention_decode(q[:nd], kc, vc, bt[:nd], ctx[:nd], scale, out=out[:nd])
    close(out, ref.attention_prefill(q, kc, vc, bt, starts, ctx, scale), atol=2e-2)


def test_prefill_spike_forces_rescale():
    # spike one key late in the context so the running max jumps at a later tile (guide §5.4 rule 26)
    hq, hkv = 32, 8
    kc, vc = _cache(32, hkv)
    kc *= 0.1
    bt = _tables(1, [200], 32, 16)
    q = torch.randn(40, hq, 128, device=DEV, dtype=BF)
    blk = bt[0, 190 // 16].item()
    kc[blk, :, 190 % 16, :] = q[-1, ::4, :] * 4  # aligns with the last query's heads
    starts = torch.tensor([0, 40], dtype=torch.int32, device=DEV)
    ctx = torch.tensor([200], dtype=torch.int32, device=DEV)
    got = ops.attention_prefill(q, kc, vc, bt, starts, ctx, 40, 128 ** -0.5)
    want = ref.attention_prefill(q, kc, vc, bt, starts, ctx, 128 ** -0.5)
    close(got, want, atol=3e-2)


def test_silu_mul_and_embedding():
    gu = torch.randn(19, 2 * 14336, device=DEV, dtype=BF)
    close(ops.silu_mul(gu), ref.silu_mul(gu), atol=2e-2)
    table = torch.randn(1000, 4096, device=DEV, dtype=BF)
    ids = torch.tensor([0, 5, 999, 1000, -1], dtype=torch.int32, device=DEV)
    assert torch.equal(ops.embedding(ids, table), ref.embedding(ids, table))


@pytest.mark.parametrize("B", [1, 9, 200])
@pytest.mark.parametrize("V,off", [(128256, 0), (16032, 16032 * 3), (32000, 0)])
def test_masked_argmax(V, off, B):
    """B < 128 takes the sliced two-stage path (ka_argmax_slices), B = 200 one workgroup per row."""
    import numpy as np
    logits = torch.randn(B, V, device=DEV, dtype=BF)
    words = (V + off + 31) // 32
    bits = torch.from_numpy(np.random.RandomState(0).randint(0, 2**32, size=(2, words), dtype=np.uint64)
                            .astype(np.uint32).view(np.int32)).to(DEV)
    midx = torch.tensor([0, 1, -1, 0, 1, -1, 0, 0, 1] * (B // 9 + 1), dtype=torch.int32, device=DEV)[:B]
    i1, v1 = ops.masked_argmax(logits, bits, midx, vocab_offset=off)
    i2, v2 = ref.masked_argmax(logits.cpu(), bits.cpu(), midx.cpu(), vocab_offset=off)
    assert torch.equal(i1.cpu(), i2.cpu())
    close(v1, v2, atol=0, rtol=0)


@pytest.mark.parametrize("B", [1, 3, 130])
def test_masked_argmax_ties_lowest_index(B):
    """Equal maxima in different workgroup slices: the lowest token id wins (torch.argmax rule)."""
    V = 128256
    logits = torch.zeros(B, V, device=DEV, dtype=BF)
    for i, pos in enumerate((100000, 70000, 9000)):
        logits[:, pos] = 5.0
    logits[0, 127000] = 5.0
    idx, val = ops.masked_argmax(logits, None, None)
    assert idx.cpu().tolist() == [9000] * B and val.cpu().tolist() == [5.0] * B


@pytest.mark.parametrize("M", [1, 7, 64, 200, 256, 300])
@pytest.mark.parametrize("off", [0, 64128])
def test_lm_head_argmax_vs_fp32(M, off):
    """Fused LM head + masked argmax (csrc/gemm_big.hip EPI_ARGMAX): the chosen token is allowed by
    the row's mask and its fp32 reference logit is the row's allowed maximum up to bf16 rounding;
    vocab_offset = the second TP=2 shard's (the mask is indexed by the global token id)."""
    import numpy as np
    V, K = 64128, 4096
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(V, K, device=DEV) * 0.02).to(BF)
    words = (V + off + 31) // 32
    bits = torch.from_numpy(np.random.RandomState(1).randint(0, 2**32, size=(2, words), dtype=np.uint64)
                            .astype(np.uint32).view(np.int32)).to(DEV)
    midx = torch.tensor([0, 1, -1] * (M // 3 + 1), dtype=torch.int32, device=DEV)[:M]
    idx, val = ops.lm_head_argmax(x, w, bits, midx, vocab_offset=off)
    ref_logits = (x.float() @ w.float().t()).cpu()
    allowed = torch.ones(M, V, dtype=torch.bool)
    b = bits.cpu().view(torch.int32).numpy().view(np.uint32)
    gid = np.arange(V) + off
    for r in range(M):
        mi = int(midx[r])
        if mi >= 0:
            allowed[r] = torch.from_numpy(((b[mi][gid >> 5] >> (gid & 31)) & 1).astype(bool))
    masked = ref_logits.masked_fill(~allowed, float("-inf"))
    best = masked.max(1).values
    got = idx.cpu().long() - off
    assert ((got >= 0) & (got < V)).all()
    assert allowed.gather(1, got[:, None]).all()
    chosen = ref_logits.gather(1, got[:, None]).squeeze(1)
    bad = ((best - chosen) > 0.02 * best.abs().clamp(min=1.0)).nonzero().flatten().tolist()
    assert not bad, [(r, int(got[r]), float(chosen[r]), float(best[r]), int(masked[r].argmax())) for r in bad[:8]]
    close(val, chosen, atol=0.05, rtol=0.02)


def test_lm_head_argmax_ties_lowest_index():
    """Equal maxima in different 256-token tiles and waves: the lowest token id wins."""
    V, K, M = 128256, 4096, 130
    v = torch.randn(K, device=DEV)
    x = v.to(BF).expand(M, K).contiguous()
    w = (torch.randn(V, K, device=DEV) * 0.001).to(BF)
    for j in (70000, 300, 9000, 300 + 128):
        w[j] = (v * 0.05).to(BF)
    idx, _ = ops.lm_head_argmax(x, w, None, None)
    assert idx.cpu().tolist() == [300] * M


@pytest.mark.parametrize("M,I,K", [(1024, 14336, 4096), (2944, 1792, 4096), (777, 512, 256), (4096, 3584, 4096)])
def test_prefill_swiglu_gemm_vs_fp32(M, I, K):
    """Prefill gate_up with the SwiGLU epilogue (csrc/gemm_big.hip EPI_SWIGLU) against the fp32
    silu(x gate^T) * (x up^T): full Llama-3-8B I, the TP=8 shard (1792), a ragged M tail."""
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w13 = (torch.randn(2 * I, K, device=DEV) / math.sqrt(K)).to(BF)
    y = ops.linear_swiglu(x, w13)
    assert y.shape == (M, I)
    g = x.float() @ w13[:I].float().t()
    u = x.float() @ w13[I:].float().t()
    close(y, torch.nn.functional.silu(g) * u, atol=2e-2, rtol=2e-2)


def test_prefill_swiglu_used_by_model_path():
    """The model's MLP takes the fused kernel for prefill-sized steps (ops.use_prefill_swiglu)."""
    x = torch.randn(max(ops.PREFILL_SWIGLU_MIN_M, ops.TILE_MAX_M + 1), 4096, device=DEV, dtype=BF)
    w13 = torch.zeros(2 * 14336, 4096, device=DEV, dtype=BF)
    assert ops.use_prefill_swiglu(x, w13) == ops.PREFILL_SWIGLU
    assert not ops.use_prefill_swiglu(x[:256], w13)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8, 12, 16])
@pytest.mark.parametrize("N,K,split,rw", [(6144, 4096, 2, 8), (4100, 4096, 1, 4), (28672, 4096, 1, 4),
                                          (1000, 14336, 4, 2), (300, 2048, 4, 1), (128256, 4096, 2, 4)])
def test_gemv_rows_vs_fp32(M, N, K, split, rw):
    """Row-streaming GEMV (csrc/gemm_skinny.hip gemv_rows_kernel): bf16 output and deferred fp32
    partials against fp32 x @ w^T, ragged N (rows past N in the last wave); M 5..16 stage 8 / 16 X
    rows (decode buckets 8 and 16)."""
    if not ops.rows_ok(M, K, split):
        pytest.skip("X slice over the LDS budget for this split")
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
    want = x.float() @ w.float().t()
    close(ops.linear_rows(x, w, split, rw), want, atol=2e-2, rtol=2e-2)
    if split > 1:
        p = ops.linear_rows(x, w, split, rw, defer_reduce=True)
        assert isinstance(p, ops.SplitK)
        close(p.P.sum(0), want, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M", [1, 4, 8])
def test_gemv_rows_swiglu_down_vs_fp32(M):
    """Batch-1..4 down projection with SiLU·mul in the row-streaming GEMV's X staging."""
    I, N = 14336, 4096
    gu = torch.randn(M, 2 * I, device=DEV, dtype=BF)
    w = (torch.randn(N, I, device=DEV) / math.sqrt(I)).to(BF)
    act = torch.nn.functional.silu(gu[:, :I].float()) * gu[:, I:].float()
    want = act @ w.float().t()
    close(ops.swiglu_linear(gu, w), want, atol=3e-2, rtol=3e-2)
    p = ops.swiglu_linear(gu, w, defer_reduce=True)
    close(p.P.sum(0) if isinstance(p, ops.SplitK) else p.float(), want, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5, 12])
@pytest.mark.parametrize("M,I", [(1, 1792), (4, 14336), (32, 14336), (100, 1792), (256, 14336), (300, 1792),
                                 (512, 1792)])
def test_decode_swiglu_gemm_vs_fp32(M, I, cfg):
    """Decode gate_up with the gemm_mfma SwiGLU epilogue over the model's [gate; up] weight (the
    weight DMAs gather 16-row gate / up chunks) against fp32 silu(x gate^T) * (x up^T)."""
    K = 4096
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w13 = (torch.randn(2 * I, K, device=DEV) / math.sqrt(K)).to(BF)
    y = ops.linear_gm_swiglu(x, w13, cfg)
    assert y.shape == (M, I)
    g = x.float() @ w13[:I].float().t()
    u = x.float() @ w13[I:].float().t()
    close(y, torch.nn.functional.silu(g) * u, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [160, 256, 320, 512])
def test_decode_swiglu_big_vs_fp32(M):
    """Decode buckets whose SwiGLU plan is csrc/gemm_big.hip (DECODE_SWIGLU_BIG): the model calls
    linear_gm_swiglu with that marker; compared with fp32 silu(x gate^T) * (x up^T)."""
    K, I = 4096, 1792
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w13 = (torch.randn(2 * I, K, device=DEV) / math.sqrt(K)).to(BF)
    y = ops.linear_gm_swiglu(x, w13, ops.DECODE_SWIGLU_BIG)
    assert y.shape == (M, I)
    g = x.float() @ w13[:I].float().t()
    u = x.float() @ w13[I:].float().t()
    close(y, torch.nn.functional.silu(g) * u, atol=2e-2, rtol=2e-2)
    saved = dict(ops.DECODE_SWIGLU_CFG)
    try:
        ops.DECODE_SWIGLU_CFG[M] = ops.DECODE_SWIGLU_BIG
        assert ops.decode_swiglu_cfg(x, w13) == (0 if ops.DECODE_SWIGLU == "0" else ops.DECODE_SWIGLU_BIG)
        # a weight gemm_big's SwiGLU cannot take (2I % 256 != 0) falls back to the unfused path
        assert ops.decode_swiglu_cfg(x, w13[:2 * 1776]) == 0
    finally:
        ops.DECODE_SWIGLU_CFG.clear()
        ops.DECODE_SWIGLU_CFG.update(saved)


@pytest.mark.parametrize("M", [128, 256, 320, 512])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336)])
def test_gemm_plan_big_dispatch(M, N, K):
    """A decode-bucket plan entry "big" sends ops.linear to csrc/gemm_big.hip (with or without
    defer_reduce: it returns the bf16 product, which the fused norm / attention consumers take)."""
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
    want = x.float() @ w.float().t()
    ops.GEMM_PLAN[(M, N, K)] = ("big", 0, 0)
    try:
        close(ops.linear(x, w), want, atol=3e-2, rtol=2e-2)
        y = ops.linear(x, w, defer_reduce=True, bf16_partials=True)
        assert not isinstance(y, ops.SplitK)
        close(y, want, atol=3e-2, rtol=2e-2)
    finally:
        ops.GEMM_PLAN.pop((M, N, K), None)


def test_decode_swiglu_plan_dispatch():
    """ops.decode_swiglu_cfg follows the per-bucket plan and the shape rules."""
    x = torch.randn(256, 4096, device=DEV, dtype=BF)
    w13 = torch.zeros(2 * 14336, 4096, device=DEV, dtype=BF)
    saved = dict(ops.DECODE_SWIGLU_CFG)
    try:
        ops.DECODE_SWIGLU_CFG.clear()
        assert ops.decode_swiglu_cfg(x, w13) == 0
        ops.DECODE_SWIGLU_CFG[256] = 2
        ops.DECODE_SWIGLU_CFG[128] = 0   # timed, unfused won
        on = ops.DECODE_SWIGLU != "0"
        assert ops.decode_swiglu_cfg(x, w13) == (2 if on else 0)
        assert ops.decode_swiglu_cfg(x[:128], w13) == 0
        assert ops.decode_swiglu_cfg(x[:200], w13) == (2 if on else 0)   # un-timed: the next bucket up
        assert ops.decode_swiglu_cfg(x[:100], w13) == 0
        x3 = torch.randn(300, 4096, device=DEV, dtype=BF)
        assert ops.decode_swiglu_cfg(x3, w13) == 0   # above every timed bucket
    finally:
        ops.DECODE_SWIGLU_CFG.clear()
        ops.DECODE_SWIGLU_CFG.update(saved)


def test_moe_topk():
    lg = torch.randn(50, 8, device=DEV, dtype=BF)
    w1, i1 = ops.moe_topk(lg, 2)
    w2, i2 = ref.moe_topk(lg, 2)
    assert torch.equal(i1.cpu().sort(1).values, i2.cpu().sort(1).values)
    close(w1.sort(1).values, w2.sort(1).values, atol=1e-5)


@pytest.mark.parametrize("M", [1, 4, 5, 16, 33, 64, 128, 200, 256])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (16032, 4096), (1000, 512)])
def test_gemm_skinny(M, N, K):
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(BF)
    want = x.float() @ w.float().t()
    for split in (1, 3, 8):
        got = ops.linear(x, w, split=split)
        close(got, want, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("rows,hidden,split", [(1, 4096, 2), (37, 4096, 8), (256, 4096, 4), (5, 8192, 3),
                                               (3, 4096, 12), (2, 1024, 6)])
def test_rmsnorm_fused_splitk_reduce(rows, hidden, split):
    """rmsnorm(SplitK partials, residual) == rmsnorm(bf16(sum partials), residual).  split 12 / 6 go
    past the kernel's unrolled slices (8 at 512 threads, 4 at 256) into its remainder loop."""
    P = torch.randn(split, rows, hidden, device=DEV) * 0.5
    w = (torch.rand(hidden, device=DEV) + 0.5).to(BF)
    res0 = torch.randn(rows, hidden, device=DEV).to(BF)
    r1, r2 = res0.clone(), res0.clone()
    got = ops.rmsnorm(ops.SplitK(P, split), w, 1e-5, residual=r1)
    want = ref.rmsnorm(P.sum(0).to(BF), w, 1e-5, r2)
    close(got, want, atol=2e-2)
    close(r1, r2, atol=1e-2)


@pytest.mark.parametrize("T", [37, 150])
def test_rope_and_silu_consume_splitk_partials_exactly(T):
    """RoPE+KV append and SiLU·mul summing the fp32 split-K partials themselves give bit-identical
    results to the reduce kernel followed by the bf16 op (T = 150: the 16-token window kernel)."""
    hq, hkv, d, split = 32, 8, 128, 4
    P = torch.randn(split, T, (hq + 2 * hkv) * d, device=DEV)
    red = ops.SplitK(P, split).resolve()                         # torch sum in the same order...
    want_bf = P[0].clone()
    for k in range(1, split):
        want_bf += P[k]
    red = want_bf.to(BF)                                         # ...exactly the reduce kernel's order
    cs = ref.rope_cos_sin(4096, d, 5e5, device=DEV)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(64 * 16, device=DEV)[:T].int()
    kc1 = torch.zeros(64, hkv, 16, d, device=DEV, dtype=BF)
    vc1 = torch.zeros(64, hkv, d, 16, device=DEV, dtype=BF)
    kc2, vc2 = kc1.clone(), vc1.clone()
    q1 = ops.rope_kv_write(red, pos, cs, slots, kc1, vc1, hq, hkv, d)
    q2 = ops.rope_kv_write(ops.SplitK(P, split), pos, cs, slots, kc2, vc2, hq, hkv, d)
    assert torch.equal(q1, q2) and torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    I = 1024
    G = torch.randn(split, T, 2 * I, device=DEV)
    acc = G[0].clone()
    for k in range(1, split):
        acc += G[k]
    assert torch.equal(ops.silu_mul(acc.to(BF)), ops.silu_mul(ops.SplitK(G, split)))


def test_kv_block_copy():
    L, NB, hkv = 4, 40, 8
    kc = torch.randn(L, NB, hkv, 16, 128, device=DEV).to(BF)
    vc = torch.randn(L, NB, hkv, 128, 16, device=DEV).to(BF)
    src = torch.tensor([3, 7, 11], dtype=torch.int32, device=DEV)
    dst = torch.tensor([20, 21, 39], dtype=torch.int32, device=DEV)
    k2, v2 = kc.clone(), vc.clone()
    k2[:, dst.long()] = k2[:, src.long()]
    v2[:, dst.long()] = v2[:, src.long()]
    ops.kv_block_copy(kc, vc, src, dst)
    assert torch.equal(kc, k2) and torch.equal(vc, v2)


def test_linear_defer_reduce_roundtrip():
    x = torch.randn(64, 4096, device=DEV, dtype=BF)
    w = (torch.randn(4096, 4096, device=DEV) * 0.02).to(BF)
    sk = ops.linear_gm(x, w, 4, 4, defer_reduce=True)
    assert isinstance(sk, ops.SplitK) and sk.split == 4
    close(sk.resolve(), x.float() @ w.float().t(), atol=3e-2, rtol=2e-2)
    sk2 = ops.linear(x, w, split=4, defer_reduce=True)
    assert isinstance(sk2, ops.SplitK)
    close(sk2.resolve(), x.float() @ w.float().t(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("cfg", [2, 4, 5, 12, 19])
def test_gemm_mfma_bf16_partials_into_rmsnorm(cfg):
    """bf16 split-K slices (o_proj / down at decode) -> fused reduce + residual + RMSNorm matches the
    fp32 reference of the whole chain, and the slices themselves are bf16(fp32 slices)."""
    M, N, K = 256, 4096, 4096
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(BF)
    sk32 = ops.linear_gm(x, w, cfg, 4, defer_reduce=True)
    sk16 = ops.linear_gm(x, w, cfg, 4, defer_reduce=True, bf16_partials=True)
    assert sk16.is_bf16 and not sk32.is_bf16 and sk16.split == sk32.split
    assert torch.equal(sk16.P, sk32.P.to(BF))
    with pytest.raises(TypeError):
        ops.silu_mul(sk16)
    g = (torch.rand(N, device=DEV) + 0.5).to(BF)
    res0 = torch.randn(M, N, device=DEV).to(BF)
    r1, r2 = res0.clone(), res0.clone()
    got = ops.rmsnorm(sk16, g, 1e-5, residual=r1)
    want = ref.rmsnorm((x.float() @ w.float().t()).to(BF), g, 1e-5, r2)
    close(got, want, atol=5e-2, rtol=3e-2)
    close(r1, r2, atol=3e-2, rtol=2e-2)


def test_gemm_autotune_plan_dispatch():
    """tune_linear fills GEMM_PLAN for every bucket (one of ops.PLAN_CHOICES) and ops.linear follows it."""
    from ai_agent_kubectl_amd.ops.autotune import tune_linear
    ws = [(torch.randn(6144, 4096, device=DEV) * 0.02).to(BF) for _ in range(3)]
    rep = tune_linear({(6144, 4096): ws}, [1, 64, 256, 320])
    assert set(k[0] for k in rep) == {1, 64, 256, 320}
    assert all(v["choice"] in ops.PLAN_CHOICES for v in rep.values())
    for M in (1, 64, 200, 256, 300, 320):   # 200 / 300: no bucket, the next bucket's plan (ops.plan_for)
        x = torch.randn(M, 4096, device=DEV, dtype=BF)
        close(ops.linear(x, ws[0]), x.float() @ ws[0].float().t(), atol=3e-2, rtol=2e-2)
    for key in list(ops.GEMM_PLAN):
        if key[1:] == (6144, 4096):
            ops.GEMM_PLAN.pop(key)


@pytest.mark.parametrize("T", [1, 7, 64, 256])
@pytest.mark.parametrize("e0,el", [(0, 8), (4, 4)])
def test_moe_experts_vs_reference(T, e0, el):
    E, H, I, k = 8, 512, 384, 2
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w13 = (torch.randn(el, 2 * I, H, device=DEV) * 0.05).to(BF)
    w2 = (torch.randn(el, H, I, device=DEV) * 0.05).to(BF)
    logits = torch.randn(T, E, device=DEV, dtype=BF)
    tw, tid = ops.moe_topk(logits, k)
    got = ops.moe_experts(x, w13, w2, tw, tid, e0)
    want = torch.zeros(T, H, device=DEV)
    for t in range(T):
        for j in range(k):
            e = int(tid[t, j]) - e0
            if 0 <= e < el:
                g = x[t].float() @ w13[e].float().t()
                a = (torch.nn.functional.silu(g[:I]) * g[I:]).to(BF).float()
                want[t] += float(tw[t, j]) * (a @ w2[e].float().t())
    close(got, want, atol=5e-2, rtol=5e-2)


def _moe_dense_ref(x, w13, w2, tw, tid, e0):
    """fp32 reference of the local experts' weighted FFN (activation rounded to bf16 like the kernels)."""
    T, H = x.shape
    el, two_i, _ = w13.shape
    I = two_i // 2
    out = torch.zeros(T, H, device=x.device)
    for e in range(el):
        sel = (tid.long() == e0 + e)                      # [T, k]
        wt = (tw * sel).sum(1)                            # router weight of expert e per token
        rows = torch.nonzero(sel.any(1)).squeeze(1)
        if rows.numel() == 0:
            continue
        g = x[rows].float() @ w13[e].float().t()
        a = (torch.nn.functional.silu(g[:, :I]) * g[:, I:]).to(BF).float()
        out[rows] += wt[rows].unsqueeze(1) * (a @ w2[e].float().t())
    return out


@pytest.mark.parametrize("src_div", [1, 2])
def test_gemm_mfma_grouped_gather_scatter(src_div):
    """Grouped ring GEMM: rows gathered through device lists (empty groups, groups larger than a
    tile, ragged tails), output rows scattered; rows listed for no group stay untouched."""
    G, N, K, R = 5, 400, 512, 900
    counts_h = [0, 1, 300, 17, 260]
    perm = torch.randperm(R)
    lists = torch.zeros(G, R, dtype=torch.int32)
    o = 0
    for e, c in enumerate(counts_h):
        lists[e, :c] = perm[o:o + c]
        o += c
    lists, counts = lists.to(DEV), torch.tensor(counts_h, dtype=torch.int32, device=DEV)
    x = torch.randn(R // src_div + 1, K, device=DEV, dtype=BF)
    w = (torch.randn(G, N, K, device=DEV) * 0.05).to(BF)
    for cfg in ops.GM_CFGS:
        out = torch.full((R, N), 7.0, device=DEV, dtype=BF)
        ops.linear_grouped(x, w, counts, lists, R, src_div=src_div, cfg=cfg, out=out)
        for e, c in enumerate(counts_h):
            r = lists[e, :c].long()
            if c:
                close(out[r], x[r // src_div].float() @ w[e].float().t(), atol=3e-2, rtol=2e-2)
        untouched = perm[o:].to(DEV).long()
        assert torch.all(out[untouched] == 7.0), cfg


@pytest.mark.parametrize("mode", ["big", "gm"])
@pytest.mark.parametrize("T,skew", [(300, False), (1100, False), (2100, True)])
@pytest.mark.parametrize("e0,el", [(0, 8), (4, 4)])
def test_moe_experts_grouped_prefill(T, skew, e0, el, mode, monkeypatch):
    """Prefill-sized MoE block (T * k > MOE_HIP_MAX_ROWS): device routing + the grouped expert GEMMs
    (KA_MOE_PREFILL big: expert-sorted rows through gemm_big's grouped mode, chunks of 256 rows per
    expert, unused chunk-table entries skipped; gm: the grouped ring kernel) == fp32 reference, and ==
    the decode-path kernels on the same rows.  skew: expert e0 gets most rows (several chunks, others
    few or none)."""
    monkeypatch.setattr(ops, "MOE_PREFILL", mode)
    E, H, I, k = 8, 512, 384, 2
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w13 = (torch.randn(el, 2 * I, H, device=DEV) * 0.05).to(BF)
    w2 = (torch.randn(el, H, I, device=DEV) * 0.05).to(BF)
    logits = torch.randn(T, E, device=DEV, dtype=BF)
    if skew:
        logits[:, e0] += 3.0
    tw, tid = ops.moe_topk(logits, k)
    got = ops.moe_experts_grouped(x, w13, w2, tw, tid, e0)
    close(got, _moe_dense_ref(x, w13, w2, tw, tid, e0), atol=5e-2, rtol=5e-2)
    close(got, ops.moe_experts(x, w13, w2, tw, tid, e0), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T,want_big", [(300, False), (1100, True)])
def test_moe_prefill_auto_picks_path_by_rows(T, want_big, monkeypatch):
    """KA_MOE_PREFILL=auto: gemm_big's grouped mode from MOE_BIG_MIN_ROWS routed rows up, the grouped
    ring kernel below (threshold lowered to 1000 rows for the test); either way == the fp32 reference."""
    monkeypatch.setattr(ops, "MOE_PREFILL", "auto")
    monkeypatch.setattr(ops, "MOE_BIG_MIN_ROWS", 1000)
    ring_calls = []
    real = ops.linear_grouped
    monkeypatch.setattr(ops, "linear_grouped", lambda *a, **kw: ring_calls.append(1) or real(*a, **kw))
    E, H, I, k = 8, 512, 384, 2
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w13 = (torch.randn(E, 2 * I, H, device=DEV) * 0.05).to(BF)
    w2 = (torch.randn(E, H, I, device=DEV) * 0.05).to(BF)
    tw, tid = ops.moe_topk(torch.randn(T, E, device=DEV, dtype=BF), k)
    got = ops.moe_experts_grouped(x, w13, w2, tw, tid, 0)
    assert (len(ring_calls) == 0) == want_big
    close(got, _moe_dense_ref(x, w13, w2, tw, tid, 0), atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("R", [1, 29, 200, 700])
def test_moe_local_experts_received_rows(R):
    """Receive side of the A5 all-to-all (models/moe.py `_local_experts`): rows tagged with a global
    expert id, unweighted FFN of this rank's experts through the HIP grouped GEMMs."""
    from ai_agent_kubectl_amd.models.moe import _local_experts
    H, I, el, e0 = 512, 384, 4, 4
    x = torch.randn(R, H, device=DEV, dtype=BF)
    L = {"w13": (torch.randn(el, 2 * I, H, device=DEV) * 0.05).to(BF),
         "w2": (torch.randn(el, H, I, device=DEV) * 0.05).to(BF)}
    er = torch.randint(e0, e0 + el, (R,), device=DEV, dtype=torch.int32)
    got = _local_experts(x, er, L, e0)
    want = torch.empty(R, H, device=DEV)
    for r in range(R):
        e = int(er[r]) - e0
        g = x[r].float() @ L["w13"][e].float().t()
        a = (torch.nn.functional.silu(g[:I]) * g[I:]).to(BF).float()
        want[r] = a @ L["w2"][e].float().t()
    close(got, want, atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("T", [1, 3])
def test_moe_experts_split_k_mixtral_geometry(T):
    """Decode row counts at the real Mixtral-8x7B expert geometry (H 4096, I 14336): the grouped
    GEMMs run split-K (fp32 slices reduced by silu_mul_splitk and moe_combine); compare with a
    forced split of 1 and with an fp32 reference of the routed experts."""
    E, H, I, k = 8, 4096, 14336, 2
    assert ops.moe_split(T * k, E, 2 * I, H) >= 1 and ops.moe_split(T * k, E, H, I) > 1
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w13 = (torch.randn(E, 2 * I, H, device=DEV) * 0.02).to(BF)
    w2 = (torch.randn(E, H, I, device=DEV) * 0.02).to(BF)
    tw, tid = ops.moe_topk(torch.randn(T, E, device=DEV, dtype=BF), k)
    got = ops.moe_experts(x, w13, w2, tw, tid, 0)
    orig = ops.moe_split
    try:
        ops.moe_split = lambda *a, **kw: 1
        unsplit = ops.moe_experts(x, w13, w2, tw, tid, 0)
    finally:
        ops.moe_split = orig
    want = torch.zeros(T, H, device=DEV)
    for t in range(T):
        for j in range(k):
            e = int(tid[t, j])
            g = x[t].float() @ w13[e].float().t()
            a = (torch.nn.functional.silu(g[:I]) * g[I:]).to(BF).float()
            want[t] += float(tw[t, j]) * (a @ w2[e].float().t())
    close(got, want, atol=3e-2, rtol=3e-2)
    close(got, unsplit, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,I", [(4096, 14336), (1000, 512)])
def test_gemv_swiglu_fused_is_exact(M, N, I):
    """Batch-1..4 down projection with SiLU·mul computed in the GEMV's X staging == SiLU·mul kernel
    then the same GEMV at the same split (bitwise), and close to the fp32 reference."""
    gu = torch.randn(M, 2 * I, device=DEV, dtype=BF)
    w = (torch.randn(N, I, device=DEV) * 0.02).to(BF)
    got = ops.swiglu_linear(gu, w)
    if ops.ROWS_SWIGLU and ops.rows_ok(M, I, ops.ROWS_SWIGLU_SPLIT):   # row-streaming GEMV
        want = ops.linear_rows(ops.silu_mul(gu), w, ops.ROWS_SWIGLU_SPLIT, ops.ROWS_SWIGLU_RW)
    else:
        want = ops.linear(ops.silu_mul(gu), w, split=ops.skinny_split(M, N, I, 256))
    assert torch.equal(got, want)
    parts = ops.swiglu_linear(gu, w, defer_reduce=True)
    if isinstance(parts, ops.SplitK):
        close(parts.resolve(), want, atol=1e-2, rtol=1e-2)
    g = gu.float()
    a = (torch.nn.functional.silu(g[:, :I]) * g[:, I:]).to(BF).float()
    close(got, a @ w.float().t(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [8, 16, 48, 200, 256, 777])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 1024), (1040, 512)])
def test_gemm_mfma_all_configs(M, N, K):
    """csrc/gemm_mfma.hip: every configuration (LDS-DMA rings, 32-deep rings, ping-pong, one wave
    per SIMD), split-K 1/2/4 with fp32 partials reduced in-kernel and deferred fp32/bf16 slabs,
    ragged M and N edges, against the fp32 reference."""
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(BF)
    want = x.float() @ w.float().t()
    for cfg in ops.GM_CFGS:
        for split in (1, 2, 4):
            if K % (64 * split):
                continue
            got = ops.linear_gm(x, w, cfg, split)
            close(got, want, atol=3e-2, rtol=2e-2)
        sk = ops.linear_gm(x, w, cfg, 2, defer_reduce=True, bf16_partials=True)
        assert sk.is_bf16 and sk.split == 2
        close(sk.P.float().sum(0), want, atol=4e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [8, 16, 64, 256, 1000])
def test_gemm_mfma_swiglu_epilogue(M):
    """SwiGLU epilogue: W13 rows interleaved in 16-row (gate, up) chunks -> silu(gate) * up computed
    from the accumulators, equal to SiLU·mul of the fp32 reference product."""
    I, K = 1024, 512
    x = torch.randn(M, K, device=DEV, dtype=BF)
    wg = (torch.randn(I, K, device=DEV) * 0.05).to(BF)
    wu = (torch.randn(I, K, device=DEV) * 0.05).to(BF)
    w13i = torch.stack([wg.view(I // 16, 16, K), wu.view(I // 16, 16, K)], 1).reshape(2 * I, K).contiguous()
    g, u = x.float() @ wg.float().t(), x.float() @ wu.float().t()
    want = torch.nn.functional.silu(g) * u
    lib = _hip.require()
    for cfg in ops.GM_CFGS:
        y = torch.empty(M, I, device=DEV, dtype=BF)
        _hip.check(lib.ka_gemm_mfma(y.data_ptr(), None, x.data_ptr(), w13i.data_ptr(), M, 2 * I, K, K, I, 1, cfg,
                                    ops.GM_EPI_SWIGLU, 0, ops._stream()), "gemm_mfma swiglu")
        close(y, want, atol=3e-2, rtol=3e-2)


# ---- csrc/gemm_big.hip split tail (prefill projections: the partial last round of 256 x 256 tiles is
# cut into K slices that hand their fp32 tiles to the last-arriving slice of the same XCD) ----
def _gb_plan(M, N, K, epi):
    full, tail = torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
    ws = ops.gemm_big_ws(torch.device(DEV))
    s = _hip.require().ka_gemm_big_plan(M, N, epi, K, ws.numel(), full.data_ptr(), tail.data_ptr())
    return s, int(full), int(tail)


@pytest.mark.parametrize("M,N,K", [(4096, 6144, 4096), (2944, 6144, 4096), (777, 6144, 4096), (4096, 4096, 4096),
                                   (2900, 4096, 14336), (513, 1024, 512), (4096, 1152, 4096), (1000, 1152, 2048)])
def test_gemm_big_linear_split_tail_vs_fp32(M, N, K):
    """ops.linear_big (EPI_BF16) over shapes whose last round of tiles is split over K and over shapes
    that need no split; full matrices against the fp32 reference, the counters left at zero (the
    next launch of another shape reuses them) and the tail error word clear."""
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
    want = x.float() @ w.float().t()
    for _ in range(4):   # later launches run on counters the first one reset; a stale-slab read
        # (the plain-load hand-off, KA_GB_TAIL_MODE 0 / 1) showed in some launches only
        got = ops.linear_big(x, w)
        close(got, want, atol=3e-2, rtol=2e-2)
    ws = ops.gemm_big_ws(torch.device(DEV))
    assert int(ws[256:256 + 1024 * 32].view(torch.int32).abs().sum()) == 0
    assert ops.gemm_big_err(torch.device(DEV)) == 0


def test_gemm_big_split_tail_plans():
    """The shapes the bench's mixed steps produce get the tile width and split tail that fill the
    last round: QKV at M = 4096 runs 192-wide tiles (512 = 2 whole rounds) instead of 384 256-wide
    ones (1.5 rounds); at M = 2944 192-wide tiles too, without a split tail (the tail runs on 256-wide
    tiles only; choose_tn prices 192-wide tiles without one)."""
    lib = _hip.require()
    assert lib.ka_gemm_big_tn(4096, 6144, 0) == 6 and lib.ka_gemm_big_tn(4096, 6144, 4) == 6
    assert _gb_plan(4096, 6144, 4096, 0)[0] == 1
    assert lib.ka_gemm_big_tn(2944, 6144, 0) == 6
    s, full, tail = _gb_plan(2944, 6144, 4096, 0)      # 12 x 32 = 384: two rounds, no split
    assert s == 1 and full == 384 and tail == 0
    assert lib.ka_gemm_big_tn(4096, 1152, 0) == 8      # 80 256-wide tiles with a split tail beat 96 192-wide ones
    assert _gb_plan(4096, 1152, 4096, 0)[0] > 1
    s, full, tail = _gb_plan(2944, 28672, 4096, 3)     # gate_up + SwiGLU: 12 x 112 = 1344 = 5 x 256 + 64
    assert s > 1 and full == 1280 and tail == 64
    assert lib.ka_gemm_big_tn(2944, 28672, 3) == 8
    assert _gb_plan(4096, 4096, 4096, 0)[0] == 1       # O: exactly one round
    assert lib.ka_gemm_big_tn(4096, 4096, 0) == 8      # (4096 is no multiple of 192)


def test_gemm_big_alternating_launches_exact():
    """The launch pattern that exposed unordered LDS-DMA completion (profiles/r5/gemm_big_clamp/):
    every gemm_big launch follows an unrelated GEMM, and every result is checked whole.  With the
    old counted vmcnt wait, 4096 x 1152 (split tail, a partial last n-tile) and 2944 x 6144 (192-wide
    tiles, a partial last m-tile) came out wrong in 1-25 % of launches; the drained schedule never."""
    other = torch.randn(4096, 4096, device=DEV, dtype=BF)
    wo = (torch.randn(6144, 4096, device=DEV) / 64).to(BF)
    for (M, N, K) in [(4096, 1152, 4096), (2944, 6144, 4096)]:
        x = torch.randn(M, K, device=DEV, dtype=BF)
        w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
        want = x.float() @ w.float().t()
        bad = 0
        for _ in range(24):
            ops.linear_big(other, wo)
            err = (ops.linear_big(x, w).float() - want).abs() > 0.03 + 0.02 * want.abs()
            bad += int(bool(err.any()))
        assert bad == 0, f"{M}x{N}x{K}: {bad} of 24 launches wrong"
    assert ops.gemm_big_err(torch.device(DEV)) == 0


@pytest.mark.parametrize("amplify", [True, False])
def test_gm_dispatched_plans_alternating_launches_exact(amplify):
    """every (configuration, split-K, epilogue) of the ring kernels that the
    persisted decode plan dispatches for Llama-3-8B buckets 128-512 (bf16 split-K partials included),
    each launch right after an unrelated GEMM and checked whole against fp32 — with the duplicate-address
    amplifier (ldx = 0: every X piece reads 8 identical rows) and without.  The kernels wait for LDS-DMA
    with vmcnt(0) only (KA_GM_SCHED / KA_PP_SAFE), so no launch may be wrong; >= 500 launches per
    combination: scripts/gm_plan_stress.py, profiles/r6/lds_dma_safety/."""
    from ai_agent_kubectl_amd.ops import stress
    combos = stress.dispatched_combos()
    assert len(combos) >= 20, combos
    res = stress.stress(combos, 6, amplify)
    bad = {c: n for c, n in res.items() if n}
    assert not bad, f"wrong launches (M, N, K, cfg, split, epi): {bad}"


@pytest.mark.parametrize("M", [2944, 1100, 4096])
def test_gemm_big_swiglu_split_tail_vs_fp32(M):
    """gate_up + SwiGLU epilogue with the split tail: silu(x g^T) * (x u^T) vs fp32 (the sum of the
    slices goes through the nonlinearity, so a lost or doubled slice shows)."""
    H, I = 4096, 14336
    x = torch.randn(M, H, device=DEV, dtype=BF)
    w13 = (torch.randn(2 * I, H, device=DEV) / math.sqrt(H)).to(BF)
    g = x.float() @ w13[:I].float().t()
    u = x.float() @ w13[I:].float().t()
    want = torch.nn.functional.silu(g) * u
    got = ops.linear_swiglu(x, w13)
    close(got, want, atol=3e-2, rtol=3e-2)
    assert ops.gemm_big_err(torch.device(DEV)) == 0


@pytest.mark.parametrize("t,S", [(2, 1), (8, 256), (4, 333)])
def test_argmax_combine_vs_reference(t, S):
    """The hand-written TP combine kernel (csrc/sampling.hip) == the torch reference, ties included."""
    vals = torch.randint(0, 4, (t, S), device=DEV).float()   # many ties
    idxs = (torch.arange(t, device=DEV).view(t, 1) * 100000 + torch.randint(0, 1000, (t, S), device=DEV)).int()
    assert torch.equal(ops.argmax_combine(vals, idxs), ref.argmax_combine(vals, idxs))
