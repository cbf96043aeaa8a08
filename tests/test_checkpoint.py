"""Checkpoint path: HF-layout safetensors -> fused / sharded engine weights.

There is no network and no real checkpoint in this image, so the test writes one: the random-init
weights of a model exported in the Hugging Face layout (`model.layers.N.self_attn.q_proj.weight`,
`mlp.gate_proj`, `block_sparse_moe.experts.E.w1`, ... split over two shard files), then
`models/weights.load_safetensors` must give back exactly the tensors `random_weights` builds for the
same TP / EP rank (those are generated in parallel-invariant units, so a TP shard of the loaded TP=1
checkpoint and the TP-rank random draw are the same numbers).  An engine built on the checkpoint
directory generates the same tokens as the random-init engine, and a `tokenizer.json` next to the
weights (a byte-level BPE built with `tokenizers`) becomes the engine's tokenizer.
"""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from ai_agent_kubectl_amd.models.config import get_config
from ai_agent_kubectl_amd.models.weights import ParallelInfo, load_safetensors, random_weights


def export_hf(cfg, W, out_dir, shards=2):
    """Write TP=1 engine weights `W` as an HF-layout checkpoint in `shards` files."""
    D, hq, hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    T = {"model.embed_tokens.weight": W["embed"], "lm_head.weight": W["lm_head"], "model.norm.weight": W["norm"]}
    for L in range(cfg.num_layers):
        p, hp = f"layers.{L}.", f"model.layers.{L}."
        qkv = W[p + "wqkv"]
        T[hp + "self_attn.q_proj.weight"] = qkv[:hq * D]
        T[hp + "self_attn.k_proj.weight"] = qkv[hq * D:(hq + hkv) * D]
        T[hp + "self_attn.v_proj.weight"] = qkv[(hq + hkv) * D:]
        T[hp + "self_attn.o_proj.weight"] = W[p + "wo"]
        T[hp + "input_layernorm.weight"] = W[p + "ln1"]
        T[hp + "post_attention_layernorm.weight"] = W[p + "ln2"]
        if cfg.is_moe:
            T[hp + "block_sparse_moe.gate.weight"] = W[p + "router"]
            I = cfg.intermediate
            for e in range(cfg.num_experts):
                ep = hp + f"block_sparse_moe.experts.{e}."
                T[ep + "w1.weight"] = W[p + "w13"][e, :I]
                T[ep + "w3.weight"] = W[p + "w13"][e, I:]
                T[ep + "w2.weight"] = W[p + "w2"][e]
        else:
            I = cfg.intermediate
            T[hp + "mlp.gate_proj.weight"] = W[p + "w13"][:I]
            T[hp + "mlp.up_proj.weight"] = W[p + "w13"][I:]
            T[hp + "mlp.down_proj.weight"] = W[p + "w2"]
    names = sorted(T)
    os.makedirs(out_dir, exist_ok=True)
    per = (len(names) + shards - 1) // shards
    for i in range(shards):
        part = {n: T[n].contiguous().clone() for n in names[i * per:(i + 1) * per]}
        save_file(part, os.path.join(out_dir, f"model-{i + 1:05d}-of-{shards:05d}.safetensors"))
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump({"model_type": cfg.family, "num_hidden_layers": cfg.num_layers}, f)
    return out_dir


@pytest.fixture(scope="module")
def checkpoints(tmp_path_factory):
    out = {}
    for model in ("tiny-llama", "tiny-mixtral"):
        cfg = get_config(model)
        W = random_weights(cfg, ParallelInfo(), seed=0)
        out[model] = export_hf(cfg, W, str(tmp_path_factory.mktemp(model)))
    return out


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
@pytest.mark.parametrize("tp,rank", [(1, 0), (2, 0), (2, 1)])
def test_safetensors_roundtrip_matches_random_weights(checkpoints, model, tp, rank):
    cfg = get_config(model)
    ep = tp if cfg.is_moe else 1
    par = ParallelInfo(rank, tp, rank if ep > 1 else 0, ep)
    got = load_safetensors(checkpoints[model], cfg, par)
    want = random_weights(cfg, par, seed=0)
    assert set(got) == set(want)
    for k in want:
        assert got[k].dtype == want[k].dtype and got[k].is_contiguous(), k
        assert torch.equal(got[k], want[k]), k


def test_single_file_checkpoint(tmp_path):
    cfg = get_config("tiny-llama")
    W = random_weights(cfg, ParallelInfo(), seed=3)
    d = export_hf(cfg, W, str(tmp_path / "one"), shards=1)
    f = os.path.join(d, "model-00001-of-00001.safetensors")
    got = load_safetensors(f, cfg, ParallelInfo())
    assert all(torch.equal(got[k], W[k]) for k in W)
    with pytest.raises(FileNotFoundError):
        load_safetensors(str(tmp_path / "missing"), cfg, ParallelInfo())


def test_engine_on_checkpoint_generates_like_random_init(checkpoints):
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    outs = []
    for spec in ("random:0", checkpoints["tiny-llama"]):
        eng = build_engine(EngineOptions(model="tiny-llama", weights=spec, device="cpu", max_batch=4,
                                         graph_buckets=(1, 2, 4), kv_cache_tokens=2048, max_model_len=256))
        be = EngineLLM(eng, max_new_tokens=6, ignore_eos=True)
        seqs = eng.generate_blocking([be.prompt_ids(q) for q in ("list pods", "get nodes")],
                                     SamplingParams(max_new_tokens=6, ignore_eos=True), forced_prefix=be._forced)
        outs.append([s.output_ids for s in seqs])
    assert outs[0] == outs[1]


def _llama3_tokenizer_json(path):
    """A small byte-level BPE with the Llama-3 special tokens at their real ids."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    corpus = ["kubectl get pods -n prod", "kubectl describe deployment api", "list all pods in namespace",
              "kubectl get nodes -o wide", "user assistant system", "kubectl logs web-1 --tail 100"] * 20
    tk.train_from_iterator(corpus, trainers.BpeTrainer(vocab_size=400, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                                        show_progress=False))
    data = json.loads(tk.to_str())
    specials = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]
    ids = [128000, 128001, 128006, 128007, 128009]
    data["added_tokens"] = [{"id": i, "content": s, "single_word": False, "lstrip": False, "rstrip": False,
                             "normalized": False, "special": True} for i, s in zip(ids, specials)]
    data["model"]["vocab"].update(dict(zip(specials, ids)))   # ids as in Llama-3 (past the BPE range)
    with open(path, "w") as f:
        json.dump(data, f)


def test_tokenizer_json_next_to_checkpoint_is_used(checkpoints, tmp_path):
    from ai_agent_kubectl_amd.engine.tokenizer import HFTokenizer, get_tokenizer, tokenizer_path
    d = checkpoints["tiny-llama"]
    _llama3_tokenizer_json(os.path.join(d, "tokenizer.json"))
    try:
        p = tokenizer_path(d)
        assert p == os.path.join(d, "tokenizer.json")
        tok = get_tokenizer(128256, "llama3", p)
        assert isinstance(tok, HFTokenizer)
        ids = tok.encode("kubectl get pods -n prod")
        assert tok.decode(ids) == "kubectl get pods -n prod"
        assert tok.bos_id == 128000 and tok.is_eos(128009)
        chat = tok.encode_chat("list pods")
        assert chat[0] == 128000 and 128009 in chat
        assert tokenizer_path("random:0") is None
    finally:
        os.remove(os.path.join(d, "tokenizer.json"))
