"""Weight creation and loading, tensor/expert-parallel aware.

Fused layouts (row-major `[out, in]`, consumed by `F.linear` / the HIP GEMV):
  wqkv [(Hq + 2 Hkv) * D / t, H]   column-parallel: this rank's q heads, then k heads, then v heads
  wo   [H, Hq * D / t]             row-parallel
  w13  [2 I / t, H]                column-parallel gate | up (each half sharded)
  w2   [H, I / t]                  row-parallel
  MoE: w13 [E_local, 2 I, H], w2 [E_local, H, I], router [E, H] (replicated)
  embed [V, H] replicated; lm_head [V / t, H] vocab-parallel.

Random init (`WEIGHTS=random:<seed>`, the BASELINE configs' "random-init weights") is generated in
*parallel-invariant units* — one seeded draw per attention head, per 1/64 of the MLP width, per
1/64 of the vocab, per expert — so a TP=t shard is bit-identical to the matching slice of the TP=1
weights.  That is what makes the virtual-TP and multi-process TP parity tests exact.

`load_safetensors` maps HF Llama / Mixtral checkpoints (`model.layers.N.self_attn.q_proj.weight`,
...) into the fused, sharded layout.
"""
from __future__ import annotations

import glob
import hashlib
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .config import ModelConfig

STD = 0.02
MLP_UNITS = 64
VOCAB_UNITS = 64


@dataclass
class ParallelInfo:
    tp_rank: int = 0
    tp_size: int = 1
    ep_rank: int = 0
    ep_size: int = 1


def _seed(*parts) -> int:
    h = hashlib.blake2b(repr(parts).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFFFFFFFFFFFFFF


def _randn(shape, seed, device, dtype, std=STD):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return (torch.randn(shape, generator=g, device=device, dtype=torch.float32) * std).to(dtype)


def _units(total: int, n_units: int, rank: int, size: int) -> List[range]:
    """Split [0,total) into n_units equal units (requires divisibility) and return this rank's unit ranges."""
    assert total % n_units == 0 and n_units % size == 0, (total, n_units, size)
    per = n_units // size
    u = total // n_units
    return [range((rank * per + i) * u, (rank * per + i + 1) * u) for i in range(per)]


def _mlp_units(inter: int) -> int:
    for n in (MLP_UNITS, 32, 16, 8, 4, 2, 1):
        if inter % n == 0:
            return n
    return 1


def _vocab_units(vocab: int) -> int:
    for n in (VOCAB_UNITS, 32, 16, 8, 4, 2, 1):
        if vocab % n == 0:
            return n
    return 1


def validate_parallel(cfg: ModelConfig, par: ParallelInfo) -> None:
    t = par.tp_size
    if cfg.num_heads % t or cfg.num_kv_heads % t:
        raise ValueError(f"TP={t} must divide heads {cfg.num_heads}/{cfg.num_kv_heads}")
    if cfg.is_moe:
        if cfg.num_experts % par.ep_size:
            raise ValueError(f"EP={par.ep_size} must divide experts {cfg.num_experts}")
    elif _mlp_units(cfg.intermediate) % t:
        raise ValueError(f"TP={t} must divide MLP units")
    if _vocab_units(cfg.vocab_size) % t:
        raise ValueError(f"TP={t} must divide the vocab units ({cfg.vocab_size})")


def random_weights(cfg: ModelConfig, par: ParallelInfo, seed: int = 0, device="cpu",
                   dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    validate_parallel(cfg, par)
    H, D = cfg.hidden, cfg.head_dim
    t, r = par.tp_size, par.tp_rank
    hq, hkv = cfg.num_heads // t, cfg.num_kv_heads // t
    W: Dict[str, torch.Tensor] = {}
    W["embed"] = torch.cat([_randn((len(u), H), _seed(seed, "embed", u.start), device, dtype)
                            for u in _units(cfg.vocab_size, _vocab_units(cfg.vocab_size), 0, 1)])
    W["lm_head"] = torch.cat([_randn((len(u), H), _seed(seed, "lm_head", u.start), device, dtype)
                              for u in _units(cfg.vocab_size, _vocab_units(cfg.vocab_size), r, t)])
    W["norm"] = torch.ones(H, device=device, dtype=dtype)
    for L in range(cfg.num_layers):
        p = f"layers.{L}."
        q = [_randn((D, H), _seed(seed, L, "q", r * hq + i), device, dtype) for i in range(hq)]
        k = [_randn((D, H), _seed(seed, L, "k", r * hkv + i), device, dtype) for i in range(hkv)]
        v = [_randn((D, H), _seed(seed, L, "v", r * hkv + i), device, dtype) for i in range(hkv)]
        W[p + "wqkv"] = torch.cat(q + k + v)
        W[p + "wo"] = torch.cat([_randn((H, D), _seed(seed, L, "o", r * hq + i), device, dtype)
                                 for i in range(hq)], dim=1)
        W[p + "ln1"] = torch.ones(H, device=device, dtype=dtype)
        W[p + "ln2"] = torch.ones(H, device=device, dtype=dtype)
        if cfg.is_moe:
            E = cfg.num_experts
            W[p + "router"] = _randn((E, H), _seed(seed, L, "router"), device, dtype)
            el = E // par.ep_size
            w13, w2 = [], []
            for i in range(el):
                e = par.ep_rank * el + i
                g = _randn((cfg.intermediate, H), _seed(seed, L, "e_gate", e), device, dtype)
                u_ = _randn((cfg.intermediate, H), _seed(seed, L, "e_up", e), device, dtype)
                w13.append(torch.cat([g, u_]))
                w2.append(_randn((H, cfg.intermediate), _seed(seed, L, "e_down", e), device, dtype))
            W[p + "w13"] = torch.stack(w13)
            W[p + "w2"] = torch.stack(w2)
        else:
            units = _units(cfg.intermediate, _mlp_units(cfg.intermediate), r, t)
            gate = [_randn((len(u), H), _seed(seed, L, "gate", u.start), device, dtype) for u in units]
            up = [_randn((len(u), H), _seed(seed, L, "up", u.start), device, dtype) for u in units]
            W[p + "w13"] = torch.cat(gate + up)
            W[p + "w2"] = torch.cat([_randn((H, len(u)), _seed(seed, L, "down", u.start), device, dtype)
                                     for u in units], dim=1)
    return W


# ------------------------------------------------------------------------------------------------
def load_safetensors(path: str, cfg: ModelConfig, par: ParallelInfo, device="cpu",
                     dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    """Load an HF-format Llama / Mixtral checkpoint (one file or a directory of shards)."""
    from safetensors import safe_open

    validate_parallel(cfg, par)
    files = [path] if os.path.isfile(path) else sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no .safetensors under {path}")
    handles = [safe_open(f, framework="pt", device="cpu") for f in files]
    index = {}
    for hnd in handles:
        for k in hnd.keys():
            index[k] = hnd

    def get(name) -> torch.Tensor:
        return index[name].get_tensor(name)

    t, r = par.tp_size, par.tp_rank
    D, H = cfg.head_dim, cfg.hidden
    hq, hkv = cfg.num_heads // t, cfg.num_kv_heads // t

    def rows(x, start, n):
        return x[start:start + n]

    W: Dict[str, torch.Tensor] = {}
    W["embed"] = get("model.embed_tokens.weight")
    lm = get("lm_head.weight") if "lm_head.weight" in index else W["embed"]
    vs = cfg.vocab_size // t
    W["lm_head"] = rows(lm, r * vs, vs)
    W["norm"] = get("model.norm.weight")
    for L in range(cfg.num_layers):
        p, hp = f"layers.{L}.", f"model.layers.{L}."
        q = rows(get(hp + "self_attn.q_proj.weight"), r * hq * D, hq * D)
        k = rows(get(hp + "self_attn.k_proj.weight"), r * hkv * D, hkv * D)
        v = rows(get(hp + "self_attn.v_proj.weight"), r * hkv * D, hkv * D)
        W[p + "wqkv"] = torch.cat([q, k, v])
        W[p + "wo"] = get(hp + "self_attn.o_proj.weight")[:, r * hq * D:(r + 1) * hq * D]
        W[p + "ln1"] = get(hp + "input_layernorm.weight")
        W[p + "ln2"] = get(hp + "post_attention_layernorm.weight")
        if cfg.is_moe:
            W[p + "router"] = get(hp + "block_sparse_moe.gate.weight")
            el = cfg.num_experts // par.ep_size
            w13, w2 = [], []
            for i in range(el):
                e = par.ep_rank * el + i
                ep = hp + f"block_sparse_moe.experts.{e}."
                w13.append(torch.cat([get(ep + "w1.weight"), get(ep + "w3.weight")]))
                w2.append(get(ep + "w2.weight"))
            W[p + "w13"] = torch.stack(w13)
            W[p + "w2"] = torch.stack(w2)
        else:
            i_l = cfg.intermediate // t
            g = rows(get(hp + "mlp.gate_proj.weight"), r * i_l, i_l)
            u = rows(get(hp + "mlp.up_proj.weight"), r * i_l, i_l)
            W[p + "w13"] = torch.cat([g, u])
            W[p + "w2"] = get(hp + "mlp.down_proj.weight")[:, r * i_l:(r + 1) * i_l]
    return {k: v.to(device=device, dtype=dtype).contiguous() for k, v in W.items()}


def build_weights(spec: str, cfg: ModelConfig, par: ParallelInfo, device="cpu", dtype=torch.bfloat16):
    if spec.startswith("random"):
        seed = int(spec.split(":", 1)[1]) if ":" in spec else 0
        return random_weights(cfg, par, seed=seed, device=device, dtype=dtype)
    return load_safetensors(spec, cfg, par, device=device, dtype=dtype)
