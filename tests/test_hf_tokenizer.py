"""Real-checkpoint tokenizer support (engine/tokenizer.py HFTokenizer): a byte-level BPE
`tokenizer.json` with the Llama-3 special tokens is trained offline here (no download), then used
for encode/decode, the SAFE_DECODE masks and a tiny-engine generation through the API backend."""
import asyncio

import pytest

from ai_agent_kubectl_amd.safety import is_safe_kubectl_command

SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]
CORPUS = ["kubectl get pods -n prod", "kubectl describe deployment api", "list all pods in namespace prod",
          "kubectl logs web-1 --tail 20", "Translate the request into one kubectl command.",
          "user assistant\n\nkubectl get svc -A"] * 20


@pytest.fixture(scope="module")
def tok_path(tmp_path_factory):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=700, special_tokens=SPECIALS,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(CORPUS, tr)
    p = tmp_path_factory.mktemp("tok") / "tokenizer.json"
    tk.save(str(p))
    return str(p)


def test_hf_tokenizer_roundtrip_and_specials(tok_path):
    from ai_agent_kubectl_amd.engine.tokenizer import HFTokenizer
    tok = HFTokenizer(tok_path, 128256, "llama3")
    for text in ("kubectl get pods -n prod", "ünïcode & spaces  x", "line\nbreak"):
        ids = tok.encode(text)
        assert tok.decode(ids) == text
    before, after = tok.chat_prefix_suffix()
    assert before[0] == tok.specials["<|begin_of_text|>"] and after[0] == tok.specials["<|eot_id|>"]
    assert tok.is_eos(tok.specials["<|eot_id|>"]) and tok.id_to_bytes[tok.specials["<|eot_id|>"]] is None
    assert tok.decode(before + tok.encode("hi") + after) == "user\n\nhiassistant\n\n"


def test_hf_tokenizer_masks_and_engine(tok_path, monkeypatch):
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.safe_decode import MASK_BODY, build_masks
    from ai_agent_kubectl_amd.engine.tokenizer import HFTokenizer, get_tokenizer
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    import numpy as np
    tok = HFTokenizer(tok_path, 128256, "llama3")
    m = build_masks(tok)
    allowed = [t for t in range(tok.vocab_size) if (m[MASK_BODY][t // 32] >> np.uint32(t % 32)) & 1]
    assert allowed and all(t < 700 or tok.is_eos(t) for t in allowed)   # only real tokens (or EOS)
    monkeypatch.setenv("TOKENIZER", tok_path)
    get_tokenizer.cache_clear()
    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=4, use_graphs=False,
                                     kv_cache_tokens=4096, max_model_len=512))
    assert isinstance(eng.tokenizer, HFTokenizer)
    be = EngineLLM(eng, max_new_tokens=8)

    async def run():
        await be.start()
        try:
            return await be.generate("list all pods in namespace prod")
        finally:
            await be.close()

    out = asyncio.run(run())
    assert out.startswith("kubectl") and is_safe_kubectl_command(out), out
    get_tokenizer.cache_clear()
