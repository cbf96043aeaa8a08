"""Deterministic synthetic tokenizer with the real vocabulary sizes.

No tokenizer files exist offline (SURVEY.md §0.1, §7.3 hard part 2), so the engine uses a
synthetic byte-level vocabulary built deterministically from a seed:

* ids 0..255: the 256 single bytes (byte fallback — any UTF-8 text round-trips exactly);
* then common English / Kubernetes / kubectl words, each with and without a leading space and
  capitalised, plus whitespace / punctuation runs — so that the reference prompt
  (`/root/reference/app.py:50-57`) encodes at roughly 4 characters per token like a real BPE;
* then seeded pseudo-words (" blorf", "zenti", ...) up to the model's vocab size;
* Llama-3 special tokens at their real ids (128000 `<|begin_of_text|>`, 128001
  `<|end_of_text|>`, 128006/128007 header ids, 128009 `<|eot_id|>`); the Llama-2/Mixtral
  vocabulary (32000) uses `<unk>`=0, `<s>`=1, `</s>`=2 and byte tokens at 3..258.

Encoding is greedy longest-match over a trie (a native C++ encoder in `runtime/` replaces it when
built).  `encode_chat` implements each family's chat template with one user turn (the LangChain
`PromptTemplate` -> single HumanMessage path).
"""
from __future__ import annotations

import functools
import os
import random
from typing import Dict, List, Optional, Sequence, Tuple

_WORDS = """
you are a the an of to and in on for with is it that this be as at by from or not no yes all any each
every one two three only exactly valid single line command commands output outputs when given user request
requests fulfil fulfils fulfill do does include including comments comment explanations explanation shell
operators operator etc itself nothing else kubernetes cli specialist kubectl get describe delete apply create
edit patch logs log exec port forward top rollout restart status history undo scale autoscale label annotate
expose run set image cordon uncordon drain taint cluster info version config view use context contexts current
pod pods service services svc deployment deployments deploy node nodes namespace namespaces ns configmap
configmaps secret secrets ingress ingresses pv pvc persistent volume volumes claim claims job jobs cronjob
cronjobs statefulset statefulsets daemonset daemonsets replicaset replicasets event events endpoint endpoints
account accounts role roles rolebinding clusterrole binding bindings networkpolicy policy policies container
containers replicas replica wide yaml json name names label labels selector field sort by watch follow tail
previous since output format show list me my what which how many count running pending failed failing crash
crashing loop crashloopbackoff ready not restarts age default system kube public production prod staging dev
development test web api frontend backend database db redis nginx postgres mysql app apps server worker cache
memory cpu usage resource resources limit limits quota quotas storage class classes network ip address port
ports traffic load balancer health check image images tag version latest new old first last recent older than
minutes minute hours hour days day seconds second ago where whose with without across inside into out about
please can could would should will want need help find give tell see check look up up down off over under more
less most least top bottom high low all_namespaces a-z n o l f c -n -o -l -f -c -A --all-namespaces --namespace
--selector --output --replicas --image --follow --tail --previous --sort-by --field-selector --show-labels
--no-headers --watch --context --dry-run=client -o=yaml -o=json -o=wide get_pods
"""

_PUNCT = ["\n", "\n\n", " \n", ".\n", ":\n", ". ", ", ", ": ", " (", ")", "(", " `", "`", "```", " ```", "`,",
          "`;", "`&&", "`||", "`)", "),", "`;`", "`&&`", "`||`", " -", " --", "--", "=", " =", "/", " /", "_",
          ".", ",", ":", ";", "'", "\"", " '", " \"", "  ", "   ", "    ", " etc", ".).", "etc.)", " etc.).",
          "-", "0", "1", "2", "3", "10", "100"]

_CONS = "bcdfghjklmnprstvwxz"
_VOWS = "aeiou"

LLAMA3_SPECIALS = {
    "<|begin_of_text|>": 128000, "<|end_of_text|>": 128001, "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007, "<|eot_id|>": 128009,
}
LLAMA2_SPECIALS = {"<unk>": 0, "<s>": 1, "</s>": 2}


def _pseudo_words(n: int, seed: int, taken: set) -> List[str]:
    rng = random.Random(seed)
    out: List[str] = []
    while len(out) < n:
        syl = rng.randint(1, 3)
        w = "".join(rng.choice(_CONS) + rng.choice(_VOWS) + (rng.choice(_CONS) if rng.random() < 0.3 else "")
                    for _ in range(syl))
        w = (" " + w) if rng.random() < 0.7 else w
        if w not in taken:
            taken.add(w)
            out.append(w)
    return out


class SyntheticTokenizer:
    def __init__(self, vocab_size: int = 128256, family: str = "llama3", seed: int = 1234):
        self.vocab_size = vocab_size
        self.family = family
        if family == "llama3":
            self.specials = dict(LLAMA3_SPECIALS)
            byte_base = 0
            n_regular = 128000
            for i in range(128256 - 128000):
                name = f"<|reserved_special_token_{i}|>"
                tid = 128000 + i
                if tid not in self.specials.values():
                    self.specials[name] = tid
            self.bos_id = 128000
            self.eos_ids = (128009, 128001)
        else:
            self.specials = dict(LLAMA2_SPECIALS)
            byte_base = 3
            n_regular = vocab_size
            self.bos_id = 1
            self.eos_ids = (2,)
        self.eos_id = self.eos_ids[0]
        n_regular = min(n_regular, vocab_size)
        pieces: List[bytes] = [bytes([b]) for b in range(256)]
        taken = set()
        words = []
        for w in _WORDS.split():
            for v in (w, " " + w, w.capitalize(), " " + w.capitalize()):
                if v not in taken and len(v) > 1:
                    taken.add(v)
                    words.append(v)
        for p in _PUNCT:
            if p not in taken and len(p.encode()) > 1:
                taken.add(p)
                words.append(p)
        n_fill = n_regular - byte_base - 256 - len(words)
        words += _pseudo_words(max(0, n_fill), seed, taken)
        pieces += [w.encode("utf-8") for w in words[: n_regular - byte_base - 256]]
        # id -> bytes
        self.id_to_bytes: List[Optional[bytes]] = [None] * vocab_size
        for i, p in enumerate(pieces):
            self.id_to_bytes[byte_base + i] = p
        self.id_to_special: Dict[int, str] = {v: k for k, v in self.specials.items()}
        self.byte_base = byte_base
        # trie over bytes: dict-of-dicts, terminal id under key -1
        self._trie: dict = {}
        for tid, p in enumerate(self.id_to_bytes):
            if p is None:
                continue
            node = self._trie
            for b in p:
                node = node.setdefault(b, {})
            node[-1] = tid
        self.max_piece = max(len(p) for p in pieces)
        self._native = None
        try:  # optional C++ encoder (runtime/_native)
            from ..runtime import native
            self._native = native.make_tokenizer(self)
        except Exception:
            self._native = None

    # ------------------------------------------------------------------------------------------
    def encode(self, text: str) -> List[int]:
        data = text.encode("utf-8")
        if self._native is not None:
            return self._native.encode(data)
        out: List[int] = []
        i, n = 0, len(data)
        trie = self._trie
        while i < n:
            node = trie
            best, best_len = -1, 0
            j = i
            while j < n:
                node = node.get(data[j])
                if node is None:
                    break
                j += 1
                t = node.get(-1)
                if t is not None:
                    best, best_len = t, j - i
            out.append(best)
            i += best_len
        return out

    def token_bytes(self, tid: int) -> bytes:
        p = self.id_to_bytes[tid] if 0 <= tid < self.vocab_size else None
        return p if p is not None else b""

    def token_text(self, tid: int) -> str:
        if tid in self.id_to_special:
            return self.id_to_special[tid]
        return self.token_bytes(tid).decode("utf-8", errors="replace")

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        buf = bytearray()
        for t in ids:
            p = self.id_to_bytes[t] if 0 <= t < self.vocab_size else None
            if p is None:
                if not skip_special and t in self.id_to_special:
                    buf += self.id_to_special[t].encode()
                continue
            buf += p
        return buf.decode("utf-8", errors="replace")

    def is_eos(self, tid: int) -> bool:
        return tid in self.eos_ids

    # ------------------------------------------------------------------------------------------
    def chat_prefix_suffix(self) -> Tuple[List[int], List[int]]:
        """Token ids that wrap a single user message: (before, after) incl. the assistant header."""
        if self.family == "llama3":
            s = self.specials
            before = [s["<|begin_of_text|>"], s["<|start_header_id|>"]] + self.encode("user") + \
                [s["<|end_header_id|>"]] + self.encode("\n\n")
            after = [s["<|eot_id|>"], s["<|start_header_id|>"]] + self.encode("assistant") + \
                [s["<|end_header_id|>"]] + self.encode("\n\n")
        else:
            before = [self.bos_id] + self.encode("[INST] ")
            after = self.encode(" [/INST]")
        return before, after

    def encode_chat(self, prompt: str) -> List[int]:
        before, after = self.chat_prefix_suffix()
        return before + self.encode(prompt) + after


def _byte_decoder() -> Dict[str, int]:
    """Inverse of the GPT-2 / tiktoken byte-level BPE alphabet (printable stand-ins for bytes)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


class HFTokenizer:
    """A real checkpoint's `tokenizer.json` (HF `tokenizers`) behind the engine's tokenizer interface.

    Llama-3 is byte-level BPE (token strings use the GPT-2 byte alphabet); Llama-2 / Mixtral are
    SentencePiece BPE (`▁` = space, `<0xNN>` byte fallback).  `id_to_bytes` gives the exact bytes of
    every regular token (the SAFE_DECODE masks are built from it); added tokens are specials."""

    def __init__(self, path: str, vocab_size: int, family: str):
        from tokenizers import Tokenizer
        if os.path.isdir(path):
            path = os.path.join(path, "tokenizer.json")
        self.tk = Tokenizer.from_file(path)
        self.vocab_size = vocab_size
        self.family = family
        added = {t.content: i for i, t in self.tk.get_added_tokens_decoder().items()} \
            if hasattr(self.tk, "get_added_tokens_decoder") else {}
        self.specials: Dict[str, int] = dict(added)
        self.id_to_special = {v: k for k, v in self.specials.items()}
        vocab = self.tk.get_vocab(with_added_tokens=False)
        byte_level = any(ch in tok for tok in list(vocab)[:2000] for ch in ("\u0120", "\u010a"))
        dec = _byte_decoder()
        self.id_to_bytes: List[Optional[bytes]] = [None] * vocab_size
        for tok, i in vocab.items():
            if i >= vocab_size or i in self.id_to_special:
                continue
            if byte_level:
                try:
                    self.id_to_bytes[i] = bytes(dec[c] for c in tok)
                except KeyError:
                    self.id_to_bytes[i] = tok.encode("utf-8")
            elif len(tok) == 6 and tok.startswith("<0x") and tok.endswith(">"):
                self.id_to_bytes[i] = bytes([int(tok[3:5], 16)])
            else:
                self.id_to_bytes[i] = tok.replace("\u2581", " ").encode("utf-8")
        sp = self.specials
        if family == "llama3":
            self.bos_id = sp.get("<|begin_of_text|>", 128000)
            self.eos_ids = tuple(sp[n] for n in ("<|eot_id|>", "<|end_of_text|>") if n in sp) or (128009,)
        else:
            self.bos_id = sp.get("<s>", 1)
            self.eos_ids = (sp.get("</s>", 2),)
        self.eos_id = self.eos_ids[0]

    def encode(self, text: str) -> List[int]:
        return self.tk.encode(text, add_special_tokens=False).ids

    def token_bytes(self, tid: int) -> bytes:
        p = self.id_to_bytes[tid] if 0 <= tid < self.vocab_size else None
        return p if p is not None else b""

    def token_text(self, tid: int) -> str:
        if tid in self.id_to_special:
            return self.id_to_special[tid]
        return self.token_bytes(tid).decode("utf-8", errors="replace")

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        buf = bytearray()
        for t in ids:
            p = self.id_to_bytes[t] if 0 <= t < self.vocab_size else None
            if p is None:
                if not skip_special and t in self.id_to_special:
                    buf += self.id_to_special[t].encode()
                continue
            buf += p
        return buf.decode("utf-8", errors="replace")

    def is_eos(self, tid: int) -> bool:
        return tid in self.eos_ids

    def chat_prefix_suffix(self) -> Tuple[List[int], List[int]]:
        if self.family == "llama3":
            s = self.specials
            before = [s["<|begin_of_text|>"], s["<|start_header_id|>"]] + self.encode("user") + \
                [s["<|end_header_id|>"]] + self.encode("\n\n")
            after = [s["<|eot_id|>"], s["<|start_header_id|>"]] + self.encode("assistant") + \
                [s["<|end_header_id|>"]] + self.encode("\n\n")
        else:
            before = [self.bos_id] + self.encode("[INST] ")
            after = self.encode(" [/INST]")
        return before, after

    def encode_chat(self, prompt: str) -> List[int]:
        before, after = self.chat_prefix_suffix()
        return before + self.encode(prompt) + after


def tokenizer_path(weights: Optional[str]) -> Optional[str]:
    """TOKENIZER env, else <WEIGHTS dir>/tokenizer.json when the weights are a local checkpoint."""
    p = os.environ.get("TOKENIZER")
    if p:
        return p
    if weights and not weights.startswith("random") and os.path.isdir(weights):
        f = os.path.join(weights, "tokenizer.json")
        if os.path.exists(f):
            return f
    return None


@functools.lru_cache(maxsize=4)
def get_tokenizer(vocab_size: int, family: str, path: Optional[str] = None):
    """The checkpoint's real tokenizer when `path` is given, else the synthetic one (random weights)."""
    if path:
        return HFTokenizer(path, vocab_size, family)
    return SyntheticTokenizer(vocab_size=vocab_size, family=family)
