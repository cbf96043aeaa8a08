"""MI355X-native natural-language -> kubectl agent service.

Same HTTP surface as mrankitvish/ai-agent-kubectl (`/root/reference/app.py`), with the remote
OpenAI call replaced by an on-node LLM engine (paged KV, continuous batching, hipGraph decode,
hand-written CDNA4 HIP kernels, RCCL tensor/expert parallelism).  See SURVEY.md / README.md.
"""
__version__ = "0.1.0"
