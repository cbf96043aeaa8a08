"""The instruction prompt and its rendering.

`PROMPT_TEMPLATE` is the reference's prompt text verbatim (`/root/reference/app.py:50-57`), so the
on-node model sees the same instruction the OpenAI model saw.  LangChain's
`PromptTemplate.format` -> `StringPromptValue` -> one *user* message;
`render_prompt` is that `format` step and the model-specific chat templates live in
`engine/tokenizer.py`.
"""
from __future__ import annotations

PROMPT_TEMPLATE = """
You are a Kubernetes CLI specialist.
When given a user request, output exactly one valid, single-line `kubectl` command that fulfils it.
Do not include comments, explanations, or shell operators (`;`, `&&`, `||`, (```) etc.).
Only output the command itself, nothing else.
User Request: {query}
Kubectl Command:
"""

# Everything before the query is identical for every request: the engine's prefix cache keys on it.
PROMPT_PREFIX, PROMPT_SUFFIX = PROMPT_TEMPLATE.split("{query}")


def render_prompt(query: str) -> str:
    return PROMPT_PREFIX + query + PROMPT_SUFFIX
