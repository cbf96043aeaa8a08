from .base import LLMBackend, LLMUnavailableError, build_backend  # noqa: F401
