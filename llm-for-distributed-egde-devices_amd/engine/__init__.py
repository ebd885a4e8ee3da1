from .kv_cache import KVCache, KVView
from .generate import Generator, GenerationResult, SamplingParams, needs_host_sampler

__all__ = ["KVCache", "KVView", "Generator", "GenerationResult", "SamplingParams", "needs_host_sampler"]
