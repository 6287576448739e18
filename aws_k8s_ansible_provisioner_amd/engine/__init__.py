from .config import EngineConfig, SamplingParams  # noqa: F401
