from .config import ModelConfig, get_config, list_models  # noqa: F401
