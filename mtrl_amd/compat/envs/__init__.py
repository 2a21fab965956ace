from .base import EnvConfig
from .metaworld import MetaworldConfig

__all__ = ["EnvConfig", "MetaworldConfig"]
