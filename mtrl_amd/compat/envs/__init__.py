from .atari import AtariConfig
from .base import EnvConfig
from .metaworld import MetaworldConfig

__all__ = ["AtariConfig", "EnvConfig", "MetaworldConfig"]
