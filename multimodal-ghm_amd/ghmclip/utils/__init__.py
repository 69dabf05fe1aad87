"""Configuration and logging utilities (reference: src/ghmclip/utils)."""
from .config import *  # noqa: F401,F403
from .logger import *  # noqa: F401,F403
