"""GHM samplers (reference: src/ghmclip/data)."""
from .data_random_GHM import *  # noqa: F401,F403
