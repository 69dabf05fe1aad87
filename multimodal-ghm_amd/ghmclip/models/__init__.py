"""Model, loss and optimizer exports (reference: src/ghmclip/models)."""
from .model import *  # noqa: F401,F403
from .optimizer import *  # noqa: F401,F403
from .cdm import *  # noqa: F401,F403
from .vlm import *  # noqa: F401,F403
