"""ghmclip — MI355X-native build of the Multimodal-GHM CLIP training path.

Same public package API as the reference's ``ghmclip`` (src/ghmclip/__init__.py);
compute runs in hand-written gfx950 HIP kernels (libghm_hip.so) and the native
host sampler (libghm_host.so).
"""
from .models import *  # noqa: F401,F403
from .data import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
