"""Evaluation paths of the reference's figure scripts that run on the device."""
from .zsc import zsc_loss  # noqa: F401
