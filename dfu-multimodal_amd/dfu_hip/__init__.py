"""dfu_hip — MI355X-native (gfx950) kernels and autograd layers for the DFU fusion training step."""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
