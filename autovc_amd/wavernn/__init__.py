from .model import WaveRNN  # noqa: F401
