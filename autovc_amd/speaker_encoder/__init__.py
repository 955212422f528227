from .model import SpeakerEncoder  # noqa: F401
