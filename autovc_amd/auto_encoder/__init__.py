# Same export as the reference's autovc/auto_encoder/__init__.py:1
from .model import AutoEncoder, FusedAdam  # noqa: F401
