"""MI355X-native AutoVC Generator (autoencoder) hot path.

`autovc_amd.auto_encoder.AutoEncoder` is a drop-in for the reference's
`autovc.auto_encoder.AutoEncoder` (autovc/auto_encoder/model.py:27); its arithmetic runs in the
hand-written gfx950 HIP kernels of libautovc_hip.so (C ABI: include/autovc_hip.h).
"""
__version__ = "0.1.0"
