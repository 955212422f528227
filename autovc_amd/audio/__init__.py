"""Audio frontends of the HIP path (autovc/audio/spectrogram.py).

The reference's `Audio` file/preprocessing class (autovc/audio/__init__.py, librosa + soundfile)
is outside the scope of this package; `load_wav` reads PCM/float WAV files with scipy.
"""
from . import spectrogram  # noqa: F401
from .spectrogram import (compute_partial_slices, mel_basis, mel_spec_auto_encoder,  # noqa: F401
                          mel_spec_speaker_encoder, mel_spectrogram)


def load_wav(path):
    """(samples float32 in [-1, 1], sample rate) of a WAV file, like librosa.load(path, sr=None)
    for mono files (multi-channel files are averaged, as librosa's default mono=True)."""
    import numpy as np
    from scipy.io import wavfile
    sr, data = wavfile.read(path)
    if data.dtype.kind == "i":
        data = data.astype(np.float32) / float(np.iinfo(data.dtype).max + 1)
    elif data.dtype.kind == "u":
        data = (data.astype(np.float32) - 128.0) / 128.0
    data = data.astype(np.float32)
    if data.ndim == 2:
        data = data.mean(axis=1)
    return data, sr
