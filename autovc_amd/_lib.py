"""ctypes binding of the HIP C-ABI library (include/autovc_hip.h -> autovc_amd/libautovc_hip.so).

The library is the only compute path of this package: there is no CPU or pure-PyTorch
fallback, and every call fails loudly (RuntimeError/ValueError) when the library is missing or a
kernel launch is rejected.  `torch` is imported first so that the library binds to the HIP
runtime torch already loaded (both carry SONAME libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AUTOVC_HIP_LIB", os.path.join(_HERE, "libautovc_hip.so"))

ACT_NONE, ACT_RELU, ACT_TANH, ACT_DBNORM = 0, 1, 2, 3
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "avc_abi_version": [],
    "avc_last_error": [],
    "avc_context_create": [_I, ctypes.POINTER(_P)],
    "avc_context_destroy": [_P],
    "avc_context_reserve": [_P, _Z],
    "avc_gemm": [_P, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P],
    "avc_conv_bn_act_forward": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _I,
                                _P, _P, _P, _P, _P, _P],
    "avc_conv_bn_act_backward": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P,
                                 _P, _P, _P, _P, _I, _P],
    "avc_conv_bn_act_forward_ex": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _I,
                                   _P, _P, _P, _P, _P, _P, _P, _P],
    "avc_conv_bn_act_backward_ex": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P,
                                    _P, _P, _P, _P, _I, _P, _P],
    "avc_conv_bn_act_forward_frag": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _I,
                                     _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "avc_conv_bn_act_forward_wg": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _I,
                                   _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "avc_conv_bn_act_backward_wg": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P,
                                    _P, _P, _P, _P, _I, _P, _P, _P],
    "avc_conv_wgrad_image_bytes": [_I, _I, _I, _I],
    "avc_conv_frag_chain_ok": [_I, _I, _I, _I],
    "avc_act_frag_bytes": [ctypes.c_long, _I],
    "avc_lstm_forward": [_P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P],
    "avc_bilstm_forward": [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P],
    "avc_lstm_backward": [_P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P,
                          _P, _P, _P, _I, _I, _P],
    "avc_lstm_backward_ex": [_P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P,
                             _P, _P, _P, _I, _I, _P, _I, _P],
    "avc_lstm_forward_ex": [_P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _P],
    "avc_bilstm_forward_ex": [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _P],
    "avc_linear_forward": [_P, _I, _I, _I, _P, _P, _P, _P, _P],
    "avc_linear_backward": [_P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P],
    "avc_frames_from_mel": [_I, _I, _I, _P, _I, _P, _P, _P],
    "avc_frames_from_mel_backward": [_I, _I, _I, _I, _P, _I, _P, _P, _I, _P],
    "avc_mel_from_frames": [_I, _I, _I, _P, _P, _P],
    "avc_codes_from_encoder": [_I, _I, _P, _P, _P],
    "avc_codes_from_encoder_backward": [_I, _I, _P, _P, _I, _P],
    "avc_decoder_input": [_I, _I, _P, _I, _P, _P, _P],
    "avc_decoder_input_backward": [_I, _I, _I, _P, _P, _I, _P],
    "avc_overlap_average": [_I, _I, _I, _I, _P, _P, _P],
    "avc_overlap_average_backward": [_I, _I, _I, _I, _P, _P, _P, _P],
    "avc_loss_forward": [_P, _I, _Z, _P, _P, _P, _I, _P],
    "avc_loss_backward": [_I, _Z, _P, _P, _P, _P, _P, _I, _P],
    "avc_clip_adam_ema": [_P, _Z, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _I, _F, ctypes.c_double, _P, _P],
    "avc_clip_adam_ema_dev": [_P, _Z, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _I, _F, ctypes.c_double, _P, _P, _P],
    "avc_timing_enable": [_I],
    "avc_lstm_tune": [_I, _I],
    "avc_bptt_mode": [_I],
    "avc_lstm_split_tune": [_I, _I, _I],
    "avc_gemm_tune": [_I],
    "avc_gemm_config": [_I],
    "avc_bn_fuse_band": [_I],
    "avc_bn_fuse": [_I],
    "avc_split_handover": [_I],
    "avc_dead_h_stores": [_I],
    "avc_debug_bnf_inject": [_I],
    "avc_lstm_persist_tune": [_I],
    "avc_lstm_persist_depth": [_I],
    "avc_lstm_persist_layers": [_I],
    "avc_lstm_persist_status": [ctypes.POINTER(ctypes.c_long)],
    "avc_persist_check": [_P, _P, ctypes.POINTER(_I)],
    "avc_lstm_persist_coop": [_I],
    "avc_lstm_persist_inproj": [_I],
    "avc_lstm_persist_qwait": [_I],
    "avc_debug_xl_census": [_P],
    "avc_debug_xl_force_remote": [_I],
    "avc_gemm_plan_rounds": [_I],
    "avc_bn_bwd_frag": [_I],
    "avc_bptt_coalesce": [_I],
    "avc_dg_dual_split": [_I],
    "avc_lstm32_tune": [_I],
    "avc_bptt_persist": [_I],
    "avc_bptt_xcd": [_I],
    "avc_debug_bptt_diag": [_I],
    "avc_debug_persist_inject": [_I],
    "avc_persist_notify": [_P, _P],
    "avc_persist_launches": [_P, ctypes.POINTER(ctypes.c_long)],
    "avc_bptt_persist_eligible": [_I, _I, _I],
    "avc_debug_persist_spin_limit": [ctypes.c_uint],
    "avc_debug_hog": [_P, _I, _I, ctypes.c_long, _P],
    "avc_debug_hog_resident": [_P, ctypes.POINTER(_I)],
    "avc_debug_hog_xcds": [_P, ctypes.POINTER(_I)],
    "avc_graph_mode": [_I],
    "avc_timing_reset": [],
    "avc_timing_read": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)],
    "avc_generator_param_count": [],
    "avc_generator_forward": [_P, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P],
    "avc_generator_forward_cached": [_P, _I, _I, _P, ctypes.c_long, _P, _P, _P, _I, _P, _P, _P, _P],
    "avc_prepared_release": [_P],
    "avc_stft_frames": [ctypes.c_long, _I],
    "avc_mel_basis": [ctypes.c_double, _I, _I, ctypes.c_double, ctypes.c_double, _I, _P, _P],
    "avc_mel_spectrogram": [_P, _P, ctypes.c_long, _I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P],
    "avc_speaker_encoder_param_count": [],
    "avc_speaker_encoder_forward": [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "avc_embedding_mean_normalize": [_I, _I, _P, _P, _P],
    "avc_wavernn_param_count": [_I],
    "avc_wavernn_persist": [_I],
    "avc_wavernn_fallbacks": [],
    "avc_wavernn_proj_tiled": [_I],
    "avc_wavernn_persist_eligible": [_I, _I, _I],
    "avc_debug_wavernn_inject": [_I],
    "avc_debug_wavernn_stamps": [_P, _I],
    "avc_wavernn_upsample": [_P, _P, _I, _P, _P, _P, _P, _P],
    "avc_wavernn_generate": [_P, _P, _I, _P, _P, _I, _I, _I, _I, ctypes.c_ulonglong, _P, _P, _P, _P, _P],
    "avc_wavernn_fold_shape": [ctypes.c_long, _I, _I, _I, ctypes.POINTER(ctypes.c_long),
                               ctypes.POINTER(ctypes.c_long)],
}
_RESTYPES = {"avc_last_error": ctypes.c_char_p, "avc_act_frag_bytes": _Z, "avc_conv_wgrad_image_bytes": _Z}

_lib = None
_lock = threading.RLock()
_contexts = {}


class HipLibraryError(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes library.  Raises if it is absent: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipLibraryError(
                    f"HIP library not found at {LIB_PATH}; build it with `make` (hipcc --offload-arch=gfx950)")
            lib = ctypes.CDLL(LIB_PATH)
            # an A/B build named by AUTOVC_HIP_LIB may predate a symbol; the in-tree build has them all
            ab = "AUTOVC_HIP_LIB" in os.environ
            for name, args in _SIGS.items():
                if ab and not hasattr(lib, name):
                    continue
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, ctypes.c_int)
            _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(status: int, what: str):
    if status != 0:
        msg = load().avc_last_error().decode(errors="replace")
        if status == 1:
            raise ValueError(f"{what}: {msg}")
        raise HipLibraryError(f"{what} failed ({status}): {msg}")


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)


def context(device: torch.device) -> int:
    """Per-device library context (owns the scratch arena)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ctx = _contexts.get(idx)
    if ctx is None:
        with _lock:
            ctx = _contexts.get(idx)
            if ctx is None:
                p = ctypes.c_void_p()
                check(load().avc_context_create(idx, ctypes.byref(p)), "avc_context_create")
                ctx = p.value
                _contexts[idx] = ctx
    return ctx


def stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def persist_launches(device: torch.device) -> int:
    """Persistent launches enqueued on the device's context so far (avc_persist_launches)."""
    n = ctypes.c_long()
    call("avc_persist_launches", context(device), ctypes.byref(n))
    return n.value


def ptr(t) -> int | None:
    """Device pointer of a contiguous fp32 CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("autovc_amd runs on the GPU only (HIP kernels); got a CPU tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"autovc_amd kernels are fp32; got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("autovc_amd kernels need contiguous tensors")
    return t.data_ptr()


TIMING_CLASSES = {"gemm": 0, "lstm_step_fwd": 1, "lstm_step_bwd": 2, "lstm32": 3, "dft64": 4, "lstm2_persist": 5,
                  "lstm1_persist": 6, "wavernn": 7}


def timing_enable(names):
    mask = 0
    for n in names:
        mask |= 1 << TIMING_CLASSES[n]
    call("avc_timing_enable", mask)


def timing_reset():
    call("avc_timing_reset")


def timing_read(name):
    ms, fl, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_long()
    call("avc_timing_read", TIMING_CLASSES[name], ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by),
         ctypes.byref(n))
    return {"ms": ms.value, "flops": fl.value, "bytes": by.value, "launches": n.value}
