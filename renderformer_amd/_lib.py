"""ctypes binding of librfhip.so (the C ABI declared in include/rf.h).

The library is built in-tree by ``__graft_entry__.build()`` into
``renderformer_amd/lib/librfhip.so``.  There is deliberately no fallback: if
the library is missing or no HIP device is present, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RF_LIB", os.path.join(_HERE, "lib", "librfhip.so"))


def source_digest(*names: str) -> str:
    """sha256 (first 16 hex digits) over csrc/<names>: ties a measured counter record (profiles/) to the
    kernel source it was taken on, so a stale record is detected instead of reported."""
    import hashlib
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(_HERE, "csrc", n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


ATTN_SOURCES = ("attention.hip", "common.h")

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float

# name -> argtypes (every function returns int status)
SIGNATURES = {
    "rf_gemm_bf16": [_P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _I, _P, _L, _P],
    "rf_gemm_f16": [_P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _I, _P, _L, _P],
    "rf_rmsnorm_f16": [_P, _L, _P, _F, _P, _L, _I, _I, _P],
    "rf_attn_fwd_sk": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _P, _I, _I, _I, _F, _P, _P, _I, _P],
    "rf_attn_fwd_dt": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _P, _I, _I, _I, _F, _P, _P, _I, _P],
    "rf_swin_attn_fwd_dt": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P],
    "rf_swin_attn_fwd_qkn": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P, _P, _F, _F, _P],
    "rf_rmsnorm": [_P, _L, _P, _F, _P, _L, _I, _I, _P],
    "rf_prenorm": [_P, _L, _P, _P, _L, _P, _I, _I, _I, _P],
    "rf_gemm_add_prenorm": [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _I, _P, _L, _P],
    "rf_gemm_rownorm": [_P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _P, _I, _F, _P, _I, _I, _I, _P, _L, _P],
    "rf_gemm_qk_rope": [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _I, _F, _P, _I, _I, _P, _P, _L, _I, _P, _I, _F, _I,
                        _P, _L, _P],
    "rf_row_rms_scale": [_P, _L, _I, _I, _P, _L, _F, _F, _P],
    "rf_attn_fwd_qn": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _P, _L, _I, _F, _F, _P, _I, _I, _I, _P, _P, _I, _P],
    "rf_qk_norm_rope": [_P, _L, _P, _L, _P, _I, _I, _I, _I, _P, _F, _F, _P, _L, _I, _P, _I, _P],
    "rf_qk_norm_rope_groups": [_P, _L, _L, _P, _L, _L, _P, _I, _I, _I, _I, _I, _P, _L, _F, _F, _P, _L, _I, _P, _I,
                               _P],
    "rf_qk_norm_rope_groups_ilv": [_P, _L, _L, _P, _L, _L, _P, _I, _I, _I, _I, _I, _P, _L, _F, _F, _P, _L, _I, _P, _I,
                               _P],
    "rf_attn_fwd": [_P, _L, _P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _I, _F, _I, _P, _L, _P],
    "rf_attn_fwd_sched": [_P, _L, _P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _F, _P, _P, _I, _P],
    "rf_attn_schedule": [_P, _I, _I, _I, _P],
    "rf_attn_combine": [_P, _L, _I, _I, _P, _I, _P, _L, _P],
    "rf_swin_attn_fwd": [_P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _I, _I, _F, _P],
    "rf_texture_pack": [_P, _L, _I, _I, _I, _P, _P, _L, _P],
    "rf_texture_pack_if": [_P, _P, _L, _I, _I, _I, _P, _P, _L, _P],
    "rf_texture_scan": [_P, _L, _I, _I, _I, _P, _P, _L, _P, _P],
    "rf_texture_scan2": [_P, _L, _I, _I, _I, _P, _P, _L, _P, _P, _P],
    "rf_texture_linear": [_P, _L, _I, _I, _P, _P, _P, _L, _I, _P, _P],
    "rf_gemm_bf16_if": [_P, _P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _I, _P, _L, _P],
    "rf_vn_encode": [_P, _L, _P, _I, _P, _L, _P],
    "rf_vn_encode_dt": [_P, _L, _P, _I, _P, _L, _I, _P],
    "rf_ray_tokens_dt": [_P, _P, _I, _I, _I, _P, _P, _I, _P],
    "rf_patchify_rays_dt": [_P, _I, _I, _I, _P, _I, _P],
    "rf_ray_tokens": [_P, _P, _I, _I, _I, _P, _P, _P],
    "rf_patchify_rays": [_P, _I, _I, _I, _P, _P],
    "rf_scene_pos": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _I, _P, _L, _P],
    "rf_embed": [_P, _L, _P, _I, _I, _P, _I, _P, _L, _P, _F, _P, _L, _P, _F, _P],
    "rf_hdr_output": [_P, _P, _I, _I, _I, _I, _F, _I, _I, _P],
    "rf_conv2d_bf16x3": [_P, _P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I,
                         _P, _P, _I, _F, _P, _L, _P],
    "rf_deconv2d_bf16x3": [_P, _P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P, _P, _P, _I, _P, _L, _P],
    "rf_conv2d_f16": [_P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _I, _F,
                      _P, _L, _P],
    "rf_deconv2d_f16": [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P, _I, _P, _L, _P],
    "rf_split_planes": [_P, _L, _I, _L, _P, _P, _I, _I, _P],
    "rf_upsample_bilinear": [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _I, _P],
    "rf_upsample_bilinear_h": [_P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P],
    "rf_conv1x1_f16_group": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "rf_conv2d_f16_group": [_I, _P, _P],
    "rf_gemm_mx8": [_P, _L, _P, _L, _P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _I, _P],
    "rf_quant_mx8": [_P, _L, _I, _I, _P, _L, _P, _L, _P],
    "rf_device_error": [],
    "rf_clear_device_error": [],
    "rf_f16_range_flag": [],
    "rf_clear_f16_range_flag": [],
    "rf_range_word_new": [_P],
    "rf_range_word_bind": [_P],
    "rf_range_word_read": [_P],
    "rf_range_word_clear": [_P],
    "rf_range_word_free": [_P],
    "rf_debug_raise_device_error": [_I, _P],
    "rf_ktimer_arm": [],
    "rf_ktimer_read": [_P, _I],
    "rf_encoder_forward": [_P, _L, _P, _P],
    "rf_decoder_forward": [_P, _L, _P, _P],
}
RF_ERR_DEVICE = 4

_lock = threading.Lock()
_lib = None


class EncoderLayer(ctypes.Structure):
    """rf.h rf_encoder_layer (device pointers of one TransformerEncoder layer's weights)"""
    _fields_ = [(n, ctypes.c_void_p) for n in ("attn_norm", "w_qkv", "qk_norm", "w_out", "ffn_norm", "w13", "w2")]


class EncoderDesc(ctypes.Structure):
    """rf.h rf_encoder_desc"""
    _fields_ = [("n_layers", _I), ("rows", _I), ("dim", _I), ("n_heads", _I), ("ffn_dim", _I),
                ("operand_dtype", _I), ("eps", _F), ("layers", _P), ("pos", _P), ("ld_pos", _L), ("freqs", _P),
                ("n_freqs", _I), ("problems", _P), ("n_problems", _I), ("bounds", _P), ("grid", _I),
                ("workspace", _P), ("gemm_ws", _P), ("gemm_ws_bytes", _L), ("attn_ws", _P), ("timer_attn", _I),
                ("qk_fused", _I)]


class DecoderLayer(ctypes.Structure):
    """rf.h rf_decoder_layer"""
    _fields_ = [(n, ctypes.c_void_p) for n in ("query_norm", "w_q", "q_norm", "kv_norm", "w_kv", "k_norm", "w_out",
                                               "self_norm", "w_self_in", "self_qk_norm", "w_self_out", "ffn_norm",
                                               "w13", "w2")]


class DecoderTap(ctypes.Structure):
    """rf.h rf_decoder_tap"""
    _fields_ = [("layer", _I), ("p_ld", _I), ("p_hi", _P), ("p_lo", _P)]


class DecoderDesc(ctypes.Structure):
    """rf.h rf_decoder_desc"""
    _fields_ = [("n_layers", _I), ("rows", _I), ("dim", _I), ("n_heads", _I), ("ffn_dim", _I),
                ("operand_dtype", _I), ("eps", _F), ("layers", _P), ("ctx", _P), ("ld_ctx", _L), ("ctx_rows", _I),
                ("ctx_dim", _I), ("ctx_norm", _P), ("w_kv_all", _P), ("kv_rows", _I), ("kv_src_rows", _P),
                ("kv_pos", _P), ("ld_kv_pos", _L), ("k_batch", _I), ("k_norm_all", _P), ("freqs", _P),
                ("n_freqs", _I), ("ray_pos", _P), ("ld_ray_pos", _L), ("ray_pos_div", _I), ("cross_problems", _P),
                ("n_cross", _I), ("cross_bounds", _P), ("cross_grid", _I), ("swin", _I), ("n_images", _I),
                ("grid_h", _I), ("grid_w", _I), ("window", _I), ("shift", _I), ("self_problems", _P), ("n_self", _I),
                ("taps", _P), ("n_taps", _I), ("workspace", _P), ("gemm_ws", _P), ("gemm_ws_bytes", _L),
                ("attn_ws", _P), ("timer_cross", _I), ("qk_fused", _I)]


class HipLibraryError(RuntimeError):
    pass


class DeviceError(RuntimeError):
    """A kernel reported a device-side failure (a stream-K hand-off that timed out, or a range table that does not
    fit its launch): the outputs of that launch are invalid.  ``renderformer_amd.ops.clear_device_error()``
    recovers (it drains the device, clears the error word and drops the stream-K workspaces).  Also raised by a
    deferred fp16 range check (``RenderFormer(range_check="deferred")``) that finds a frame whose fp16 operands
    overflowed."""


def load(require_device: bool = True):
    """Load librfhip.so (torch must be imported first so both share one HIP runtime)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipLibraryError(
                    f"librfhip.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
            lib = ctypes.CDLL(LIB_PATH)
            for name, args in SIGNATURES.items():
                fn = getattr(lib, name, None)
                if fn is None:  # (an older build selected with RF_LIB for an A/B: calling it raises AttributeError)
                    continue
                fn.argtypes = args
                fn.restype = ctypes.c_int
            # return types of the non-int entry points; each guarded like the signature loop above, so an older
            # library selected with RF_LIB loads and only a call to a symbol it lacks fails
            for name, res, args in (("rf_last_error", ctypes.c_char_p, []), ("rf_abi_version", ctypes.c_int, None),
                                    ("rf_build_flags", ctypes.c_int, []),
                                    ("rf_attn_workspace_bytes", ctypes.c_int64, [_L, _I, _I]),
                                    ("rf_gemm_workspace_bytes", ctypes.c_int64, []),
                                    ("rf_scene_pos_partials", ctypes.c_int64, [_I, _I]), ("rf_attn_grid", None, []),
                                    ("rf_encoder_workspace_bytes", ctypes.c_int64, [_I, _I, _I, _I]),
                                    ("rf_decoder_workspace_bytes", ctypes.c_int64, [_P])):
                fn = getattr(lib, name, None)
                if fn is None:
                    continue
                if res is not None:
                    fn.restype = res
                if args is not None:
                    fn.argtypes = args
            _lib = lib
    if require_device and not torch.cuda.is_available():
        raise HipLibraryError("renderformer_amd needs a HIP device (MI355X); none is visible")
    return _lib


def study_build() -> bool:
    """True for the study build of the library (rf_build_flags(): RF_BUILD_STUDY): the measured-slower kernels and
    ablation variants are compiled only there; the production build refuses them (RF_ERR_UNSUPPORTED)."""
    lib = load(require_device=False)
    if getattr(lib, "rf_build_flags", None) is None:  # a pre-round-5 library (RF_LIB): no study variants
        return False
    return bool(lib.rf_build_flags() & 1)


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.rf_last_error().decode(errors="replace")
        if rc == 1:
            raise ValueError(msg)
        if rc == RF_ERR_DEVICE:
            raise DeviceError(f"{name}: {msg} -- recover with renderformer_amd.ops.clear_device_error()")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def stream(device=None) -> int:
    """Current stream of `device` (default: the current device; the model wraps every render in a
    torch.cuda.device guard for its own device, so its launches never land on another device's stream)."""
    return torch.cuda.current_stream(device).cuda_stream
