"""ctypes binding of libsegamd.so -- the C-ABI declared in include/segamd.h.

The library is REQUIRED: there is no CPU or eager-PyTorch fallback on the
product path.  If the shared object is missing or fails to load, `lib()` raises.
Every call returns a hipError_t; `check` turns a non-zero code into an exception.
"""
from __future__ import annotations

import ctypes
import os
import threading

from .build import LIB_PATH, source_hash

_V = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float

# name -> (restype, argtypes); mirrors include/segamd.h one-to-one.
PROTOTYPES = {
    "seg_conv_igemm": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _I, _I, _I, _I, _V, _L, _V, _V]),
    "seg_conv_igemm_act": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _I, _I, _I, _I, _V, _L, _V, _I,
                                _V, _I, _V]),
    "seg_conv_igemm_bf16": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _I, _I, _I, _I, _V, _L, _V, _I,
                                 _V, _I, _V]),
    "seg_conv_igemm_f16": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _I, _I, _I, _I, _V, _L, _V, _I,
                                _V, _I, _V]),
    "seg_conv_igemm_splits": (_I, [_L, _I, _I, _I]),
    "seg_igemm_force_tile": (_I, [_I]),
    "seg_conv_halo_ok": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_halo_pick": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_halo_row_tiles": (_I, [_I, _I, _I]),
    "seg_conv_halo": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _V, _L, _V, _V]),
    "seg_conv_wino_pick": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_wino_row_tiles": (_I, [_I, _I, _I]),
    "seg_conv_wino_tile_rows": (_I, []),
    "seg_conv_wino": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _V, _L, _V, _V, _V]),
    "seg_conv_wino_fused": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _V, _L, _V, _V]),
    "seg_conv_wino_fused_ok": (_I, [_I, _I, _I, _L]),
    "seg_conv_wino_wgrad_pick": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_wino_wgrad_splits": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_wino_wgrad": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _I, _V, _I, _V]),
    "seg_conv_wino_wgrad16_splits": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_wino_wgrad16": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _I, _V, _I, _V]),
    "seg_conv_wino_wgrad_reduce": (_I, [_V, _I, _V, _I, _I, _I, _I, _V]),
    "seg_pack_batch": (_I, [_V, _I, _L, _V]),
    "seg_conv_igemm_row_tiles": (_I, [_L, _I, _V]),
    "seg_pack_conv_weight": (_I, [_V, _V, _I, _I, _I, _I, _I, _I, _V]),
    "seg_conv_wgrad_splits": (_I, [_L, _I, _I, _I]),
    "seg_conv_wgrad_splits_bf16": (_I, [_L, _I, _I, _I]),
    "seg_conv_wgrad": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _V, _I, _V]),
    "seg_conv_wgrad_bf16": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _V, _I, _V]),
    "seg_conv_wgrad_reduce": (_I, [_V, _I, _V, _I, _I, _I, _I, _I, _V]),
    "seg_pack_dw_weight": (_I, [_V, _V, _I, _V]),
    "seg_dw_fwd": (_I, [_V, _L, _I, _I, _I, _I, _V, _V, _I, _V, _V, _L, _I, _I, _I, _V]),
    "seg_dw_fwd_bias_act": (_I, [_V, _L, _I, _I, _I, _I, _V, _V, _I, _V, _L, _I, _I, _I, _V]),
    "seg_dw_dgrad": (_I, [_V, _L, _I, _I, _I, _I, _V, _V, _L, _I, _I, _I, _I, _V]),
    "seg_dw_wgrad_blocks": (_L, [_I, _I, _I, _I]),
    "seg_dw_wgrad": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _V, _V, _I, _I, _I, _I, _V, _V]),
    "seg_nchw_to_nhwc": (_I, [_V, _I, _I, _I, _I, _V, _I, _V]),
    "seg_chan_workspace_floats": (_L, [_L, _I]),
    "seg_bn_stats": (_I, [_V, _L, _L, _I, _V, _V, _F, _F, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "seg_bn_stats_tiles": (_I, [_V, _I, _I, _L, _I, _V, _V, _F, _F, _V, _V, _V, _V, _V, _V, _V, _V]),
    "seg_bn_stats_tiles_ws": (_I, [_V, _I, _I, _L, _I, _V, _V, _F, _F, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "seg_bn_stats_tiles_work_floats": (_L, [_I, _I]),
    "seg_bn_eval_coef": (_I, [_V, _V, _V, _V, _F, _I, _V, _V, _V]),
    "seg_bn_apply": (_I, [_V, _L, _L, _I, _V, _V, _I, _V, _L, _V, _L, _V]),
    "seg_bn_backward": (_I, [_V, _L, _V, _L, _L, _I, _V, _V, _V, _V, _V, _I, _V, _V, _V, _V, _L, _V]),
    "seg_bn_eval_backward": (_I, [_V, _L, _V, _L, _L, _I, _V, _V, _I, _V, _L, _V]),
    "seg_colsum": (_I, [_V, _L, _L, _I, _V, _V, _I, _V]),
    "seg_add": (_I, [_V, _L, _V, _L, _L, _I, _V, _L, _V]),
    "seg_upsample_fwd": (_I, [_V, _L, _I, _I, _I, _I, _V, _L, _I, _I, _I, _V]),
    "seg_upsample_bwd": (_I, [_V, _L, _I, _I, _I, _I, _I, _V, _L, _I, _I, _I, _I, _V]),
    "seg_upsample_to_nchw": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _I, _I, _V]),
    "seg_maxpool2_fwd": (_I, [_V, _L, _I, _I, _I, _I, _V, _L, _V]),
    "seg_maxpool2_bwd": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _V, _L, _I, _V]),
    "seg_ce_workspace_floats": (_L, [_L]),
    "seg_ce_upsample_loss": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _I, _I, _V, _V, _V]),
    "seg_ce_upsample_grad": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _I, _I, _V, _V, _V, _L, _V]),
    "seg_bn_fold_batch": (_I, [_V, _I, _L, _V]),
    "seg_preprocess_bgr": (_I, [_V, _I, _I, _I, _L, _V, _I, _I, _I, _F, _F, _F, _F, _F, _F, _V]),
    "seg_argmax_nearest": (_I, [_V, _L, _I, _I, _I, _I, _I, _I, _V, _I, _I, _V]),
    "seg_resize_u8": (_I, [_V, _I, _I, _I, _L, _V, _I, _I, _I, _V, _V]),
    "seg_augment": (_I, [_V, _V, _I, _I, _I, _V, _F, _F, _F, _F, _F, _F, _V, _V, _V]),
    "seg_adam_step": (_I, [_V, _V, _I, _I, _F, _F, _F, _F, _V]),
    "seg_adam_step_skip": (_I, [_V, _V, _I, _I, _F, _F, _F, _F, _V, _V]),
    # launch tape (csrc/tape.hip, seg_amd/tape.py)
    "seg_tape_fn_index": (_I, [ctypes.c_char_p]),
    "seg_tape_fn_nargs": (_I, [_I]),
    "seg_tape_create": (_I, [_V, _I, _V, _L, _I, _V]),
    "seg_tape_destroy": (_I, [_V]),
    "seg_tape_set_arg": (_I, [_V, _L, _L]),
    "seg_tape_timing": (_I, [_V, _V, _I, _I]),
    "seg_tape_elapsed": (_I, [_V, _V]),
    "seg_tape_timeline": (_I, [_V, _I, _V]),
    "seg_tape_run": (_I, [_V, _I, _V, _V, _V]),
    "seg_set_combine_spin": (_I, [_I]),
    "seg_build_hash": (_I, [ctypes.c_char_p, _I]),
    "seg_conv_igemm2_plan": (_I, [_L, _I, _I, _I, _V]),
    "seg_conv_pw_row_tiles": (_I, [_L]),
    "seg_conv_pw": (_I, [_V, _L, _L, _I, _V, _I, _V, _V, _L, _I, _V, _L, _V, _V, _V, _I, _V]),
    "seg_conv_igemm2_bf16io": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _V, _L, _V, _V, _V]),
    "seg_igemm2_force_tile": (_I, [_I]),
    "seg_igemm2_tune": (_I, [_I, _I]),
    "seg_conv_wgrad2_ok": (_I, [_I, _I, _I, _I, _I]),
    "seg_conv_wgrad2_blocks": (_I, [_I, _I, _I]),
    "seg_conv_wgrad2_bf16io": (_I, [_V, _L, _V, _L, _I, _I, _I, _I, _I, _V, _V]),
    "seg_bn_bwd_coef": (_I, [_V, _L, _V, _L, _L, _I, _V, _V, _V, _V, _V, _I, _V, _V, _V, _V, _V]),
    "seg_bn_bwd_apply": (_I, [_V, _L, _V, _L, _L, _I, _V, _V, _V, _I, _V, _V, _L, _V]),
    "seg_bn_bwd_finalize_tiles": (_I, [_V, _I, _L, _I, _V, _V, _V, _V, _V, _V]),
    "seg_conv_igemm_bnout_ok": (_I, [_L, _I, _I]),
    "seg_mbconv_ok": (_I, [_I, _I, _I, _I, _I]),
    "seg_mbconv_tune": (_I, [_I]),
    "seg_stem_pre_f16": (_I, [_V, _I, _I, _L, _I, _I, _F, _F, _F, _F, _F, _F, _V, _I, _V, _I, _I, _V, _L, _V]),
    "seg_pw2_ok": (_I, [_I, _I, _I]),
    "seg_pw2_f16": (_I, [_V, _L, _L, _I, _V, _V, _I, _I, _V, _V, _I, _V, _L, _V]),
    "seg_conv_igemm_tiles": (_I, [_L, _I]),
    "seg_conv_igemm_act_ic": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _V, _L, _I, _I, _I, _I, _I, _I, _V, _L, _I,
                                   _V, _I, _I, _V, _V]),
    "seg_conv_igemm_plan_b1": (_I, [_L, _I, _I, _I, _V]),
    "seg_mbconv_work_floats": (_L, [_I, _I, _I, _I, _I, _I, _V]),
    "seg_mbconv_f16": (_I, [_V, _L, _I, _I, _I, _I, _V, _V, _I, _V, _V, _I, _V, _V, _I, _V, _L, _V, _L, _V, _V,
                            _V]),
    "seg_conv_igemm_bnout": (_I, [_V, _L, _I, _I, _I, _I, _V, _I, _V, _L, _I, _I, _V, _L, _V, _L, _V, _V, _V, _I,
                                  _V, _V]),
}
# bf16-storage variants: same C signature shape as their fp32 namesakes (pointers stay void*)
for _n in ("seg_add", "seg_bn_stats", "seg_bn_apply", "seg_bn_backward", "seg_colsum", "seg_dw_fwd", "seg_dw_dgrad",
           "seg_dw_wgrad", "seg_ce_upsample_loss", "seg_ce_upsample_grad", "seg_upsample_fwd", "seg_upsample_bwd",
           "seg_upsample_to_nchw", "seg_nchw_to_nhwc", "seg_maxpool2_fwd", "seg_maxpool2_bwd"):
    PROTOTYPES[_n + "_bf16io"] = PROTOTYPES[_n]
PROTOTYPES["seg_conv_igemm_bf16io"] = PROTOTYPES["seg_conv_igemm"]
PROTOTYPES["seg_bn_bwd_coef_bf16io"] = PROTOTYPES["seg_bn_bwd_coef"]
PROTOTYPES["seg_conv_igemm_bnout_bf16io"] = PROTOTYPES["seg_conv_igemm_bnout"]
PROTOTYPES["seg_conv_igemm_bf16_ic"] = PROTOTYPES["seg_conv_igemm_act_ic"]
PROTOTYPES["seg_conv_igemm_f16_ic"] = PROTOTYPES["seg_conv_igemm_act_ic"]
PROTOTYPES["seg_conv_igemm_bnout_bf16io_w16"] = PROTOTYPES["seg_conv_igemm_bnout"]
PROTOTYPES["seg_bn_bwd_apply_bf16io"] = PROTOTYPES["seg_bn_bwd_apply"]
PROTOTYPES["seg_conv_wgrad_bf16io"] = PROTOTYPES["seg_conv_wgrad"]
# lazy-BN (input transform) variants: + in_scale, in_shift, in_act before the stream
for _n in ("seg_conv_igemm", "seg_conv_wgrad"):
    _r, _a = PROTOTYPES[_n]
    for _sfx in ("_xf", "_bf16_xf", "_bf16io_xf"):
        PROTOTYPES[_n + _sfx] = (_r, _a[:-1] + [_V, _V, _I, _V])
PROTOTYPES["seg_conv_halo_bf16io"] = PROTOTYPES["seg_conv_halo"]
PROTOTYPES["seg_conv_igemm_bf16io_w16"] = PROTOTYPES["seg_conv_igemm"]
PROTOTYPES["seg_conv_halo_bf16io_w16"] = PROTOTYPES["seg_conv_halo"]
PROTOTYPES["seg_conv_igemm_bf16io_xf_w16"] = PROTOTYPES["seg_conv_igemm_bf16io_xf"]
PROTOTYPES["seg_conv_pw_bf16io"] = PROTOTYPES["seg_conv_pw"]

_lock = threading.Lock()
_lib = None


class SegLibError(RuntimeError):
    pass


def lib():
    """Load libsegamd.so (must already be built: __graft_entry__.build()).  SEG_LIB_PATH
    may name another build of the same library (A/B timing of kernel variants)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = os.environ.get("SEG_LIB_PATH", LIB_PATH)
            if not os.path.exists(path):
                raise SegLibError(
                    f"HIP library {path} is missing; build it with `python __graft_entry__.py` "
                    "(there is no CPU fallback for the segamd hot path)")
            import torch  # noqa: F401  -- load torch's libamdhip64 first so both share one HIP runtime
            h = ctypes.CDLL(path)
            for name, (res, args) in PROTOTYPES.items():
                if path != LIB_PATH and not hasattr(h, name):
                    continue  # an older A/B build (SEG_LIB_PATH) may predate an entry point
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            if path == LIB_PATH:  # a SEG_LIB_PATH variant is built from other sources on purpose
                buf = ctypes.create_string_buffer(80)
                h.seg_build_hash(buf, 80)
                if buf.value.decode() != source_hash():
                    raise SegLibError(f"HIP library {path} was built from other sources than this tree "
                                      "(source hash mismatch); rebuild it with `python __graft_entry__.py`")
            _lib = h
    return _lib


def check(rc: int, name: str = "") -> None:
    if rc != 0:
        raise SegLibError(f"segamd kernel {name} failed: hipError_t {rc}")


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise SegLibError(f"segamd kernel {name} failed: hipError_t {rc}")
    return rc


def query(name: str, *args) -> int:
    return getattr(lib(), name)(*args)
