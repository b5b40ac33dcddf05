"""ctypes binding of libcodenerf_hip.so (the C ABI in include/codenerf.h).

The library is loaded lazily on first use and AFTER ``import torch``, so its
``libamdhip64.so.7`` dependency resolves to the HIP runtime torch already
loaded (one runtime, one set of streams).  There is no CPU fallback: if the
library is missing or no GPU is visible, every op raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CODENERF_LIB", os.path.join(_HERE, "lib", "libcodenerf_hip.so"))

CN_OK, CN_EINVAL, CN_EUNSUPPORTED = 0, -1, -2
CN_NUM_PARAMS = 18
CN_FMT_F32, CN_FMT_BF16X3, CN_FMT_BF16X3_T, CN_FMT_F32_W16, CN_FMT_F32_W16_T, CN_FMT_BF16X3_W16 = 0, 1, 2, 3, 4, 5
FORMATS = {"f32": CN_FMT_F32, "bf16x3": CN_FMT_BF16X3, "bf16x3_t": CN_FMT_BF16X3_T, "f32_w16": CN_FMT_F32_W16,
           "f32_w16_t": CN_FMT_F32_W16_T, "bf16x3_w16": CN_FMT_BF16X3_W16}


def kernel_format(precision: str) -> str:
    """Packed format / field kernel that runs a precision: "f32" -> the 16x16x4 two-waves-per-SIMD
    fp32 kernel ("f32_w16"; CODENERF_F32_KERNEL=v1 selects the 32x32x2 one), "bf16x3" -> itself."""
    if precision == "f32":
        return "f32" if os.environ.get("CODENERF_F32_KERNEL") == "v1" else "f32_w16"
    if precision == "f32_v1":          # fp32, the 32x32x2 one-wave-per-SIMD kernel (mlp.hip)
        return "f32"
    return precision
CN_CODE_BIAS_STRIDE = 520

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_f = ctypes.c_float
_i = ctypes.c_int
_fp = ctypes.POINTER(ctypes.c_float)



class FieldPrep(ctypes.Structure):
    """cn_field_prep (include/codenerf.h): one model's part of cn_field_prepare_models."""
    _fields_ = [("params", ctypes.POINTER(_p)), ("code_bias", _p), ("packed", _p), ("packed_t", _p), ("zero", _p),
                ("n_zero", _i64), ("code_act", _p)]


class CodeDzJob(ctypes.Structure):
    """cn_code_dz_job (include/codenerf.h): one field's part of cn_code_dz."""
    _fields_ = [("params", ctypes.POINTER(_p)), ("g_code", _p), ("workspace", _p)]


class FieldTrainBwd(ctypes.Structure):
    """cn_field_train_bwd (include/codenerf.h): one field's part of cn_field_backward_train_multi."""
    _fields_ = [("packed_t", _p), ("params", ctypes.POINTER(_p)), ("masks", _p), ("saved", _p), ("x_enc", _p),
                ("d_raw", _p), ("pts", _p), ("ro", _p), ("rd", _p), ("z", _p), ("n_rays", _i64), ("n_samples", _i64),
                ("chunk_rows", _i64), ("code_index", _p), ("n_codes", _i64), ("freqs_xyz", _fp), ("freqs_dir", _fp),
                ("workspace", _p), ("grads", ctypes.POINTER(_p)), ("g_code", _p), ("d_pts", _p), ("d_ro", _p),
                ("d_rd", _p)]


class FieldFusedBwd(ctypes.Structure):
    """cn_field_fused_bwd (include/codenerf.h): one field's part of cn_field_backward_fused_multi."""
    _fields_ = [("packed_t", _p), ("masks", _p), ("d_raw", _p), ("pts", _p), ("ro", _p), ("rd", _p), ("z", _p),
                ("n_rays", _i64), ("n_samples", _i64), ("chunk_rows", _i64), ("code_index", _p), ("n_codes", _i64),
                ("freqs_xyz", _fp), ("freqs_dir", _fp), ("g_code", _p), ("d_pts", _p), ("d_ro", _p), ("d_rd", _p),
                ("workspace", _p)]


class CodeActJob(ctypes.Structure):
    """cn_code_act_job (include/codenerf.h): one field's part of cn_code_bias_backward_act_multi."""
    _fields_ = [("params", ctypes.POINTER(_p)), ("code_act", _p), ("g_code", _p), ("grads", ctypes.POINTER(_p)),
                ("workspace", _p)]


# name -> (restype, argtypes); mirrors include/codenerf.h one to one.
SIGNATURES = {
    "cn_version": (ctypes.c_char_p, []),
    "cn_error_string": (ctypes.c_char_p, [_i]),
    "cn_ray_directions": (_i, [_i64, _i64, _f, _f, _f, _p, _p]),
    "cn_ray_bundle": (_i, [_p, _i64, _p, _i64, _p, _p, _p]),
    "cn_gather_rays": (_i, [_p, _p, _i64, _i64, _p, _i64, _p, _p, _p]),
    "cn_pose_rays": (_i, [_p, _p, _p, _p, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p, _p, _p, _p]),
    "cn_pose_rays_backward": (_i, [_p, _p, _p, _i64, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p]),
    "cn_random_select": (_i, [_i64, _i64, _i64, ctypes.c_uint64, ctypes.c_uint64, _p, _p]),
    "cn_pose_error": (_i, [_p, _p, _i64, _p, _p, _p]),
    "cn_srn_unpack": (_i, [_p, _i64, _i64, _i64, _p, _i64, _p, _p, _p]),
    "cn_sample_uniform": (_i, [_p, _p, _i64, _p, _p, _p, _i64, _p, _p, _p, _p]),
    "cn_ray_points": (_i, [_p, _p, _p, _i64, _i64, _p, _p]),
    "cn_sample_pdf": (_i, [_p, _p, _p, _i64, _p, _i64, _i64, _i64, _p, _i64, _p, _p, _p]),
    "cn_posenc": (_i, [_p, _i64, _i64, _fp, _i64, _i, _p, _p]),
    "cn_volume_render": (_i, [_p, _p, _p, _i64, _i64, _p, _p, _p, _p, _p, _p]),
    "cn_mlp_packed_floats": (_i64, [_i]),
    "cn_mlp_pack": (_i, [ctypes.POINTER(_p), _i, _p, _p]),
    "cn_code_bias": (_i, [ctypes.POINTER(_p), _p, _p, _i64, _p, _p]),
    "cn_field_prepare": (_i, [ctypes.POINTER(_p), _p, _p, _i64, _p, _p, _p, _p, _i64, _p]),
    "cn_field_prepare_models": (_i, [ctypes.POINTER(FieldPrep), _i, _p, _p, _i64, _p]),
    "cn_field_train_saved_floats": (_i64, [_i, _i64]),
    "cn_mlp_forward": (_i, [_p, _i, _p, _p, _i64, _p, _i64, _p, _p]),
    "cn_radiance_field": (_i, [_p, _i, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p]),
    "cn_radiance_field_train": (_i, [_p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p, _p]),
    "cn_mlp_forward_train": (_i, [_p, _p, _p, _i64, _p, _i64, _p, _p, _p]),
    "cn_encode_inputs": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p]),
    "cn_field_backward_workspace_floats": (_i64, [_i64]),
    "cn_field_backward_dx_offset": (_i64, [_i64]),
    "cn_field_backward": (_i, [ctypes.POINTER(_p), _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p, _i64, _fp, _fp,
                               _p, ctypes.POINTER(_p), _p, _p, _p, _p, _p]),
    "cn_field_backward_fmt": (_i, [_i, ctypes.POINTER(_p), _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p, _i64,
                                   _fp, _fp, _p, ctypes.POINTER(_p), _p, _p, _p, _p, _p]),
    "cn_field_mask_words": (_i64, [_i64]),
    "cn_radiance_field_masks": (_i, [_p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p, _p]),
    "cn_field_mask_words_fmt": (_i64, [_i, _i64]),
    "cn_radiance_field_masks_fmt": (_i, [_i, _p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p,
                                         _p]),
    "cn_field_backward_fused": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p, _i64, _fp, _fp, _p, _p,
                                     _p, _p, _p]),
    "cn_field_backward_fused_workspace_floats": (_i64, [_i, _i64, _i64]),
    "cn_field_backward_fused_ws": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p, _i64, _fp, _fp, _p,
                                        _p, _p, _p, _p, _p]),
    "cn_radiance_field_train_w16": (_i, [_p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p, _p,
                                         _p]),
    "cn_radiance_field_train_fmt": (_i, [_i, _p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _fp, _fp, _p, _p, _p,
                                         _p]),
    "cn_field_backward_train_workspace_floats": (_i64, [_i64]),
    "cn_field_backward_train": (_i, [_p, ctypes.POINTER(_p), _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p,
                                     _i64, _fp, _fp, _p, ctypes.POINTER(_p), _p, _p, _p, _p, _p]),
    "cn_field_backward_train_fmt": (_i, [_i, _p, ctypes.POINTER(_p), _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p,
                                     _i64, _fp, _fp, _p, ctypes.POINTER(_p), _p, _p, _p, _p, _p]),
    "cn_field_backward_train_multi": (_i, [_i, ctypes.POINTER(FieldTrainBwd), _i, _p]),
    "cn_field_backward_fused_multi": (_i, [_i, ctypes.POINTER(FieldFusedBwd), _i, _p, _p]),
    "cn_code_bias_backward_act_multi": (_i, [ctypes.POINTER(CodeActJob), _i, _p, _p, _i64, _p]),
    "cn_field_backward_x3": (_i, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p, _i64, _fp, _fp, _p, _p, _p, _p,
                                  _p]),
    "cn_code_bias_backward": (_i, [ctypes.POINTER(_p), _p, _p, _i64, _p, _p, _p, ctypes.POINTER(_p), _p]),
    "cn_code_bias_backward_workspace_floats": (_i64, [_i64]),
    "cn_code_bias_backward_act": (_i, [ctypes.POINTER(_p), _p, _p, _i64, _p, _p, ctypes.POINTER(_p), _p, _p]),
    "cn_code_dz": (_i, [ctypes.POINTER(CodeDzJob), _i, _i64, _p, _p, _i, _p]),
    "cn_code_bias_backward_ws": (_i, [ctypes.POINTER(_p), _p, _p, _i64, _p, _p, _p, ctypes.POINTER(_p), _p, _i, _p]),
    "cn_volume_render_backward": (_i, [_p, _p, _p, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _i, _p]),
    "cn_ray_bundle_backward": (_i, [_p, _i64, _i64, _p, _p, _p, _p]),
    "cn_gather_rays_backward": (_i, [_p, _p, _i64, _i64, _p, _i64, _p, _p, _p]),
    "cn_posenc_backward": (_i, [_p, _i64, _i64, _fp, _i64, _i, _p, _p, _p]),
    "cn_ray_points_backward": (_i, [_p, _p, _i64, _i64, _p, _p, _p]),
    "cn_gemm_nn":(_i, [_p, _i64, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p]),
    "cn_gemm_tn": (_i, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p]),
    "cn_gemm_nn_x3": (_i, [_p, _i64, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p]),
    "cn_gemm_tn_x3": (_i, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p]),
    "cn_gemm_tn_workspace_floats": (_i64, [_i64, _i64, _i64]),
    "cn_gemm_tn_ws": (_i, [_i, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p, _p]),
    "cn_render_loss_workspace_doubles": (_i64, [_i64]),
    "cn_render_loss": (_i, [_p, _p, _p, _i64, _i64, _p, _p, _i64, _i64, _f, _p, _p, _p]),
    "cn_render_loss_psnr": (_i, [_p, _p, _p, _i64, _i64, _p, _p, _i64, _i64, _f, _p, _p, _p, _p]),
    "cn_render_loss_backward": (_i, [_p, _p, _p, _i64, _i64, _p, _p, _i64, _i64, _f, _p, _p, _p, _p, _p, _p, _i, _p]),
    "cn_adamw_step": (_i, [_p, _p, _p, _p, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64),
                           ctypes.c_double, ctypes.c_double, ctypes.c_double, _p]),
    "cn_adamw_scalars": (_i, [_i64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(_i64), ctypes.c_double, ctypes.c_double, _p]),
    "cn_adamw_step_dev": (_i, [_p, _p, _p, _p, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64), _p,
                               ctypes.c_double, ctypes.c_double, ctypes.c_double, _p]),
}

_lib: Optional[ctypes.CDLL] = None


class CodeNerfError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise CodeNerfError(
            f"libcodenerf_hip.so not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _check_provenance(lib)
    _lib = lib
    return lib


def _check_provenance(lib) -> None:
    """Refuse a library built from other sources than the tree next to it (codenerf/provenance.py):
    a stale prebuilt .so would otherwise run silently in place of the checked-out kernels."""
    from . import provenance
    if os.environ.get("CODENERF_ALLOW_STALE") == "1" or not os.path.isdir(os.path.join(provenance._PKG, "csrc")):
        return
    built = provenance.version_of(lib.cn_version().decode()).get("src")
    here = provenance.source_hash()
    if built != here:
        raise CodeNerfError(f"{LIB_PATH} was built from sources {built}, the tree holds {here}: rebuild it "
                            "(`make -C code-nerf_amd/csrc`) or set CODENERF_ALLOW_STALE=1")


def check(rc: int, what: str) -> None:
    if rc != CN_OK:
        msg = load().cn_error_string(rc).decode()
        raise CodeNerfError(f"{what} failed: {msg} (code {rc})")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    """The current HIP stream of t's device, as the C ABI's cn_stream_t."""
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def host_floats(values) -> "ctypes.Array":
    vals = [float(v) for v in values]
    return (ctypes.c_float * max(1, len(vals)))(*vals)


def pointer_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), arr
