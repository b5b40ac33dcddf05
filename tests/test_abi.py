"""The C-ABI library: loads without a GPU and exports every symbol include/codenerf.h declares."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "codenerf.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cn_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib_path():
    import torch  # noqa: F401  (the HIP runtime must come from torch's copy, as in production)
    from codenerf import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "code-nerf_amd", "csrc"), "-j8"], check=True)
    return _lib.LIB_PATH


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ["cn_ray_directions", "cn_ray_bundle", "cn_gather_rays", "cn_sample_uniform", "cn_ray_points",
              "cn_sample_pdf", "cn_posenc", "cn_volume_render", "cn_mlp_pack", "cn_code_bias", "cn_mlp_forward",
              "cn_radiance_field"]:
        assert s in syms, s


def test_library_exports_every_declared_symbol(lib_path):
    lib = ctypes.CDLL(lib_path)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_table_matches_header(lib_path):
    from codenerf import _lib
    assert sorted(_lib.SIGNATURES) == declared_symbols()
    lib = _lib.load(lib_path)
    assert lib.cn_version().decode().startswith("libcodenerf_hip")
    assert lib.cn_mlp_packed_floats(0) == 327424 and lib.cn_mlp_packed_floats(1) == 295936
    assert lib.cn_mlp_packed_floats(3) == 36 * 8192 + 1024
    assert lib.cn_mlp_packed_floats(5) == 36 * 8192 + 1024   # bf16x3_w16: the same 1.15 MB stream as hi/lo bf16
    assert lib.cn_error_string(-1).decode().startswith("invalid argument")


def test_argument_errors_need_no_gpu(lib_path):
    """Argument validation happens on the host before any launch (no device needed)."""
    from codenerf import _lib
    lib = _lib.load(lib_path)
    assert lib.cn_volume_render(None, None, None, 1, 1, None, None, None, None, None, None) == _lib.CN_EINVAL
    assert lib.cn_sample_pdf(None, None, None, 0, None, 1, 300, 8, None, 0, None, None, None) == _lib.CN_EINVAL
    assert lib.cn_radiance_field(None, 0, None, None, 1, None, None, None, None, 1, 1, 1, None, None, None, None) \
        == _lib.CN_EINVAL
    import ctypes
    one = (ctypes.c_int64 * 1)(0)
    assert lib.cn_adamw_step(None, None, None, None, 1, one, one, None, None, one, 0.9, 0.999, 1e-8, None) \
        == _lib.CN_EINVAL


def test_ops_refuse_cpu_tensors():
    import torch
    from codenerf import ops
    with pytest.raises(ValueError):
        ops.posenc(torch.zeros(3, 3), [1.0, 2.0], True)


def test_backward_workspace_layout(lib_path):
    """The d x block sits inside the workspace the library sizes (no hand-kept stride in Python)."""
    from codenerf import _lib
    lib = _lib.load(lib_path)
    for m in (1, 257, 100000):
        ws, off = lib.cn_field_backward_workspace_floats(m), lib.cn_field_backward_dx_offset(m)
        assert 0 < off and off + 90 * m <= ws
    assert lib.cn_field_backward_dx_offset(0) == -1


def test_deterministic_eval_backward_workspace(lib_path):
    """cn_field_backward_fused_workspace_floats: the deterministic eval backward's partials -- up to 8 wave
    rows of 520 g_code floats per workgroup (one per 128-sample tile, at most 512), the workgroups'
    rows, 6 floats per wave of 16 (fp32) / 32 (3xbf16) samples, 3 per sample -- and -1 for bad
    arguments; the ws entry refuses the arguments cn_field_backward_fused refuses, before any launch."""
    from codenerf import _lib
    lib = _lib.load(lib_path)
    up4 = lambda n: (n + 3) // 4 * 4
    for fmt_t, ws in ((_lib.CN_FMT_F32_W16_T, 16), (_lib.CN_FMT_BF16X3_T, 32)):
        for n_rays, s in ((1, 32), (2048, 64), (2048, 128), (37, 64), (100000, 64)):
            m = n_rays * s
            blocks = min((m + 127) // 128, 512)
            want = blocks * 8 * 520 + blocks * 520 + up4((m + ws - 1) // ws * 6) + 3 * m
            assert lib.cn_field_backward_fused_workspace_floats(fmt_t, n_rays, s) == want, (fmt_t, n_rays, s)
        assert lib.cn_field_backward_fused_workspace_floats(fmt_t, 0, 64) == -1
    assert lib.cn_field_backward_fused_workspace_floats(_lib.CN_FMT_F32_W16, 16, 64) == -1   # not a transposed pack
    args = [_lib.CN_FMT_F32_W16_T] + [None] * 7 + [1, 64, 1, None, 1, None, None, None, None, None, None, None, None]
    assert lib.cn_field_backward_fused_ws(*args) == _lib.CN_EINVAL


def test_library_built_from_this_tree(lib_path):
    """cn_version() carries the hash of the sources it was compiled from (codenerf/provenance.py)."""
    from codenerf import _lib, provenance
    lib = _lib.load(lib_path)
    v = provenance.version_of(lib.cn_version().decode())
    assert v.get("src") == provenance.source_hash(), (v, provenance.source_hash())
