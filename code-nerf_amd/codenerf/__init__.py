"""codenerf — MI355X-native (gfx950 HIP) Code-NeRF renderer.

A drop-in for the ray-marching hot path of akashsharma02/code-nerf: the
``codenerf.nerf`` and ``codenerf.models`` modules mirror
``view_synthesis.nerf`` and ``view_synthesis.models``; every op runs in
libcodenerf_hip.so (C ABI: include/codenerf.h) on the current HIP stream.
"""
from . import _lib  # noqa: F401

__version__ = "0.2.0"


def load_library():
    """Load libcodenerf_hip.so now (it is otherwise loaded on first use)."""
    return _lib.load()


def build_info() -> dict:
    """{"version": cn_version(), "src": hash compiled in, "git": HEAD at build, "tree_src": hash of this tree}."""
    from . import provenance
    v = _lib.load().cn_version().decode()
    info = provenance.version_of(v)
    return {"version": v, "src": info.get("src"), "git": info.get("git"), "tree_src": provenance.source_hash()}
