"""Build provenance: a hash of the HIP sources the library is compiled from.

``make`` (csrc/Makefile) runs this file as a script and compiles the hash into
``cn_version()``; ``__graft_entry__.smoke()`` recomputes it from the checked-out
tree and asserts the loaded library was built from exactly these sources, so a
GPU record proves which code ran.  No torch import: the Makefile runs it bare.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # code-nerf_amd/
_ROOT = os.path.dirname(_PKG)


def source_files():
    csrc = os.path.join(_PKG, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")))
    files.append(os.path.join(_ROOT, "include", "codenerf.h"))
    return files


def source_hash() -> str:
    """sha256 over (relative path, contents) of every csrc/*.hip, csrc/*.h and include/codenerf.h."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, _ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def git_head() -> str:
    try:
        out = subprocess.run(["git", "-C", _ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                             timeout=10)
        head = out.stdout.strip() or "nogit"
        dirty = subprocess.run(["git", "-C", _ROOT, "status", "--porcelain", "--", "code-nerf_amd/csrc", "include"],
                               capture_output=True, text=True, timeout=10).stdout.strip()
        return head + ("+dirty" if dirty else "")
    except (OSError, subprocess.SubprocessError):
        return "nogit"


def version_of(version_string: str) -> dict:
    """Parse cn_version(): 'libcodenerf_hip <ver> (gfx950) src=<hash> git=<head>'."""
    out = {}
    for tok in version_string.split():
        if "=" in tok:
            k, v = tok.split("=", 1)
            out[k] = v
    return out


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "header":
        print(f'#define CN_SRC_HASH "{source_hash()}"\n#define CN_GIT_HEAD "{git_head()}"')
    else:
        print(source_hash())
