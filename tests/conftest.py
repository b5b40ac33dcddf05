"""Shared pytest setup: marker registration and import paths.

``-m "not gpu"`` runs on any CPU host (oracle vs golden fixtures, host logic,
C-ABI load/export checks, gloo world_size-2 tests); ``-m gpu`` needs an
MI355X and calls the HIP path through the C ABI.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "code-nerf_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def rendezvous() -> str:
    """A ``file://`` init_method for a spawned gloo group (or a bench worker): no TCP port to pick and then
    lose to another process before the store binds it (EADDRINUSE, seen once on a shared GPU box)."""
    import tempfile
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="cn_rdv_"), "store")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP path through the C ABI)")


# Achieved parity margins: every at-size parity check reports its observed error and its bound
# through margin(); with CN_MARGINS=<path> set they are appended there as JSON lines (the GPU runs
# set it and the summary goes to profiles/<round>/parity_margins.json), and they are always printed.
MARGINS_PATH = os.environ.get("CN_MARGINS")


def margin(test: str, quantity: str, err: float, bound: float, **info) -> float:
    """Record (and print) ``err`` against ``bound`` for ``test`` / ``quantity``, then assert it."""
    err, bound = float(err), float(bound)
    rec = {"test": test, "quantity": quantity, "err": err, "bound": bound,
           "ratio": (err / bound) if bound > 0 else None, **info}
    print("MARGIN " + json.dumps(rec))
    if MARGINS_PATH:
        with open(MARGINS_PATH, "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert err <= bound, rec
    return err
