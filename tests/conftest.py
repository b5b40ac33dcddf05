"""Shared pytest setup: marker registration and import paths.

``-m "not gpu"`` runs on any CPU host (oracle vs golden fixtures, host logic,
C-ABI load/export checks, gloo world_size-2 tests); ``-m gpu`` needs an
MI355X and calls the HIP path through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "code-nerf_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP path through the C ABI)")
