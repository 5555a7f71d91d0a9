"""Shared pytest setup: `gpu` marker, import paths for the product package and the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gpar-at-scale_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 kernels)")


def pytest_sessionstart(session):
    """Build libgparhip.so in-tree if it is missing (the ABI / host tests load it)."""
    lib = os.path.join(ROOT, "gpar-at-scale_amd", "libgparhip.so")
    if not os.path.exists(lib):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "gpar-at-scale_amd"), "-j8"], check=False)
