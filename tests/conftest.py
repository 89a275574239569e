"""Test configuration: the ``gpu`` marker and import paths.

``-m "not gpu"`` tests run in the build container (no GPU): the oracle against
the golden fixtures, the host-side logic, and the C-ABI library's load/export
check.  ``-m gpu`` tests are the parity tests proper and call the HIP path.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aa-rmvsnet_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
