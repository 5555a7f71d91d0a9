"""The device Nelder-Mead record (gpar-at-scale_amd/csrc/nm_dev.hpp, stepped by chain_carry_lml
in the chains fit) against the host machine (nelder_mead.hpp, pinned to the oracle's NelderMead by
tests/test_host.py): tests/nm/nm_dev_check.cpp steps both on the same objective values over
budgets, tolerances, iteration caps and +inf values, and fails at the first bit that differs."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gpar-at-scale_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_device_nm_record_steps_like_the_host_machine(tmp_path):
    exe = tmp_path / "nm_dev_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unknown-pragmas", "-I", CSRC,
                    os.path.join(ROOT, "tests", "nm", "nm_dev_check.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
