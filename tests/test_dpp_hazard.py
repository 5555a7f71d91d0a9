"""The inline-asm DPP64 FMAs of the filter recursions (fmac_row, device_common.hpp) are invisible
to the compiler's hazard recognizer: check the built library's gfx950 code for a VALU write of a
DPP source within the two preceding instructions (tools/dpp_hazard_check.py).  CPU only: it reads
the in-tree libgparhip.so with the ROCm LLVM tools."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gpar-at-scale_amd", "libgparhip.so")
TOOLS = ["/opt/rocm/lib/llvm/bin/llvm-objcopy", "/opt/rocm/lib/llvm/bin/clang-offload-bundler",
         "/opt/rocm/lib/llvm/bin/llvm-objdump"]


@pytest.mark.skipif(not os.path.exists(LIB) or not all(os.path.exists(t) for t in TOOLS),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_dpp_source_written_by_valu_just_before():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dpp_hazard_check.py"), LIB],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    n = int(r.stdout.split()[1])
    assert n > 1000   # the whitening, adjoint and cached-whitening instantiations


def test_checker_flags_a_hazard():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dpp_hazard_check as H
    ok = """0000 <k>:
  v_mov_b64_e32 v[2:3], 0
  s_waitcnt lgkmcnt(0)
  v_add_f64 v[8:9], v[8:9], v[10:11]
  v_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:0 row_mask:0xf bank_mask:0xf
"""
    bad = """0000 <k>:
  v_mov_b64_e32 v[2:3], 0
  v_mov_b64_e32 v[4:5], v[12:13]
  v_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:0 row_mask:0xf bank_mask:0xf
"""
    nop = """0000 <k>:
  v_mov_b64_e32 v[4:5], v[12:13]
  s_nop 1
  v_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:0 row_mask:0xf bank_mask:0xf
"""
    assert H.check_listing(ok) == (1, [])
    n, hz = H.check_listing(bad)
    assert n == 1 and len(hz) == 1
    assert H.check_listing(nop) == (1, [])
