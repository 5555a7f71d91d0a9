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


def test_checker_follows_branch_predecessors():
    """A DPP FMA at a loop header: the VALU write just before the back-edge branch is adjacent
    on the taken path even though the instruction laid out before the label is harmless
    (ADVICE r05); a join reached only by a branch, after an unconditional branch, is checked
    against the branch's block only."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dpp_hazard_check as H
    loop = """0000 <k>:
  v_mov_b64_e32 v[4:5], 0
  s_nop 4
0010 <L0>:
  v_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:0 row_mask:0xf bank_mask:0xf
  s_add_u32 s0, s0, 1
  v_mov_b64_e32 v[4:5], v[12:13]
  s_cbranch_scc1 L0
  s_endpgm
"""
    n, hz = H.check_listing(loop)
    assert n == 1 and len(hz) == 1, hz
    join = """0000 <k>:
  v_mov_b64_e32 v[4:5], v[12:13]
  s_cbranch_execz L1
  v_mov_b64_e32 v[8:9], 0
  s_nop 3
  s_branch L2
0020 <L1>:
  s_nop 3
0030 <L2>:
  v_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:0 row_mask:0xf bank_mask:0xf
  s_endpgm
"""
    assert H.check_listing(join) == (1, [])
    safe_loop = loop.replace("  v_mov_b64_e32 v[4:5], v[12:13]\n  s_cbranch_scc1 L0",
                             "  v_mov_b64_e32 v[4:5], v[12:13]\n  s_nop 1\n  s_cbranch_scc1 L0")
    assert H.check_listing(safe_loop) == (1, [])


def test_store_data_hazard_is_flagged():
    """The cause of round 5's wrong gains records: a wide store whose data VGPRs the
    next VALU instruction rewrites; one wait state (s_nop 0) or any other instruction between
    them is enough."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dpp_hazard_check as H
    bad = """0000 <k>:
  global_store_dwordx4 v[94:95], v[32:35], off
  v_mov_b64_e32 v[34:35], v[12:13]
"""
    n, hz = H.check_store_listing(bad)
    assert n == 1 and len(hz) == 1
    ok = bad.replace("off\n", "off\n  s_nop 0\n")
    assert H.check_store_listing(ok) == (1, [])
    other = bad.replace("v[34:35], v[12:13]", "v[36:37], v[12:13]")
    assert H.check_store_listing(other) == (1, [])
