"""gemm4's counted-wait K loop is only correct if hipcc never touches a fragment register while its asm LDS read is
outstanding (csrc/gemm4.hip ``G4_CNT``): compile the kernel for gfx950 on the host and simulate the LDS counter
over every 256-row K loop (tools/g4_isa_check.py).  The GPU numerics tests catch the same fault at run time."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from taboo_brittleness_amd import isa_check as g4_isa_check  # noqa: E402


@pytest.mark.skipif(not os.path.exists(g4_isa_check.HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_gemm4_counted_waits_never_touch_outstanding_reads():
    ls = g4_isa_check.loops(g4_isa_check.compile_asm())
    assert sorted(ls) == [f"gemm4_kernel<256, {e}>" for e in range(7)]
    for name, (pre, body) in ls.items():
        assert pre, name
        assert sum("lgkmcnt(" in x and "lgkmcnt(0)" not in x for x in body) >= 16, name   # the counted waits exist
        assert g4_isa_check.check_loop(body, pre) == [], name


def test_checker_flags_a_copy_of_an_outstanding_read():
    body = ["s_waitcnt lgkmcnt(1)", "v_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[4:7], a[0:3]",
            "ds_read_b128 v[8:11], v20 offset:0x800", "ds_read_b128 v[0:3], v20",
            "v_bfi_b32 v30, s4, v9, v9"]
    bad = g4_isa_check.check_loop(body)
    assert bad and "v_bfi_b32" in bad[0]
    # the next pass: lgkmcnt(1) retires v[8:11] but not v[0:3], which the MFMA reads
    assert any("v_mfma" in b for b in bad)
