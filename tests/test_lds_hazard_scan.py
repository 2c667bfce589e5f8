"""The static LDS-read hazard check (tools/lds_hazard_scan.py): the scanner
flags a recycled in-flight destination and accepts a counted wait, and the
CrossNet kernels (the inline-asm fragment reads of crossnet_w4_kernel and
crossnet_dw_w4_kernel) compile free of such hazards.  CPU only: hipcc
cross-compiles for gfx950."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))
import lds_hazard_scan as scan  # noqa: E402

_BAD = """_Zk:
\t;;#ASMSTART
\tds_read_b64_tr_b16 v[66:67], v68
\t;;#ASMEND
\tv_lshl_add_u64 v[66:67], v[148:149], 0, s[0:1]
\tglobal_load_lds_dwordx4 v[66:67], off
\ts_waitcnt lgkmcnt(0)
.Lfunc_end0:
"""

_GOOD = """_Zk:
\t;;#ASMSTART
\tds_read_b128 v[4:7], v1
\t;;#ASMEND
\t;;#ASMSTART
\tds_read_b128 v[8:11], v1 offset:64
\t;;#ASMEND
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(1)
\t;;#ASMEND
\tv_add_f32_e32 v4, v4, v5
\ts_waitcnt lgkmcnt(0)
\tv_add_f32_e32 v8, v8, v9
.Lfunc_end0:
"""


def test_scanner_flags_recycled_destination():
    hits = scan.scan_asm(_BAD)
    assert len(hits) == 1 and hits[0][2].startswith("v_lshl_add_u64")


def test_scanner_accepts_counted_waits():
    assert scan.scan_asm(_GOOD) == []


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc absent")
def test_crossnet_kernels_free_of_lds_hazards():
    hits = scan.scan_file(os.path.join(scan.CSRC, "interact.hip"))
    assert hits == [], hits[:5]
