"""Every library kernel source's inline-asm loads are never touched before their
lgkmcnt wait in the compiled gfx950 code (tools/asm_wait_scan.py).  A compiler copy
of a register that an asm ds_read is still writing reads stale data; this happened
in attention_v3 before its reads and wait became one asm statement."""
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import asm_wait_scan  # noqa: E402

CSRC = ROOT / "improving-learned-index_amd" / "csrc"


@pytest.mark.skipif(not Path(asm_wait_scan.HIPCC).exists() and shutil.which("hipcc") is None,
                    reason="hipcc not available")
@pytest.mark.parametrize("src", ["enc_attn.hip", "enc_gemm256.hip", "enc_gemm.hip", "enc_misc.hip",
                                 "encoder.hip", "index.hip", "sparse.hip"])
def test_no_early_use_of_asm_lds_reads(src):
    hits = asm_wait_scan.scan_asm(asm_wait_scan.compile_asm(CSRC / src))
    assert hits == [], hits[:5]


def test_scanner_flags_a_copy_before_the_wait():
    asm = "\n".join([
        "_ZN2di1kEv:",
        ";;#ASMSTART", "ds_read_b128 v[4:7], v1", ";;#ASMEND",
        "v_mov_b32_e32 v20, v5",
        ";;#ASMSTART", "s_waitcnt lgkmcnt(0)", ";;#ASMEND",
        "v_mov_b32_e32 v21, v6",
    ])
    hits = asm_wait_scan.scan_asm(asm)
    assert [h[1] for h in hits] == ["v_mov_b32_e32 v20, v5"]
