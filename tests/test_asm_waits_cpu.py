"""Every library kernel source's inline-asm loads are never touched before their
lgkmcnt wait in the compiled gfx950 code (tools/asm_wait_scan.py).  A compiler copy
of a register that an asm ds_read is still writing reads stale data; this happened
in attention_v3 before its reads and wait became one asm statement.  Likewise no
inline-asm instruction reads an MFMA result within the hazard window: an asm v_max3
over the S accumulators read stale values (round 5)."""
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
    text = asm_wait_scan.compile_asm(CSRC / src)
    hits = asm_wait_scan.scan_asm(text)
    assert hits == [], hits[:5]
    # and no inline asm reads an MFMA result inside the MFMA -> VALU hazard window (the
    # compiler's wait states cover its own readers only)
    mh = asm_wait_scan.scan_mfma_asm_reads(text)
    assert mh == [], mh[:5]


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


def test_scanner_flags_an_asm_read_of_a_fresh_mfma_result():
    asm = "\n".join([
        "_ZN2di1kEv:",
        "v_mfma_f32_16x16x32_bf16 v[8:11], v[0:3], v[4:7], 0",
        ";;#ASMSTART", "v_max3_f32 v20, v8, v9, v10", ";;#ASMEND",
        "s_nop 7", "s_nop 7", "s_nop 7",
        ";;#ASMSTART", "v_max3_f32 v21, v8, v9, v10", ";;#ASMEND",
        ";;#ASMSTART", "ds_read_b128 v[8:11], v30", ";;#ASMEND",
    ])
    hits = asm_wait_scan.scan_mfma_asm_reads(asm)
    assert [h[1] for h in hits] == ["v_max3_f32 v20, v8, v9, v10"]
