"""Static check of the hand-scheduled LDS reads (developer tool + CPU test).

Several kernels read LDS fragments with inline-asm ds_read instructions (so that
the compiler does not drain an in-flight LDS-DMA prefetch with vmcnt(0)) and wait
for them with an explicit s_waitcnt lgkmcnt.  The compiler sees an asm output as
defined when the asm statement ends, so it may legally schedule a copy or a use of
such a register ABOVE the wait -- reading a register the LDS is still writing.
This scans the gfx950 assembly of a source file and reports every instruction
that touches a destination register of an inline-asm ds_read (global / buffer
load) before the next lgkmcnt (vmcnt) wait, and every inline-asm instruction that
touches an MFMA result within the MFMA -> VALU hazard window (scan_mfma_asm_reads).

    python tools/asm_wait_scan.py improving-learned-index_amd/csrc/enc_attn.hip
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

HIPCC = "/opt/rocm/bin/hipcc"


def _regs(s):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", s):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", s):
        out.add(int(m.group(1)))
    return out


def scan_asm(text):
    """[(function, instruction)] touching a pending asm ds_read destination."""
    hits, fn, pending, pending_vm, in_asm = [], None, set(), set(), False
    for ln in text.split("\n"):
        if re.match(r"^_Z\S+:", ln):
            fn, pending, pending_vm = ln.split(":")[0], set(), set()
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if in_asm and t.startswith("ds_read"):
            pending |= _regs(t.split()[1].rstrip(","))
        elif in_asm and re.match(r"(global_load|buffer_load)", t) and "lds" not in t:
            pending_vm |= _regs(t.split()[1].rstrip(","))
        elif "s_waitcnt" in t and ("lgkmcnt" in t or "vmcnt" in t):
            if "lgkmcnt" in t:
                pending = set()
            if "vmcnt" in t:
                pending_vm = set()
        elif (pending or pending_vm) and not in_asm and re.match(r"(v_|global_|buffer_|ds_|flat_)", t):
            ops = t.split(None, 1)[1].split(",") if " " in t else []
            touched = set()
            for o in ops:
                touched |= _regs(o)
            if touched & (pending | pending_vm):
                hits.append((fn, t))
    return hits


def scan_mfma_asm_reads(text, window=24):
    """[(function, asm instruction)] reading (a source operand) a VGPR that an MFMA wrote fewer than
    `window` wait states (instructions, s_nop n counting n + 1) earlier in program order.
    The compiler inserts the MFMA -> VALU hazard wait states before its own readers of an
    MFMA result, not before an inline-asm one (an asm v_max3 over the S accumulators read
    stale values, round 5).  Linear scan: conservative across branches."""
    hits, fn, recent, in_asm = [], None, [], False
    for ln in text.split("\n"):
        if re.match(r"^_Z\S+:", ln):
            fn, recent = ln.split(":")[0], []
        t = ln.strip()
        if not t or t.startswith((";", ".")) and not t.startswith(";;#ASM"):
            continue
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"s_nop\s+(\d+)", t)
        step = int(m.group(1)) + 1 if m else 1
        if in_asm and recent and re.match(r"(v_|ds_|global_|buffer_)", t):
            # source operands only (a read-after-write; the destination of an asm load
            # lands after the LDS / memory latency)
            ops = (t.split(None, 1)[1] if " " in t else "").split(",")[1:]
            touched = set()
            for o in ops:
                touched |= _regs(o)
            if any(touched & regs for regs, _ in recent):
                hits.append((fn, t))
        if re.match(r"v_mfma", t):
            recent.append((_regs(t.split(None, 1)[1].split(",")[0]), 0))
        recent = [(r, d + step) for r, d in recent if d + step < window]
    return hits


def compile_asm(src, arch="gfx950"):
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "k.s"
        subprocess.run([HIPCC, f"--offload-arch={arch}", "-O3", "-std=c++17", "--cuda-device-only",
                        "-I", str(Path(src).resolve().parent), "-S", "-o", str(out), str(src)],
                       check=True, capture_output=True)
        return out.read_text()


def main(argv):
    bad = 0
    for src in argv:
        text = compile_asm(src)
        hits = scan_asm(text)
        print(f"{src}: {len(hits)} early touch(es) of pending asm loads")
        for fn, ins in hits[:10]:
            print("   ", fn[:70], "|", ins)
        mh = scan_mfma_asm_reads(text)
        print(f"{src}: {len(mh)} inline-asm touch(es) of fresh MFMA results")
        for fn, ins in mh[:10]:
            print("   ", fn[:70], "|", ins)
        bad += len(hits) + len(mh)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
