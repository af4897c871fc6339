"""Instruction-class count of attention_x3's hot loop, per 32-key sub-chunk (static, ISA).

Compiles csrc/enc_attn.hip for gfx950, takes the shipped instantiation
(attention_x3_kernel<true, true, true, 8, 3>), finds its two-tile whole-chunk loop (the
backward branch whose body holds 2 x 48 MFMAs: two 32-key sub-chunks of 12 S^T + 12
O^T products per query tile), and counts instruction classes over that body, split
into the common path, the rescale branch (the blocks with the permlane max: taken
when a score passes the lazy max), and the per-chunk staging (barrier + LDS-DMA).
The stage buffer (0 / 1) picks one of two fragment-read blocks per site at run time:
those blocks count half.  Static counts: branches taken rarely (a partial chunk's
masks, the rescale's exec-masked multiply) still count in their part.

    python tools/isa_mix.py [--kernel NAME] [--json out.json]
"""
import argparse
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import asm_wait_scan  # noqa: E402  (compile_asm)

SRC = Path(__file__).resolve().parents[1] / "improving-learned-index_amd" / "csrc" / "enc_attn.hip"
KERNEL = "_ZN2di19attention_x3_kernelILb1ELb1ELb1ELi8ELi3ELi64EEEvPKDF16bPKiiiiPDF16bS4_S4_i"

CLASSES = [
    ("mfma", r"v_mfma"),
    ("permlane", r"v_permlane"),
    ("exp", r"v_exp"),
    ("split (cvt / perm to bf16)", r"v_cvt|v_perm"),
    ("max", r"v_max|v_pk_max"),
    ("compare / select", r"v_cmp|v_cndmask"),
    ("f32 arithmetic", r"v_(pk_)?(fma|fmac|fmamk|fmaak|mul|add|sub)_f32"),
    ("move", r"v_mov|v_accvgpr"),
    ("bit / integer", r"v_(and|or|xor|lshl|lshr|ashr|bfe|bfi|bitop3|not|add_u32|sub_u32|add3|lshl_add|lshl_or|and_or|mad_u|mul_lo|mul_hi|readfirstlane|readlane|writelane)"),
    ("LDS read", r"ds_read"),
    ("LDS-DMA", r"global_load_lds|buffer_load.*lds"),
    ("wait", r"s_waitcnt"),
    ("barrier", r"s_barrier"),
    ("branch", r"s_cbranch|s_branch"),
    ("scalar", r"s_"),
    ("other vector", r"v_|global_|buffer_|ds_"),
]


def classify(ins):
    for name, pat in CLASSES:
        if re.match(pat, ins):
            return name
    return "other"


def blocks_of(text, kernel):
    i = text.index(kernel + ":")
    j = text.index(".Lfunc_end", i)
    blocks, cur = [], None
    for ln in text[i:j].split("\n"):
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?", ln)
        if m:
            cur = {"label": m.group(1), "ins": []}
            blocks.append(cur)
            continue
        t = ln.strip()
        if cur is None or not t or t.startswith(";") or t.startswith("."):
            continue
        cur["ins"].append(t.split()[0])
        cur.setdefault("targets", []).extend(re.findall(r"(\.LBB\d+_\d+)", t))
    return blocks


def hot_loop(blocks, mfma_per_iter=96):
    """(first, last) block index of the smallest backward-branch range with the MFMA count."""
    index = {b["label"]: k for k, b in enumerate(blocks)}
    best = None
    for k, b in enumerate(blocks):
        for tgt in b.get("targets", []):
            s = index.get(tgt)
            if s is None or s > k:
                continue
            n = sum(ins.startswith("v_mfma") for bb in blocks[s:k + 1] for ins in bb["ins"])
            if n == mfma_per_iter and (best is None or k - s < best[1] - best[0]):
                best = (s, k)
    return best


def mix(kernel=KERNEL):
    text = asm_wait_scan.compile_asm(SRC)
    blocks = blocks_of(text, kernel)
    rng = hot_loop(blocks)
    if rng is None:
        raise SystemExit("no loop with 96 MFMAs found")
    parts = {"common": {}, "rescale (rare)": {}, "staging (per 64-key chunk)": {}}
    for b in blocks[rng[0]:rng[1] + 1]:
        ins = b["ins"]
        # a fragment-read arm of the stage-buffer choice (only reads, a wait, a branch):
        # one of each pair runs
        arm = all(x.startswith(("ds_read", "s_waitcnt", "s_branch", "s_cbranch")) for x in ins) and any(
            x.startswith("ds_read") for x in ins)
        w = 0.5 if arm else 1.0
        if any(x.startswith("v_permlane") for x in ins):
            part = "rescale (rare)"
        elif any(x.startswith("s_barrier") or "lds" in x and x.startswith("global_load") for x in ins):
            part = "staging (per 64-key chunk)"
        else:
            part = "common"
        for x in ins:
            c = classify(x)
            parts[part][c] = parts[part].get(c, 0) + w
    # per 32-key sub-chunk: the loop body is one 64-key chunk = 2 sub-chunks
    per_sub = {p: {c: v / 2 for c, v in d.items()} for p, d in parts.items()}
    return {"kernel": kernel, "blocks": [blocks[rng[0]]["label"], blocks[rng[1]]["label"]],
            "per_32key_subchunk": per_sub}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default=KERNEL)
    ap.add_argument("--json")
    a = ap.parse_args()
    r = mix(a.kernel)
    print(f"{r['kernel']}: loop {r['blocks'][0]} .. {r['blocks'][1]}, per 32-key sub-chunk (two query tiles)")
    for part, d in r["per_32key_subchunk"].items():
        tot = sum(d.values())
        vec = sum(v for c, v in d.items() if c not in ("mfma", "wait", "barrier", "branch", "scalar", "LDS read", "LDS-DMA"))
        print(f"  {part}: {tot:g} instructions, {vec:g} VALU, {d.get('mfma', 0):g} MFMA")
        for c, v in sorted(d.items(), key=lambda kv: -kv[1]):
            print(f"    {c:28s} {v:g}")
    if a.json:
        Path(a.json).write_text(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
