"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel and per launch.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads exactly half the bytes of a wide
coalesced (16 B/lane) streaming read (MI355X_MICROARCH.md §HBM), hence the 2x.
"""
import csv
import re
import json
import sys
from collections import defaultdict
from pathlib import Path


_TARGS = [(r"DF16b", "bf16"), (r"f", "f32"), (r"Li(\d+)E", None), (r"Lb1E", "true"),
          (r"Lb0E", "false"), (r"j", "u32"), (r"i", "i32")]


def _short_mangled(name):
    """_ZN2di14gemm_nt_kernelIDF16bLi1EEEv... -> gemm_nt_kernel<bf16,1> (binutils'
    c++filt cannot demangle DF16b, and rocprofv3's own demangler garbles it)."""
    m = re.match(r"_ZN2di(\d+)", name)
    if not m:
        return None
    n = int(m.group(1))
    pos = m.end()
    ident = name[pos:pos + n]
    pos += n
    if pos >= len(name) or name[pos] != "I":
        return ident
    pos += 1
    args = []
    while pos < len(name) and name[pos] != "E":
        for pat, rep in _TARGS:
            mm = re.compile(pat).match(name, pos)
            if mm:
                args.append(rep if rep is not None else mm.group(1))
                pos = mm.end()
                break
        else:
            return ident
    return f"{ident}<{','.join(args)}>"


def short(name):
    sm = _short_mangled(name)
    if sm:
        return sm
    n = name.split("(")[0]
    return n.split("::")[-1]  # keeps template arguments: gemm256_kernel<6> != <7>


def main(root):
    root = Path(root)
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)   # kernel -> dispatch durations (ns) of every pass
    clocks = defaultdict(list)  # kernel -> GRBM_GUI_ACTIVE / 8 XCDs / that dispatch's ns
    for f in root.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                v = float(row["Counter_Value"])
                vals[k][row["Counter_Name"]].append(v)
                dur = None
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                if dur and dur > 0:
                    durs[k].append(dur)
                    if row["Counter_Name"] == "GRBM_GUI_ACTIVE":
                        clocks[k].append(v / 8.0 / dur)
    out = {"kernels": {}, "note": __doc__.strip().splitlines()[2]}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if durs[k]:
            # durations of the profiled dispatches themselves (the counters' own run)
            d["duration_ns_avg"] = sum(durs[k]) / len(durs[k])
        if clocks[k]:
            # the clock each dispatch held: its busy cycles per XCD over its own duration
            d["effective_clock_ghz"] = sum(clocks[k]) / len(clocks[k])
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"]:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out["kernels"][k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
