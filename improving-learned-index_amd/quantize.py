"""CLI: 8-bit quantization of an impact TSV (drop-in for
`python -m src.deep_impact.indexing.quantize -i in -o out [-m max]`,
reference src/deep_impact/indexing/quantize.py:13-58).

Parsing and writing are native host code; max and int(v * 255 / max) run on the
GPU in fp64 (di_quantize_file).  Output bytes equal the reference's.

Multi-GPU (torchrun --nproc-per-node N -m improving_learned_index_amd.quantize ...):
every rank quantizes a contiguous line range with the global max (one
all_reduce(MAX) of the shard maxima, parallel.quantize_sharded); rank 0 joins the
parts into the single-process file.
"""
from __future__ import annotations

import argparse
import ctypes
import logging
from pathlib import Path
from typing import Optional, Union

from . import parallel
from ._lib import check, lib

IMPACT_SCORE_QUANTIZATION_BITS = 8  # src/utils/defaults.py:26
logger = logging.getLogger("quantize")


def _shard_max(path, device=0) -> float:
    used = ctypes.c_double(0.0)
    check(lib().di_quantize_file(str(path).encode(), None, -1.0, IMPACT_SCORE_QUANTIZATION_BITS,
                                 device, ctypes.byref(used)))
    return used.value


def _negative_max(input_file_path, output_file_path):
    """An explicit negative max: the reference's scale is negative, every int(v * scale)
    <= 0, so every line is written empty -- after the same parse (ValueError on a
    malformed line, quantize.py:41-42)."""
    with open(input_file_path, encoding="utf-8") as f, \
            open(output_file_path, "w", encoding="utf-8") as out:
        for line in f:
            for t in line.strip().split(", "):
                _, score = t.strip().split(": ")
                float(score)
            out.write("\n")


def _quantize_one(input_file_path, output_file_path, max_val, device) -> "ctypes.c_double":
    used = ctypes.c_double(0.0)
    check(lib().di_quantize_file(str(input_file_path).encode(), str(output_file_path).encode(),
                                 float(max_val) if max_val is not None else -1.0,
                                 IMPACT_SCORE_QUANTIZATION_BITS, device, ctypes.byref(used)))
    return used


def quantize_file(input_file_path: Union[str, Path], output_file_path: Union[str, Path],
                  max_val: Optional[float] = None, device: int = 0,
                  sharded: Optional[bool] = None) -> float:
    """quantize.py:27-47.  max_val None: the file's max; an explicit 0 raises
    ZeroDivisionError and a negative one writes empty lines, as the reference.
    sharded: None = doc-sharded under torchrun (WORLD_SIZE > 1: every rank must call
    it), False = this process alone quantizes the whole file."""
    if max_val is not None and max_val == 0:
        raise ZeroDivisionError("float division by zero")  # quantize.py:37
    if max_val is not None and max_val < 0:
        _negative_max(input_file_path, output_file_path)
        return float(max_val)
    world, rank, local = parallel.dist_env()
    if world > 1 and sharded is not False:
        parallel.init_group("gloo")
        dev = parallel.rank_device(local)
        return parallel.quantize_sharded(
            input_file_path, output_file_path, max_val, world, rank,
            lambda p: _shard_max(p, dev), lambda i, o, m: _quantize_one(i, o, m, dev))
    used = _quantize_one(input_file_path, output_file_path, max_val, device)
    if max_val is None:
        logger.info(f"Found max value: {used.value}")
    else:
        logger.info(f"Using given max value: {max_val}")
    return used.value


def main(argv=None):
    p = argparse.ArgumentParser(description="Quantize a DeepImpact collection.")
    p.add_argument("-i", "--input_file_path", type=Path, required=True)
    p.add_argument("-o", "--output_file_path", type=Path, required=True)
    p.add_argument("-m", "--max_val", type=float, default=None)
    p.add_argument("--device", type=int, default=0)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    quantize_file(a.input_file_path, a.output_file_path, a.max_val, a.device)


if __name__ == "__main__":
    main()
