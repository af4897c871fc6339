"""CLI: 8-bit quantization of an impact TSV (drop-in for
`python -m src.deep_impact.indexing.quantize -i in -o out [-m max]`,
reference src/deep_impact/indexing/quantize.py:13-58).

Parsing and writing are native host code; max and int(v * 255 / max) run on the
GPU in fp64 (di_quantize_file).  Output bytes equal the reference's.
"""
from __future__ import annotations

import argparse
import ctypes
import logging
from pathlib import Path
from typing import Optional, Union

from ._lib import check, lib

IMPACT_SCORE_QUANTIZATION_BITS = 8  # src/utils/defaults.py:26
logger = logging.getLogger("quantize")


def quantize_file(input_file_path: Union[str, Path], output_file_path: Union[str, Path],
                  max_val: Optional[float] = None, device: int = 0) -> float:
    used = ctypes.c_double(0.0)
    check(lib().di_quantize_file(str(input_file_path).encode(), str(output_file_path).encode(),
                                 float(max_val) if max_val is not None else -1.0,
                                 IMPACT_SCORE_QUANTIZATION_BITS, device, ctypes.byref(used)))
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
