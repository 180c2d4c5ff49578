#!/usr/bin/env python
"""Diagnostic: build boxmot_amd/lib/libbxassoc_<name>.so with extra -D flags (kernel tuning
sweeps; select one at run time with BX_LIB_PATH).  Usage: build_variant.py NAME [-DX=Y ...]"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from boxmot_amd import _native as N  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = ROOT / "boxmot_amd" / "lib" / f"libbxassoc_{name}.so"
subprocess.run(["/opt/rocm/bin/hipcc", *N.HIPCC_FLAGS, *defs, "-o", str(out),
                *[str(N.CSRC / s) for s in N.SOURCES]], check=True)
print(out)
