"""CPU-side checks of the drop-in boundary: the HIP library builds for gfx950, loads, and exports
every symbol include/*.h declares; without a GPU the engine fails loudly (no fallback)."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from boxmot_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def lib_path():
    return N.build()


HEADERS = sorted((ROOT / "include").glob("*.h"))


def declared_symbols():
    syms = set()
    for h in HEADERS:
        text = h.read_text()
        syms |= set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(bx_\w+)\s*\(", text, re.M))
    return sorted(syms)


def test_header_matches_binding_table():
    assert declared_symbols() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol(lib_path):
    nm = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (bx_\w+)$", nm, re.M))
    missing = set(declared_symbols()) - exported
    assert not missing, missing
    lib = ctypes.CDLL(str(lib_path))
    for s in declared_symbols():
        assert getattr(lib, s)


def test_code_object_targets_gfx950(lib_path):
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", str(lib_path)], capture_output=True,
                         text=True)
    text = out.stdout + out.stderr
    if out.returncode != 0 or not text.strip():
        text = subprocess.run(["strings", str(lib_path)], capture_output=True, text=True).stdout
    assert "gfx950" in text


@pytest.mark.parametrize("header", HEADERS, ids=lambda h: h.name)
def test_no_torch_types_in_abi(header):
    text = header.read_text()
    assert "torch" not in text.split("*/", 1)[1].lower() and "at::" not in text


def test_engine_without_gpu_fails_loudly(lib_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from boxmot_amd.engine import Engine

    with pytest.raises(N.NativeUnavailable):
        Engine("bytetrack")
    from boxmot_amd.engine import OcsortEngine

    with pytest.raises(N.NativeUnavailable):
        OcsortEngine()
    assert N.device_count() == 0
