"""The C-ABI library builds, loads without a GPU, and exports every symbol
include/crispr_nw.h declares (no compute calls here)."""
import os
import re

from crispresso_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="crispr_nw.h", prefix="nw_"):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", text))


def test_header_and_binding_agree():
    assert declared_symbols() == set(_lib.EXPORTS)
    assert declared_symbols("crispr_quant.h", "nwq_") == set(_lib.QUANT_EXPORTS)
    assert declared_symbols("crispr_flash.h", "nwf_") == set(_lib.FLASH_EXPORTS)
    assert declared_symbols("crispr_synth.h", "nw_synth_") == set(_lib.SYNTH_EXPORTS)


def test_library_exports_every_declared_symbol():
    exported = _lib.exported_symbols()
    missing = [k for k, v in exported.items() if not v]
    assert not missing, missing


def test_create_without_gpu_fails_loudly():
    import ctypes

    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.nw_create(0, ctypes.byref(h))
    if rc == _lib.NW_OK:  # running on a GPU box: fine, clean up
        lib.nw_destroy(h)
    else:
        assert rc == _lib.NW_E_HIP
        assert not h.value


def test_stat_layout_matches_header():
    assert _lib.STAT_DTYPE.itemsize == 32
    assert _lib.STAT_FIELDS[0] == "aln_len" and _lib.STAT_FIELDS[-1] == "flags"
