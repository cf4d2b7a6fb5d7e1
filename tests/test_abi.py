"""C-ABI checks that need no GPU: the library loads, exports every symbol include/jmt.h declares,
the ctypes descriptor matches the C struct layout, and argument validation fails loudly."""
import ctypes as C
import os
import re
import subprocess

import pytest

from jmt import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "jmt.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(jmt_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_version():
    lib = _lib.load()
    assert lib.jmt_abi_version() == 3
    assert lib.jmt_kernel_count() > 0


def test_every_declared_symbol_is_exported_and_bound():
    lib = _lib.load()
    fns = header_functions()
    assert len(fns) >= 20
    for f in fns:
        assert hasattr(lib, f), f"{f} not exported"
        assert f in _lib.EXPORTED, f"{f} has no ctypes prototype"


def test_nm_exports_match_header():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = set(re.findall(r" T (jmt_[a-z0-9_]+)", out))
    assert set(header_functions()) <= exported


def test_gemm_desc_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    fields = [f for f, _ in _lib.GemmDesc._fields_]
    body = "\n".join(f'  printf("{f} %zu\\n", offsetof(jmt_gemm_desc, {f}));' for f in fields)
    prog.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "jmt.h"
int main(void) {{
  printf("sizeof %zu\\n", sizeof(jmt_gemm_desc));
{body}
  return 0;
}}
""")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(prog), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    got = dict(line.split() for line in out if line.strip())
    assert int(got["sizeof"]) == C.sizeof(_lib.GemmDesc)
    for f in fields:
        assert int(got[f]) == getattr(_lib.GemmDesc, f).offset, f


def test_argument_validation_fails_loudly():
    lib = _lib.load()
    assert lib.jmt_gemm(None, None) == -1
    assert b"null descriptor" in lib.jmt_last_error()
    d = _lib.GemmDesc()
    d.ab_dtype = 7
    assert lib.jmt_gemm(C.byref(d), None) == -1
    assert b"ab_dtype" in lib.jmt_last_error()
    d.ab_dtype, d.c_dtype = _lib.BF16, _lib.BF16
    d.M, d.N, d.K = 16, 16, 16
    d.n_a = d.n_b = d.n_c = 1
    d.lda, d.ldb = 12, 16          # lda not a multiple of 8 bf16 elements
    assert lib.jmt_gemm(C.byref(d), None) == -1
    assert b"lda" in lib.jmt_last_error()
    with pytest.raises(_lib.JMTError):
        _lib.check(-1, "probe")
    assert lib.jmt_layernorm_fwd(0, 0, 4, 4096, None, 0, None, 0, None, None, 1e-5, None, 0,
                                 None, None, None) == -1


def test_workspace_size():
    lib = _lib.load()
    assert lib.jmt_gemm_workspace_bytes(512, 512, 1, 1) == 0
    assert lib.jmt_gemm_workspace_bytes(512, 512, 6, 4) == 4 * 6 * 512 * 512 * 4


def test_missing_library_raises(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.JMTError, match="no CPU/torch fallback"):
        _lib.load(str(tmp_path / "nope.so"))
    _lib._lib = None
    _lib.load()
