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
    assert lib.jmt_abi_version() == 7
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
    # the fp32 partial slabs (ABI 6: no arrival counters)
    assert lib.jmt_gemm_workspace_bytes(512, 512, 6, 4) == 4 * 6 * 512 * 512 * 4


def test_missing_library_raises(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.JMTError, match="no CPU/torch fallback"):
        _lib.load(str(tmp_path / "nope.so"))
    _lib._lib = None
    _lib.load()


CSRC = os.path.join(REPO, "joint-multimodal-transformer-6th-abaw_amd", "csrc")


def test_host_code_under_asan():
    """SURVEY.md §5 sanitizer build: the library's host code (argument checks, planners, error
    formatting, registration) compiled with AddressSanitizer (`make asan`: -Xarch_host
    -fsanitize=address, device code at -O0 and never launched) and driven through every
    validating entry point of include/jmt.h with invalid arguments (csrc/abi_check.cpp); ASan
    must report nothing and every call must fail with an error message."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not installed")
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-C", CSRC, "asan", "-j", jobs], check=True, timeout=1200,
                   stdout=subprocess.DEVNULL)
    exe = os.path.join(CSRC, "build", "asan", "abi_check")
    syms = subprocess.run(["nm", exe], capture_output=True, text=True).stdout
    assert "__asan_init" in syms or "__asan_report_load" in syms, "not ASan-instrumented"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0"))
    assert "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0 and "abi_check: ok" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_default_build_has_no_bounds_counters():
    assert _lib.load().jmt_bounds_violations(0) == -1


def test_planner_split_k_ping_pong_choice():
    """The planner's split count for the weight-gradient shapes (a few 256 x 256 tiles over
    B x T rows) comes from the split-K ping-pong kernel (cfg 44): one (tile, split) item per CU
    (256 here: the CU count falls back to 256 without a device), at least 4 K-tiles per split;
    shapes with tiles enough, under 24 tiles, K under 8192 rows or not whole 256 x 256 tiles keep
    the previous plan."""
    from jmt._lib import BF16
    lib = _lib.load()
    plan = lambda M, N, K, b: lib.jmt_gemm_plan_splits(BF16, M, N, K, b)
    assert plan(1024, 512, 19200, 6) == 5          # 48 tiles
    assert plan(1024, 512, 19200, 3) == 10         # 24 tiles
    assert plan(1024, 3072, 19200, 1) == 5         # 48 tiles (out_layer1's weight gradient)
    assert plan(3072, 1024, 1536, 1) == 1          # short K (< 8192 rows): no cfg 44
    assert plan(19200, 512, 512, 3) == 1           # 450 tiles: no split
    # under 24 tiles (and M not a multiple of 256) the 128 x 128 split plan keeps its choice
    assert plan(512, 512, 19200, 3) != 21
    assert plan(128, 1024, 19200, 2) != 256 // 8
