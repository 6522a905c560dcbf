"""C-ABI checks that need no GPU: libicap_hip.so loads, exports every entry point include/icap.h declares,
the ctypes binding mirrors the header (names, struct layouts via gcc offsetof), and host-only queries work."""

import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from icap import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "icap.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(icap_\w+)\s*\(", src)))


def test_header_functions_exported_and_bound():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), f"{n} declared in icap.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} declared in icap.h but not bound in _lib.SIGNATURES"
    assert set(_lib.SIGNATURES) == set(names)


def test_version_and_workspace_queries():
    lib = _lib.load()
    assert lib.icap_version() >= 1
    assert lib.icap_layernorm_bwd_workspace_bytes(8320, 768) > 0
    assert lib.icap_cross_entropy_workspace_bytes(100) == 400
    assert lib.icap_colsum_workspace_bytes(3200, 3072) >= 3072 * 4
    assert lib.icap_adamw_workspace_bytes(1000) >= 4


@pytest.mark.parametrize("struct,cname", [(_lib.GemmArgs, "icap_gemm_args"), (_lib.AttnArgs, "icap_attn_args"),
                                          (_lib.AdamWArgs, "icap_adamw_args")])
def test_struct_layout_matches_header(struct, cname):
    fields = [f for f, _ in struct._fields_]
    prog = ["#include <stdio.h>", "#include <stddef.h>", '#include "icap.h"', "int main(void){",
            f'printf("%zu\\n", sizeof({cname}));']
    prog += [f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    prog += ["return 0;}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(prog))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        vals = [int(x) for x in subprocess.check_output([exe]).split()]
    assert vals[0] == C.sizeof(struct)
    for f, off in zip(fields, vals[1:]):
        assert getattr(struct, f).offset == off, f


def test_error_reporting_without_gpu():
    # argument validation runs before any HIP call: a bad GEMM must fail with a message, not crash
    a = _lib.GemmArgs()
    a.M, a.N, a.K = 4, 4, 3  # K not a multiple of 4/8
    a.A = a.B = a.C = 16
    a.lda = a.ldb = a.ldc = 4
    with pytest.raises(_lib.IcapError, match="K must be a multiple"):
        _lib.call("icap_gemm", C.byref(a), None)


def _gemm_args(M, N, K, **kw):
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.in_dtype = a.c_dtype = _lib.BF16
    a.A = a.B = a.C = 1 << 20  # never dereferenced: the plan is host-only
    a.lda, a.ldb, a.ldc = K, K, N
    a.alpha = 1.0
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_gemm_kernel_name_query_without_gpu():
    """icap_gemm_kernel_name names the instantiation icap_gemm would launch (bench.py keys its roofline by it,
    matching rocprofv3's kernel names)."""
    lib = _lib.load()
    assert lib.icap_gemm_kernel_name(C.byref(_gemm_args(8320, 50304, 768, path=2))) is None  # ring kernel removed
    tile = lib.icap_gemm_kernel_name(C.byref(_gemm_args(8320, 50304, 768, path=1))).decode()
    assert tile.startswith("icap::gemm_kernel<") and "unsigned short, unsigned short" in tile
    # automatic choice: the 256 x 256 kernel on many full tile rounds and on long K, the tile kernels on the train
    # step's two-round K = 768 products (the rule measured in profiles/r02_gemm256_bench.txt)
    name = lambda *a, **k: lib.icap_gemm_kernel_name(C.byref(_gemm_args(*a, **k))).decode()  # noqa: E731
    assert name(8320, 50304, 768) == "icap::gemm256_kernel<unsigned short>"
    assert name(4096, 4096, 4096) == "icap::gemm256_kernel<unsigned short>"
    assert name(8320, 3072, 768).startswith("icap::gemm_kernel<")
    assert name(8320, 3072, 768, path=3) == "icap::gemm256_kernel<unsigned short>"
    skinny = lib.icap_gemm_kernel_name(C.byref(_gemm_args(128, 2304, 768))).decode()
    # 2304 columns over 4 row blocks: 3 slabs per block (192 blocks <= 256 CUs), K = 768 in 3 k-steps per wave
    assert skinny == "icap::gemm_skinny_kernel<unsigned short, unsigned short, 3, 2, 3>", skinny
    mp = lib.icap_gemm_kernel_name(C.byref(_gemm_args(128, 768, 3072))).decode()
    assert mp == "icap::gemm_skinny_kernel<unsigned short, unsigned short, 1, 2, 12>", mp
    f32 = lib.icap_gemm_kernel_name(C.byref(_gemm_args(8320, 768, 768, c_dtype=_lib.F32))).decode()
    assert "unsigned short, float" in f32
    assert lib.icap_gemm_kernel_name(C.byref(_gemm_args(8, 8, 3))) is None  # invalid K


def test_beam_layout_exported_and_consistent():
    """BeamState takes the done / anc word offsets from icap_beam_layout (the library's own carve-up),
    not a Python restatement. The offsets are increasing, 16-byte aligned, and total matches the workspace size."""
    from icap import ops

    for B, W, T, L in [(1, 1, 1, 1), (3, 4, 67, 50), (128, 4, 65, 50), (7, 8, 129, 128)]:
        o = ops.beam_layout(B, W, T, L)
        vals = [o[k] for k in ops.BEAM_LAYOUT_FIELDS]
        assert vals == sorted(vals) and all(v % 4 == 0 for v in vals), o
        assert o["total"] * 4 == _lib.load().icap_beam_workspace_bytes(B, W, T, L)
        assert o["anc"] + T * B * W <= o["total"] and o["done"] + B <= o["anc"]
