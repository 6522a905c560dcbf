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


# C scalar type in icap.h -> the ctypes class a binding must use (ctypes aliases: c_int is c_int32, c_long is
# c_int64 and c_ulong is c_uint64 / c_size_t on this LP64 platform)
_SCALARS = {"int": C.c_int, "int32_t": C.c_int32, "int64_t": C.c_int64, "uint64_t": C.c_uint64, "size_t": C.c_size_t,
            "float": C.c_float}
_STRUCTS = {"icap_gemm_args": _lib.GemmArgs, "icap_attn_args": _lib.AttnArgs, "icap_adamw_args": _lib.AdamWArgs,
            "icap_beam_args": _lib.BeamArgs, "icap_transpose_item": _lib.TransposeItem,
            "icap_colsum_item": _lib.ColsumItem, "icap_ln_param_item": _lib.LnParamItem}


def header_prototypes():
    """name -> (return type, [parameter type]) for every prototype of icap.h (comments stripped, whitespace
    normalised, parameter names dropped)."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for ret, name, params in re.findall(r"([A-Za-z_][\w\s\*]*?)\b(icap_\w+)\s*\(([^)]*)\)\s*;", src):
        ret = " ".join(ret.replace("*", " * ").split())
        ps = []
        for prm in params.split(","):
            prm = " ".join(prm.replace("*", " * ").split())
            if prm in ("", "void"):
                continue
            toks = prm.split()
            ps.append(" ".join(toks[:-1]) if toks[-1] != "*" else prm)  # drop the parameter name
        out[name] = (ret, ps)
    return out


def _ctype_ok(ctype: str, py) -> bool:
    """Does ctypes class `py` bind C type `ctype` (pointers: c_void_p, or POINTER(the struct's class))?"""
    t = ctype.replace("const ", "").strip()
    if t.endswith("*"):
        base = t[:-1].strip()
        if base == "char":
            return py in (C.c_char_p, C.c_void_p)
        if base in _STRUCTS and py is C.POINTER(_STRUCTS[base]):
            return True
        return py is C.c_void_p
    if t == "void":
        return py is None
    return py is _SCALARS[t]


def test_signatures_match_header_prototypes():
    """every binding has the header's arity and C types, so a parameter added to
    icap.h without the binding (or the reverse) fails here instead of shifting the stream handle."""
    protos = header_prototypes()
    assert set(protos) == set(_lib.SIGNATURES)
    for name, (ret, params) in protos.items():
        res, args = _lib.SIGNATURES[name]
        assert len(args) == len(params), f"{name}: header has {len(params)} parameters, binding {len(args)}"
        assert _ctype_ok(ret, res), f"{name}: return {ret} bound as {res}"
        for i, (ct, py) in enumerate(zip(params, args)):
            assert _ctype_ok(ct, py), f"{name}: parameter {i} is {ct}, bound as {py}"


def test_integration_snippets_match_header():
    """The ctypes snippets in INTEGRATION.md run as written against the header: every `lib.icap_X.argtypes = [...]`
    list has the prototype's arity and types, and every `lib.icap_X(...)` call passes that many arguments."""
    import ast

    protos = header_prototypes()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", doc, flags=re.S)
    n_lists = n_calls = 0
    for blk in blocks:
        for node in ast.walk(ast.parse(blk)):
            if (isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Attribute)
                    and node.targets[0].attr == "argtypes"):
                name = node.targets[0].value.attr
                types = eval(compile(ast.Expression(node.value), "<doc>", "eval"), {"C": C})
                params = protos[name][1]
                assert len(types) == len(params), f"INTEGRATION.md {name}: {len(types)} argtypes, header {len(params)}"
                for i, (ct, py) in enumerate(zip(params, types)):
                    assert _ctype_ok(ct, py), f"INTEGRATION.md {name}: parameter {i} is {ct}, doc binds {py}"
                n_lists += 1
            if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                    and node.func.attr.startswith("icap_") and isinstance(node.func.value, ast.Name)
                    and node.func.value.id == "lib"):
                name = node.func.attr
                assert len(node.args) == len(protos[name][1]), f"INTEGRATION.md call of {name}: {len(node.args)} args"
                n_calls += 1
    assert n_lists >= 3 and n_calls >= 3, (n_lists, n_calls)


def test_version_and_workspace_queries():
    lib = _lib.load()
    assert lib.icap_version() >= 1
    assert lib.icap_layernorm_bwd_workspace_bytes(8320, 768) > 0
    assert lib.icap_cross_entropy_workspace_bytes(100) == 400
    assert lib.icap_colsum_workspace_bytes(3200, 3072) >= 3072 * 4
    assert lib.icap_adamw_workspace_bytes(1000) >= 4


@pytest.mark.parametrize("struct,cname", [(_lib.GemmArgs, "icap_gemm_args"), (_lib.AttnArgs, "icap_attn_args"),
                                          (_lib.AdamWArgs, "icap_adamw_args"), (_lib.LnParamItem, "icap_ln_param_item")])
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
