"""CPU-only: properties of the built gfx950 code objects in libicap_hip.so (llvm-objdump on the bundles).

No VOP3P packed 2 x 32-bit instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 / v_pk_mov_b32) in any kernel: with them a kernel
co-resident with tile-GEMM waves returned slightly wrong rows (DESIGN.md "Concurrency: the packed-FP32 race", tools/ab/ln_race_probe.py); the
Makefile compiles with -fno-slp-vectorize -fno-vectorize and the sources use no float2 / float4 vector arithmetic."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "gpt2-image-captioning_amd", "icap", "libicap_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _code_objects(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libicap_hip.so not built")
    # a built library is always checked: without the disassembler the guard would pass silently
    assert os.path.exists(OBJDUMP), f"{OBJDUMP} is needed to check the built libicap_hip.so"
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)  # --offloading writes the bundles next to its input
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path)
    objs = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in libicap_hip.so"
    return objs


def test_no_packed_fp32(tmp_path):
    bad = {}
    for o in _code_objects(tmp_path):
        dis = subprocess.run([OBJDUMP, "-d", str(o)], check=True, capture_output=True, text=True).stdout
        # the 2 x 32-bit VOP3P class as a whole (round 6, DESIGN.md "the packed-FP32 race"): the FP32 add / mul / fma
        # and the 64-bit move the vectorizer emits with them
        n = len(re.findall(r"\bv_pk_(?:(?:add|mul|fma)_f32|mov_b32)\b", dis))
        if n:
            bad[o.name] = n
    assert not bad, f"packed-FP32 instructions in {bad}"


def test_makefile_keeps_vectorizers_off():
    """The flags that keep packed FP32 out are in CXXFLAGS, and EXTRA cannot switch the vectorizers back on (the
    Makefile rejects it)."""
    mk = open(os.path.join(HERE, "..", "gpt2-image-captioning_amd", "csrc", "Makefile")).read()
    assert "-fno-slp-vectorize -fno-vectorize" in mk
    r = subprocess.run(["make", "-n", "-C", os.path.join(HERE, "..", "gpt2-image-captioning_amd", "csrc"),
                        "EXTRA=-fslp-vectorize"], capture_output=True, text=True)
    assert r.returncode != 0 and "vectoriz" in (r.stdout + r.stderr), (r.returncode, r.stderr[-400:])
