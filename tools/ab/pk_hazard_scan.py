"""Round 6: is the packed-FP32 failure of the LayerNorm backward a missing hazard wait in its own
instruction stream? Scans the gfx950 assembly of one kernel built WITH the vectorizers (the form that failed beside
tile-GEMM waves) for every VOP3P packed-FP32 instruction (v_pk_add / mul / fma _f32) and reports, for each, the
writers of its source VGPRs (instruction class, distance in instructions, wait / nop instructions in between) and the
readers of its destination. Usage:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics --save-temps -c layernorm.hip   # no -fno-*vectorize
    python tools/ab/pk_hazard_scan.py layernorm-hip-amdgcn-amd-amdhsa-gfx950.s _ZN4icap14ln_bwd8_kernelItLb1ELi3E
"""
import collections
import re
import sys


def vregs(tok):
    """VGPR numbers named by one operand token: v7, v[4:5]."""
    m = re.fullmatch(r"-?\|?v\[(\d+):(\d+)\]\|?", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"-?\|?v(\d+)\|?", tok)
    return {int(m.group(1))} if m else set()


def parse(lines):
    ins = []
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        ops = [t.strip() for t in re.split(r",\s*", rest.split(" row_")[0].split(" quad_perm")[0]) if t.strip()]
        ins.append((op, ops, s))
    return ins


def klass(op, text):
    if op.startswith("v_pk_") and op.endswith("_f32"):
        return "pk_f32"
    if "row_" in text or "quad_perm" in text or "row_bcast" in text or op.endswith("_dpp"):
        return "dpp"
    if op.startswith("v_permlane"):
        return "permlane"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", op):
        return "trans"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "lane_xfer"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    return "other"


def main(path, sym):
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(sym) and l.rstrip().endswith(":") or
                 (l.startswith(sym) and ": " in l))
    end = next(i for i in range(start + 1, len(text)) if "s_endpgm" in text[i])
    ins = parse(text[start + 1: end + 1])
    print(f"{sym}: {len(ins)} instructions, {sum(1 for o, _, t in ins if klass(o, t) == 'pk_f32')} packed-FP32")
    writer_cls, dist_hist, reader_cls, near = collections.Counter(), collections.Counter(), collections.Counter(), []
    for i, (op, ops, t) in enumerate(ins):
        if klass(op, t) != "pk_f32":
            continue
        dst = vregs(ops[0]) if ops else set()
        for src in ops[1:]:
            rs = vregs(src)
            if not rs:
                continue
            for j in range(i - 1, max(-1, i - 200), -1):
                oj, opsj, tj = ins[j]
                if opsj and vregs(opsj[0]) & rs and not oj.startswith(("s_", "ds_write", "global_store", "buffer_store")):
                    cls = klass(oj, tj)
                    gap = [klass(o2, t2) for o2, _, t2 in ins[j + 1: i]]
                    writer_cls[cls] += 1
                    dist_hist[min(i - j, 9)] += 1
                    if cls in ("dpp", "permlane", "trans", "lane_xfer") or i - j <= 1:
                        near.append((i - j, cls, tj, t, "nop" in gap))
                    break
        for j in range(i + 1, min(len(ins), i + 6)):
            oj, opsj, tj = ins[j]
            if any(vregs(x) & dst for x in opsj[1:]):
                reader_cls[klass(oj, tj)] += 1
    print("writers of packed-FP32 source operands, by class:", dict(writer_cls))
    print("distance (instructions) from that writer:", dict(sorted(dist_hist.items())), "(9 = 9 or more)")
    print("readers of packed-FP32 results within 5 instructions, by class:", dict(reader_cls))
    print(f"packed-FP32 sources written by DPP / permlane / transcendental / lane transfer, or by the instruction "
          f"right before: {len(near)}")
    for d, cls, tj, t, nop in near[:40]:
        print(f"  d={d} {cls:9s} {'(nop between) ' if nop else ''}{tj[:70]:70s} -> {t[:60]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
