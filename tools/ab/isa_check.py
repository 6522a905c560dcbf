"""Quick ISA sanity check of the GEMM kernels in a --save-temps .s: waterfall loops around LDS-DMA and the
vmcnt waits inside the main loop (span from the first to the last MFMA)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "gemm256"
pw = re.compile(r"vmcnt\(\d+\)")
for name in re.findall(r"^(_ZN4icap\w+):", s, re.M):
    if pat not in name:
        continue
    i = s.find(name + ":")
    j = s.find(".Lfunc_end", i)
    lines = s[i:j].split("\n")
    wf = sum(1 for k, l in enumerate(lines)
             if "buffer_load" in l and "lds" in l and any("s_cbranch_execnz" in x for x in lines[k + 1:k + 5]))
    mf = [k for k, l in enumerate(lines) if "v_mfma" in l]
    loop = "\n".join(lines[max(mf[0] - 250, 0):mf[-1] + 5]) if mf else ""
    print(f"{name[:60]:60s} waterfall_dma={wf} loop_waits={pw.findall(loop)}")
