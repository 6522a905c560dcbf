"""Host side of tools/microbench/mx_probe.hip: which operand / scale lane maps of v_mfma_scale_f32_16x16x128_f8f6f4
(e4m3 A and B, E8M0 scales) reproduce the device's outputs exactly. Prints the error of every hypothesis per trial."""
import itertools
import sys

import numpy as np


def e4m3(code):
    code = np.asarray(code, dtype=np.int64)
    s = np.where(code & 0x80, -1.0, 1.0)
    e = (code >> 3) & 15
    m = code & 7
    v = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7.0))
    return s * v


KMAPS = {  # lane l, byte j -> k
    "k=32g+j": lambda l, j: 32 * (l >> 4) + j,
    "k=16g+j|64+16g+j-16": lambda l, j: 16 * (l >> 4) + j if j < 16 else 64 + 16 * (l >> 4) + j - 16,
    "k=8g+j%8+32(j//8)": lambda l, j: 8 * (l >> 4) + j % 8 + 32 * (j // 8),
}


def e4m3_rne(x):
    """fp32 -> e4m3fn value by round-to-nearest-even (|x| <= 448): the quantizer's contract (oracle.mx_quantize)."""
    x = np.asarray(x, dtype=np.float64)
    a = np.abs(x)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -6)))
    step = 2.0 ** (e - 3)
    return np.sign(x) * np.round(a / step) * step  # np.round is half-to-even


def run(path):
    raw = open(path, "rb").read()
    rec = 8 + 2048 * 2 + 256 * 2 + 1024
    ntr = 4
    X = np.frombuffer(raw[ntr * rec: ntr * rec + 8192 * 4], np.float32)
    Q = np.frombuffer(raw[ntr * rec + 8192 * 4: ntr * rec + 8192 * 5], np.uint8)
    dev = e4m3(Q)
    ref = e4m3_rne(X)
    bad = np.nonzero(dev != ref)[0]
    print(f"cvt_pk_fp8_f32 vs RNE e4m3fn: {len(bad)} of {len(X)} differ" +
          (f"; first {[(float(X[i]), float(dev[i]), float(ref[i])) for i in bad[:6]]}" if len(bad) else ""))
    for t in range(ntr):
        b = raw[t * rec:(t + 1) * rec]
        osa, osb = (int(v) for v in np.frombuffer(b[:8], np.int32))
        A = np.frombuffer(b[8:2056], np.uint8).reshape(64, 32)
        B = np.frombuffer(b[2056:4104], np.uint8).reshape(64, 32)
        SA = np.frombuffer(b[4104:4360], np.uint32)
        SB = np.frombuffer(b[4360:4616], np.uint32)
        D = np.frombuffer(b[4616:5640], np.float32).reshape(64, 4)
        got = np.zeros((16, 16))
        for l in range(64):
            for r in range(4):
                got[4 * (l >> 4) + r, l & 15] = D[l, r]
        for (kn, km), sbyte, smap in itertools.product(KMAPS.items(), ["opsel", "byte0"], ["lanegroup", "datak"]):
            Am = np.zeros((16, 128)); Bm = np.zeros((128, 16))
            As = np.zeros((16, 4)); Bs = np.zeros((4, 16))
            for l in range(64):
                for j in range(32):
                    k = km(l, j)
                    Am[l & 15, k] = e4m3(A[l, j]); Bm[k, l & 15] = e4m3(B[l, j])
                ba = osa if sbyte == "opsel" else 0
                bb = osb if sbyte == "opsel" else 0
                ea = (int(SA[l]) >> (8 * ba)) & 255
                eb = (int(SB[l]) >> (8 * bb)) & 255
                kb = (l >> 4) if smap == "lanegroup" else km(l, 0) // 32
                As[l & 15, kb] = 2.0 ** (ea - 127); Bs[kb, l & 15] = 2.0 ** (eb - 127)
            ref = np.zeros((16, 16))
            for kb in range(4):
                sl = slice(32 * kb, 32 * kb + 32)
                ref += (Am[:, sl] * As[:, kb:kb + 1]) @ (Bm[sl, :] * Bs[kb:kb + 1, :])
            err = np.abs(ref - got).max() / np.abs(ref).max()
            err_t = np.abs(ref.T - got).max() / np.abs(ref).max()
            print(f"trial {t} (opsel {osa},{osb}) {kn:24s} scale-byte {sbyte:6s} scale-block {smap:9s}: "
                  f"rel err {err:.3g} (transposed C {err_t:.3g})")


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mx_probe.bin")
