"""Compare v_mfma_f64_16x16x4_f64 results with candidate fp64 evaluation orders (exact rationals)."""
import sys
from fractions import Fraction as F
import numpy as np

raw = open(sys.argv[1], "rb").read()
T = int(np.frombuffer(raw[:4], np.int32)[0])
d = np.frombuffer(raw[4:], np.float64)
A = d[:T * 64].reshape(T, 16, 4)
B = d[T * 64:T * 128].reshape(T, 4, 16)
C = d[T * 128:T * 384].reshape(T, 16, 16)
D = d[T * 384:].reshape(T, 16, 16)

def rnd(x):
    return float(x)  # Fraction -> nearest double (correct rounding)

def fma(a, b, c):
    return rnd(F(a) * F(b) + F(c))

cands = {
    "fma k=0..3": lambda a, b, c: fma(a[3], b[3], fma(a[2], b[2], fma(a[1], b[1], fma(a[0], b[0], c)))),
    "fma k=3..0": lambda a, b, c: fma(a[0], b[0], fma(a[1], b[1], fma(a[2], b[2], fma(a[3], b[3], c)))),
    "exact once": lambda a, b, c: rnd(sum((F(a[k]) * F(b[k]) for k in range(4)), F(c))),
    "dot exact + c": lambda a, b, c: rnd(F(rnd(sum((F(a[k]) * F(b[k]) for k in range(4)), F(0)))) + F(c)),
}
hits = {k: 0 for k in cands}
n = 0
for t in range(T):
    for i in range(16):
        for j in range(16):
            a = [float(A[t, i, k]) for k in range(4)]
            b = [float(B[t, k, j]) for k in range(4)]
            c = float(C[t, i, j])
            for k, f in cands.items():
                if f(a, b, c) == D[t, i, j]:
                    hits[k] += 1
            n += 1
for k, v in hits.items():
    print(f"{k:16s} {v}/{n} identical")
