"""Generate the 128-entry table of ref_logf (cwq_refmath.h): for the top 7 mantissa bits i of
a float's m in [1, 2), c_i = float32(1 / centre_i) (c_0 = 1, c_127 = 1/2) and L_i = -ln(c_i) in double,
less ln 2 for i >= 64 (those use the exponent e + 1, so that results near 0 come from small
terms).  High precision from decimal; prints the C++ initialisers."""
from decimal import Decimal, getcontext
import numpy as np

getcontext().prec = 60
LN2 = Decimal(2).ln()
cs, ls = [], []
for i in range(128):
    # the buckets either side of 1 (v in [1, 1 + 2^-7) and [1 - 2^-8, 1)) take c = 1 / 0.5
    # and L = 0 exactly: log(1 + r) with r = v - 1 exact, no cancellation against L
    c = np.float32(1.0) if i == 0 else np.float32(0.5) if i == 127 else np.float32(1.0 / (1.0 + (i + 0.5) / 128.0))
    L = -Decimal(float(c)).ln()
    if i >= 64:
        L -= LN2
    cs.append(float(c).hex())
    ls.append(float(L).hex())
print("// c_i")
for k in range(0, 128, 4):
    print("    " + ", ".join(f"{h}f" for h in cs[k:k + 4]) + ",")
print("// L_i")
for k in range(0, 128, 4):
    print("    " + ", ".join(ls[k:k + 4]) + ",")
