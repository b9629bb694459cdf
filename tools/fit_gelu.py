"""Coefficients of the exp-only GELU used by the GEMM epilogues (csrc/k_gemm.hip gelu2):

    GELU(x) = relu(x) - |x|/2 * erfc(|x|/sqrt2),   erfc(z) ~= 2^P(z), z = min(|x|/sqrt2, 5.7)

P is the degree-6 least-squares fit of log2(erfc(z)) on Chebyshev nodes of [0, 5.7], weighted
by the GELU error each log2-unit causes (|x|/2 * erfc * ln2).  Prints the coefficients
(highest degree first) and the fp32-evaluated max |GELU error| vs the exact erf form over
x in [-12, 12].  usage: python tools/fit_gelu.py
"""
import numpy as np
from scipy.special import erf, erfc

ZMAX, DEG = 5.7, 6


def main():
    z = np.cos(np.pi * (np.arange(4000) + 0.5) / 4000) * ZMAX / 2 + ZMAX / 2
    w = 0.5 * np.sqrt(2) * z * erfc(z) * np.log(2) + 1e-12
    c, *_ = np.linalg.lstsq(np.vander(z, DEG + 1) * w[:, None], np.log2(erfc(z)) * w, rcond=None)
    c = c.astype(np.float32)
    x = np.linspace(-12, 12, 2000001).astype(np.float32)
    zz = np.minimum(np.abs(x) * np.float32(0.70710678), np.float32(ZMAX))
    q = np.full_like(zz, c[0])
    for ci in c[1:]:
        q = q * zz + ci
    g = np.maximum(x, np.float32(0)) - (np.float32(0.5) * np.abs(x)) * np.exp2(q).astype(np.float32)
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    print("coefficients (high -> low):", ", ".join(f"{v:.9e}f" for v in c))
    print(f"max |GELU error| in fp32: {np.abs(g - ref).max():.3e}")


if __name__ == "__main__":
    main()
