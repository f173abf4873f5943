"""Generate the golden fixtures in tests/golden/.

Two kinds of fixture, kept apart:

1. ANALYTIC known answers (``analytic.json``) computed here in closed form / exact rational
   arithmetic, independent of both the oracle and the product:
   * 1D Gauss-Legendre rules (n = 2, 3, 4) and Gauss-Lobatto nodes (p = 1, 2, 4) on [0, 1]
     (MFEM's H1 default basis and integration points);
   * Q1 element matrices on the unit square / unit cube: mass, stiffness, convection with
     c = (1, -2[, 0.5]) — exact fractions;
   * Q2 1D mass and stiffness (GLL nodes 0, 1/2, 1): exact fractions (tensor factors of the hex
     p=2 operator of BASELINE config 2).
2. ORACLE regression vectors (``oracle_vectors.npz``): outputs of oracle/cdfem_oracle.c on small
   seeded inputs (the reference holds no golden vectors for this path and MFEM is not in the
   image — SURVEY.md §4, §8c — so these pin the oracle against its own history and give the GPU
   tests fixed inputs; they are labelled as oracle-generated, not reference-generated).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys
from fractions import Fraction as F
from math import sqrt

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))


def gauss_legendre_closed(n):
    """Closed-form Gauss-Legendre nodes/weights mapped to [0,1]."""
    if n == 2:
        t = [-1 / sqrt(3), 1 / sqrt(3)]
        w = [1.0, 1.0]
    elif n == 3:
        t = [-sqrt(3 / 5), 0.0, sqrt(3 / 5)]
        w = [5 / 9, 8 / 9, 5 / 9]
    elif n == 4:
        a = sqrt(3 / 7 - 2 / 7 * sqrt(6 / 5))
        b = sqrt(3 / 7 + 2 / 7 * sqrt(6 / 5))
        wa = (18 + sqrt(30)) / 36
        wb = (18 - sqrt(30)) / 36
        t = [-b, -a, a, b]
        w = [wb, wa, wa, wb]
    else:
        raise ValueError(n)
    return [(ti + 1) / 2 for ti in t], [wi / 2 for wi in w]


def gll_closed(p):
    if p == 1:
        return [0.0, 1.0]
    if p == 2:
        return [0.0, 0.5, 1.0]
    if p == 4:
        a = sqrt(3 / 7)
        return [0.0, (1 - a) / 2, 0.5, (1 + a) / 2, 1.0]
    raise ValueError(p)


def poly_int01(coeffs):
    """Exact integral over [0,1] of a polynomial with Fraction coefficients (ascending)."""
    return sum(c / (k + 1) for k, c in enumerate(coeffs))


def pmul(a, b):
    out = [F(0)] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] += x * y
    return out


def pder(a):
    return [k * a[k] for k in range(1, len(a))] or [F(0)]


def lagrange_polys(nodes):
    polys = []
    for j, xj in enumerate(nodes):
        p = [F(1)]
        for k, xk in enumerate(nodes):
            if k != j:
                p = pmul(p, [F(-xk) / (xj - xk), F(1) / (xj - xk)])
        polys.append(p)
    return polys


def matrices_1d(nodes):
    L = lagrange_polys(nodes)
    dL = [pder(p) for p in L]
    n = len(nodes)
    M = [[poly_int01(pmul(L[i], L[j])) for j in range(n)] for i in range(n)]
    K = [[poly_int01(pmul(dL[i], dL[j])) for j in range(n)] for i in range(n)]
    # A[i][j] = int phi_i phi_j'  (test i, trial j)
    A = [[poly_int01(pmul(L[i], dL[j])) for j in range(n)] for i in range(n)]
    return M, K, A


def kron(*ms):
    out = ms[0]
    for m in ms[1:]:
        n1, n2 = len(out), len(m)
        out = [[out[i // n2][j // n2] * m[i % n2][j % n2] for j in range(n1 * n2)] for i in range(n1 * n2)]
    return out


def madd(*ms):
    return [[sum(m[i][j] for m in ms) for j in range(len(ms[0]))] for i in range(len(ms[0]))]


def mscale(s, m):
    return [[s * v for v in row] for row in m]


def tensor_matrices(nodes, dim, c):
    """Exact unit-square/cube element matrices in lexicographic order (x fastest)."""
    M1, K1, A1 = matrices_1d(nodes)
    # lexicographic x-fastest: index = dx + n*dy (+ n^2 dz) -> kron(z, y, x)
    if dim == 2:
        M = kron(M1, M1)
        K = madd(kron(M1, K1), kron(K1, M1))
        Cm = madd(mscale(F(c[0]), kron(M1, A1)), mscale(F(c[1]), kron(A1, M1)))
    else:
        M = kron(M1, M1, M1)
        K = madd(kron(M1, M1, K1), kron(M1, K1, M1), kron(K1, M1, M1))
        Cm = madd(mscale(F(c[0]), kron(M1, M1, A1)), mscale(F(c[1]), kron(M1, A1, M1)),
                  mscale(F(c[2]), kron(A1, M1, M1)))
    return M, K, Cm


def to_float(m):
    return [[float(v) for v in row] for row in m]


def analytic():
    out = {"gauss_legendre": {}, "gll": {}, "elements": {}}
    for n in (2, 3, 4):
        x, w = gauss_legendre_closed(n)
        out["gauss_legendre"][str(n)] = {"x": x, "w": w}
    for p in (1, 2, 4):
        out["gll"][str(p)] = gll_closed(p)
    c3 = (F(1), F(-2), F(1, 2))
    for dim, p in ((2, 1), (3, 1), (2, 2), (3, 2)):
        nodes = [F(0), F(1)] if p == 1 else [F(0), F(1, 2), F(1)]
        M, K, Cm = tensor_matrices(nodes, dim, c3[:dim])
        out["elements"][f"dim{dim}_p{p}"] = {"mass": to_float(M), "stiffness": to_float(K),
                                             "convection": to_float(Cm), "c": [float(v) for v in c3[:dim]]}
    return out


def oracle_vectors():
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    rng = np.random.default_rng(20261015)
    data = {}
    cases = [("h3p2", 3, 3, 2, 0.0), ("h3p2_pert", 3, 3, 2, 0.25), ("h3p1", 3, 4, 1, 0.0),
             ("q2p1", 2, 8, 1, 0.0), ("q2p3_pert", 2, 4, 3, 0.2)]
    for name, dim, n, p, pert in cases:
        m = O.BoxMesh(dim, n, p, perturb=pert)
        c = (1.0, -2.0, 0.5)[:dim]
        x = rng.uniform(-1, 1, m.nl)
        A = O.fa_assemble(m, kappa=0.1, alpha=1.0, s=1.0, c=c)
        data[f"{name}_verts"] = m.verts
        data[f"{name}_dofmap"] = m.dofmap
        data[f"{name}_x"] = x
        data[f"{name}_y"] = A.mult(x)
        data[f"{name}_diag"] = A.diag()
        prm = O.mms_params(O.MMS_SIN, dim, kappa=0.1, s=1.0, c=c, p=p)
        data[f"{name}_b"] = O.lf_assemble(m, prm)
    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **data)


if __name__ == "__main__":
    with open(os.path.join(HERE, "analytic.json"), "w") as f:
        json.dump(analytic(), f, indent=1)
    oracle_vectors()
    print("wrote", os.listdir(HERE))
