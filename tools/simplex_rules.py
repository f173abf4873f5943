"""Generate the tabulated simplex quadrature rules of MFEM's IntegrationRules (intrules.cpp, the
rules IntRules.Get(Geometry::TRIANGLE / TETRAHEDRON, order) returns; MFEM is not vendored here, so
this restates them from MFEM's published tables: orbit structure and parameters).

Each rule is written as symmetric orbits (MFEM's AddTriMidPoint / AddTriPoints3 / AddTriPoints3R /
AddTriPoints6, AddTetMidPoint / AddTetPoints4 / AddTetPoints6 / AddTetPoints12) with the published
parameters; the parameters are then refined by Newton's method on the moment equations of the rule's
degree (so the tables carry full double precision and are exact to that degree), and the script
prints the C tables for continuum-mechanics-mfem_amd/csrc/simplex_rules.inc and
oracle/simplex_rules.inc.  Reference measure: the unit simplex (area 1/2, volume 1/6), MFEM's
weights.

    python tools/simplex_rules.py > /tmp/rules.inc
"""
import itertools
import math

import numpy as np

# ---- triangle orbits: generators of (x, y) point lists from parameters -----------------------------


def tri_mid():
    return [(1 / 3, 1 / 3)]


def tri_p3(a, b=None):              # AddTriPoints3(a[, b]): (a,a), (a,b), (b,a); b = 1 - 2a
    b = 1 - 2 * a if b is None else b
    return [(a, a), (a, b), (b, a)]


def tri_p3r(a, b, c=None):          # AddTriPoints3R(a, b[, c]): (a,b), (c,a), (b,c); c = 1 - a - b
    c = 1 - a - b if c is None else c
    return [(a, b), (c, a), (b, c)]


def tri_p6(a, b, c=None):           # AddTriPoints6(a, b[, c])
    c = 1 - a - b if c is None else c
    return [(a, b), (b, a), (a, c), (c, a), (b, c), (c, b)]


# rules: order -> list of (orbit kind, params, weight); "3b" = AddTriPoints3b(b): a = (1 - b) / 2
TRI = {
    1: [("mid", (), 0.5)],
    2: [("3", (1 / 6,), 1 / 6)],
    3: [("mid", (), -0.28125), ("3", (0.2,), 25 / 96)],
    4: [("3", (0.091576213509770743460,), 0.054975871827660933819),
        ("3", (0.44594849091596488632,), 0.11169079483900573285)],
    5: [("mid", (), 0.1125), ("3", (0.10128650732345633880,), 0.062969590272413576298),
        ("3", (0.47014206410511508977,), 0.066197076394253090369)],
    6: [("3", (0.063089014491502228340,), 0.025422453185103408460),
        ("3", (0.24928674517091042129,), 0.058393137863189683013),
        ("6", (0.053145049844816947353, 0.31035245103378440542), 0.041425537809186787597)],
    7: [("3r", (0.062382265094402118174, 0.067517867073916085443), 0.026517028157436251429),
        ("3r", (0.055225456656926611737, 0.32150249385198182267), 0.043881408714446055037),
        ("3r", (0.034324302945097146470, 0.66094919618673565761), 0.028775042784981585738),
        ("3r", (0.51584233435359177926, 0.27771616697639178257), 0.067493187009802774463)],
    8: [("mid", (), 0.0721578038388935841255455552445323),
        ("3", (0.170569307751760206622293501491464,), 0.0516086852673591251408957751460645),
        ("3", (0.0505472283170309754584235505965989,), 0.0162292488115990401554629641708902),
        ("3", (0.459292588292723156028815514494169,), 0.0475458171336423123969480521942921),
        ("6", (0.008394777409957605337213834539296, 0.263112829634638113421785786284643),
         0.0136151570872174971324223450369544)],
    9: [("mid", (), 0.0485678981413994169096209912536443),
        ("3b", (0.020634961602524744433,), 0.0156673501135695352684274156436046),
        ("3b", (0.12582081701412672546,), 0.0389137705023871396583696781497019),
        ("3", (0.188203535619032730240961280467335,), 0.0398238694636051265164458871320226),
        ("3", (0.0447295133944527098651065899662763,), 0.0127888378293490156308393992794999),
        ("6", (0.0368384120547362836348175987833851, 0.2219629891607656956751025276931919),
         0.0216417696886446886446886446886446)],
}


def tri_points(kind, prm):
    if kind == "mid":
        return tri_mid()
    if kind == "3":
        return tri_p3(*prm)
    if kind == "3b":
        b = prm[0]
        return tri_p3((1 - b) / 2, b)
    if kind == "3r":
        return tri_p3r(*prm)
    if kind == "6":
        return tri_p6(*prm)
    raise ValueError(kind)


# ---- tetrahedron orbits ---------------------------------------------------------------------------
def tet_points(kind, prm):
    if kind == "mid":
        return [(0.25, 0.25, 0.25)]
    if kind == "4":                 # AddTetPoints4(a): three coordinates a, the fourth 1 - 3a
        a = prm[0]
        b = 1 - 3 * a
        return [(a, a, a), (a, a, b), (a, b, a), (b, a, a)]
    if kind == "6":                 # AddTetPoints6(a): two coordinates a, two b = 1/2 - a
        a = prm[0]
        b = 0.5 - a
        return [(a, a, b), (a, b, a), (b, a, a), (a, b, b), (b, a, b), (b, b, a)]
    if kind == "12":                # AddTetPoints12(a, bc): two a, then b, c with b + c = 1 - 2a
        a, b = prm
        c = 1 - 2 * a - b
        bary = set(itertools.permutations((a, a, b, c)))
        return sorted((p[1], p[2], p[3]) for p in bary)
    raise ValueError(kind)


TET = {
    1: [("mid", (), 1 / 6)],
    2: [("4", (0.13819660112501051518,), 1 / 24)],
    3: [("mid", (), -2 / 15), ("4", (1 / 6,), 0.075)],
    4: [("mid", (), -0.0131555555555555556), ("4", (1 / 14,), 0.00762222222222222222),
        ("6", (0.100596423833200785,), 0.0248888888888888889)],
    5: [("4", (0.31088591926330060980,), 0.018781320953002641800),
        ("4", (0.092735250310891226402,), 0.012248840519393658257),
        ("6", (0.045503704125649649492,), 0.0070910034628469110730)],
    6: [("4", (0.21460287125915202929,), 0.0066537917096945820166),
        ("4", (0.040673958534611353116,), 0.0016795351758867738247),
        ("4", (0.32233789014227551034,), 0.0092261969239424536825),
        ("12", (0.063661001875017525299, 0.26967233145831580803), 0.0080357142857142857143)],
}


def monomial_integral(exps):
    """int over the unit simplex of prod x_i^e_i = prod e_i! / (d + sum e)!"""
    d = len(exps)
    return math.prod(math.factorial(e) for e in exps) / math.factorial(d + sum(exps))


def expand(rule, pts_of):
    P, W = [], []
    for kind, prm, w in rule:
        for p in pts_of(kind, prm):
            P.append(p)
            W.append(w)
    return np.array(P), np.array(W)


def residual(flat, rule, pts_of, dim, deg):
    # unpack parameters
    k = 0
    r2 = []
    for kind, prm, _ in rule:
        n = len(prm)
        r2.append((kind, tuple(flat[k:k + n]), flat[k + n]))
        k += n + 1
    P, W = expand(r2, pts_of)
    res = []
    for tot in range(deg + 1):
        for e in itertools.product(range(tot + 1), repeat=dim):
            if sum(e) != tot:
                continue
            q = float(np.sum(W * np.prod(P ** np.array(e), axis=1)))
            res.append(q - monomial_integral(e))
    return np.array(res), r2


def refine(rule, pts_of, dim, deg):
    x = np.array([v for _, prm, w in rule for v in (*prm, w)], dtype=float)
    fixed = [i for i, v in enumerate(x)]
    for _ in range(50):
        r, _ = residual(x, rule, pts_of, dim, deg)
        if np.abs(r).max() < 1e-17:
            break
        J = np.zeros((len(r), len(x)))
        h = 1e-7
        for i in range(len(x)):
            xp = x.copy()
            xp[i] += h
            J[:, i] = (residual(xp, rule, pts_of, dim, deg)[0] - r) / h
        dx = np.linalg.lstsq(J, -r, rcond=None)[0]
        x += dx
    r, rule2 = residual(x, rule, pts_of, dim, deg)
    del fixed
    return rule2, float(np.abs(r).max())


def main():
    out = ["/* generated by tools/simplex_rules.py: MFEM IntRules simplex tables, refined to double precision */"]
    for name, table, pts_of, dim in (("tri", TRI, tri_points, 2), ("tet", TET, tet_points, 3)):
        for deg, rule in sorted(table.items()):
            rule2, err = refine(rule, pts_of, dim, deg)
            drift = max(abs(a - b) for (_, p0, w0), (_, p1, w1) in zip(rule, rule2)
                        for a, b in zip((*p0, w0), (*p1, w1)))
            assert err < 1e-15, (name, deg, err)
            assert drift < 1e-7, (name, deg, drift)   # the published parameters, not another rule
            P, W = expand(rule2, pts_of)
            out.append(f"/* {name} order {deg}: {len(W)} points, moment residual {err:.1e}, "
                       f"refinement drift {drift:.1e} */")
            out.append(f"static const double k_{name}{deg}[] = {{")
            for p, w in zip(P, W):
                out.append("    " + ", ".join(f"{v:.17g}" for v in (*p, w)) + ",")
            out.append("};")
    print("\n".join(out))


if __name__ == "__main__":
    main()
