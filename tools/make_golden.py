#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

The reference cannot be run here (its build needs CMake, a configure-time
generated El/config.h, MPI and an external BLAS), and
its own tests hold no golden vectors.  These fixtures are therefore computed
from the reference's *definitions*, in plain Python integer arithmetic, by
code independent of oracle/oracle.c, so that they pin the oracle:

  layout.npz   local block of every rank for every [U,V] pair the path uses,
               grids 1x2, 2x2, 2x4, two alignments, root 0 and last, of a
               13x11 matrix whose entries encode their global index.
               Definitions: Shift/Length (include/El/core/Element/decl.hpp,
               src/core/Element/impl.hpp: Shift = (rank-align) mod stride,
               Length = number of i in [0,n) with i = shift mod stride),
               grid ranks (src/core/Grid.cpp:58-206: column-major VC,
               mc = vc mod r, mr = vc div r, vr = mr + c*mc), [CIRC,CIRC]
               only on root (ElementMatrix/CIRC_CIRC.cpp), [MD,*]/[*,MD]
               only on the root diagonal, stride lcm(r,c) (MD_STAR.cpp).
  hash.npz     hash_unit(seed,i,j) for seeds 1..3 (the synthetic Uniform
               input of SURVEY §8d; splitmix64 as published by Steele/Vigna).
  gemm_exact.npz  small integer-valued GEMMs in all four orientations with
               dyadic alpha/beta whose exact results are representable in
               f64, f32, f16 and bf16: C_out = alpha op(A) op(B) + beta C_in
               evaluated in Python integers (any summation order gives these
               bits), the contract of src/core/imports/blas/Gemm.hpp:47-260.

Run:  python tools/make_golden.py   (writes tests/golden/*.npz, deterministic)
"""
from __future__ import annotations

import os
import random

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")

MC, MD, MR, VC, VR, STAR, CIRC = range(7)
NAMES = {MC: "MC", MD: "MD", MR: "MR", VC: "VC", VR: "VR", STAR: "STAR", CIRC: "CIRC"}
PAIRS = [(MC, MR), (MC, STAR), (STAR, MR), (MR, MC), (MR, STAR), (STAR, MC), (VC, STAR), (STAR, VC),
         (VR, STAR), (STAR, VR), (STAR, STAR), (CIRC, CIRC), (MD, STAR), (STAR, MD)]
M64 = (1 << 64) - 1


def diagonals(r: int, c: int) -> list[list[tuple[int, int]]]:
    """Grid.cpp:105-107,157-185: gcd(r,c) diagonals; diagonal d lists the grid
    coordinates (i mod r, (d + i) mod c), i = 0 .. lcm-1, in MD-rank order."""
    from math import gcd
    g = gcd(r, c)
    lcm = r * c // g
    return [[(i % r, (d + i) % c) for i in range(lcm)] for d in range(g)]


def grid_ranks(vc: int, r: int, c: int) -> dict:
    mc, mr = vc % r, vc // r
    diag = [(d, row.index((mc, mr))) for d, row in enumerate(diagonals(r, c)) if (mc, mr) in row][0]
    return {MC: (mc, r), MR: (mr, c), VC: (vc, r * c), VR: (mr + c * mc, r * c), STAR: (0, 1), CIRC: (0, 1),
            MD: (diag, len(diagonals(r, c)[0]))}


def local_rows(n: int, rank: int, align: int, stride: int) -> list[int]:
    shift = (rank - align) % stride
    return list(range(shift, n, stride))


def local_block(G: np.ndarray, U: int, V: int, r: int, c: int, vc: int, ca: int, ra: int, root: int):
    if U == CIRC:
        return G.copy() if vc == root else np.zeros((0, 0), G.dtype)
    ranks = grid_ranks(vc, r, c)
    if MD in (U, V):  # only the root diagonal holds the matrix (MD_STAR.cpp:166-167)
        (diag, pos), lcm = ranks[MD]
        if diag != root:
            return np.zeros((0, 0), G.dtype)
        ranks[MD] = (pos, lcm)
    cr, cs = ranks[U]
    rr, rs = ranks[V]
    rows = local_rows(G.shape[0], cr, ca, cs)
    cols = local_rows(G.shape[1], rr, ra, rs)
    return G[np.ix_(rows, cols)] if rows and cols else np.zeros((len(rows), len(cols)), G.dtype)


def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def hash_unit(seed: int, i: int, j: int) -> float:
    h = splitmix64(seed ^ splitmix64((i * 0xD1B54A32D192ED03 + 0x1234567) & M64))
    h = splitmix64(h ^ ((j * 0xA0761D6478BD642F) & M64))
    return (h >> 11) * 2.0 ** -53


def make_layout() -> dict:
    H, W = 13, 11
    G = np.array([[i + 1000.0 * j for j in range(W)] for i in range(H)], dtype=np.float64, order="F")
    out = {"G": G}
    for (r, c) in [(1, 2), (2, 2), (2, 4)]:
        p = r * c
        for (U, V) in PAIRS:
            for variant in range(2):
                strides = grid_ranks(0, r, c)
                ca = 0 if variant == 0 else (strides[U][1] - 1 if U != CIRC else 0)
                ra = 0 if variant == 0 else (strides[V][1] // 2 if V != CIRC else 0)
                root = 0 if variant == 0 else (len(diagonals(r, c)) - 1 if MD in (U, V) else p - 1)
                for vc in range(p):
                    key = f"g{r}x{c}_{NAMES[U]}_{NAMES[V]}_a{ca}_{ra}_root{root}_vc{vc}"
                    out[key] = np.asfortranarray(local_block(G, U, V, r, c, vc, ca, ra, root))
    return out


def make_hash() -> dict:
    pts = [(0, 0), (1, 0), (0, 1), (7, 3), (127, 128), (4095, 17), (32767, 32767), (65535, 1), (123456, 654321)]
    ij = np.array(pts, dtype=np.int64)
    out = {"ij": ij}
    for seed in (1, 2, 3, 42):
        out[f"seed{seed}"] = np.array([hash_unit(seed, i, j) for (i, j) in pts], dtype=np.float64)
    return out


def make_gemm_exact() -> dict:
    rng = random.Random(20261015)
    out = {}
    m, n, k = 23, 19, 31
    alpha, beta = 2.0, -0.5
    for ta in "NT":
        for tb in "NT":
            A_ = [[rng.randint(-3, 3) for _ in range(k)] for _ in range(m)]  # op(A): m x k
            B_ = [[rng.randint(-3, 3) for _ in range(n)] for _ in range(k)]  # op(B): k x n
            C_ = [[2 * rng.randint(-8, 8) for _ in range(n)] for _ in range(m)]
            # alpha = 2, beta = -1/2 and C_ even: the result is an exact integer
            Cout = [[2 * sum(A_[i][l] * B_[l][j] for l in range(k)) - C_[i][j] // 2 for j in range(n)]
                    for i in range(m)]
            opA = np.array(A_, dtype=np.float64)
            opB = np.array(B_, dtype=np.float64)
            tag = ta + tb
            out[f"{tag}_A"] = np.asfortranarray(opA if ta == "N" else opA.T)
            out[f"{tag}_B"] = np.asfortranarray(opB if tb == "N" else opB.T)
            out[f"{tag}_C"] = np.asfortranarray(np.array(C_, dtype=np.float64))
            out[f"{tag}_out"] = np.asfortranarray(np.array(Cout, dtype=np.float64))
    out["alpha_beta"] = np.array([alpha, beta])
    # |values| <= 2*9*31 + 8 = 566 < 2^11: exact in f64/f32/f16 and in every
    # intermediate sum; bf16 (8 significant bits) holds the inputs exactly and
    # the output after one rounding of the exact value (tests round it).
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, fn in (("layout", make_layout), ("hash", make_hash), ("gemm_exact", make_gemm_exact)):
        data = fn()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **data)
        print(f"{name}.npz: {len(data)} arrays")


if __name__ == "__main__":
    main()
