#!/usr/bin/env python3
"""Golden GEMM fixtures from the reference CPU path's own BLAS: Intel MKL.

The reference's CPU El::Gemm ends in `blas::Gemm` -> `dgemm_` / `sgemm_`
(src/core/imports/blas/Gemm.hpp:395-452, called from Gemm_impl<CPU> at
src/blas_like/level3/Gemm.cpp:141-161), linked against MKL in the reference's
documented build (conda `mkl 2021.4.0`, MKL_THREADING_LAYER
GNU or SEQUENTIAL).  That MKL is present in this container
(/opt/conda/lib/libmkl_rt.so, "oneAPI MKL 2021.4 Product Build 20210904"), so
the floating-point results of the reference's CPU path can be produced here at
its exact call sites without building or running any reference code:

  mkl_local.npz  C := alpha op(A) op(B) + beta C for f64 and f32, all four
                 orientations, odd shapes: ONE dgemm_/sgemm_ call each, as
                 Gemm_impl<CPU> issues it (LocalGemm on a 1x1 grid).
  mkl_summa.npz  El::Gemm(NORMAL, NORMAL, alpha, A, B, beta, C, GEMM_SUMMA_C)
                 on r x c grids as the reference computes it rank by rank:
                 Scale(beta, C) (Gemm.cpp:282: one multiplication per local
                 entry), then for every Blocksize() panel (NN.hpp:370-384)
                 A1[MC,*] = A(:, k:k+nb), B1Trans[MR,*] = B(k:k+nb, :)^T and
                 LocalGemm(NORMAL, TRANSPOSE, alpha, A1[MC,*], B1Trans[MR,*],
                 1, C) = dgemm_('N','T', mloc, nloc, nb, alpha, A1, mloc,
                 B1T, nloc, 1, Cloc, mloc) on every rank's local block.

  mkl_summa_orient.npz
                 the other orientations and the Dot variant, rank by rank:
                 SUMMA_C for NT / TN / TT (NT.hpp:251-294: dgemm_('N','N') of
                 A1[MC,*] and B1Trans[*,MR]; TN.hpp:252-291: dgemm_('T','T') of
                 A1[*,MC] and B1Trans[MR,*]; TT.hpp:195-240: dgemm_('T','N') of
                 A1[*,MC] and B1Trans[*,MR]) and SUMMA_Dot for TN / NN
                 (TN.hpp:371-416, NN.hpp:461-511: per 2000 x 2000 block of C,
                 every VC rank's dgemm_ over its k-rows into C11[*,*], the
                 contributions summed in rank order, C11 += sum: AxpyContract);
                 plus C1 at its own size (NN f64 4096^3 on 2x2, nb = 128) stored
                 as a sample: rows 0::37 x columns 0::41 of the result.

Inputs are oracle.hash_matrix(seed) draws in [-0.1, 0.1) (Gemm_Suite.cpp:158-172
values, alpha = 0.5, beta = -0.5); only their seeds are stored.  MKL runs with
MKL_THREADING_LAYER=SEQUENTIAL and MKL_CBWR=COMPATIBLE (bit-reproducible on any
x86 host).  Re-run:  python tools/make_mkl_golden.py  (writes tests/golden/).
This script is test infrastructure: nothing on the GPU box loads MKL.
"""
from __future__ import annotations

import ctypes as c
import os
import sys

os.environ["MKL_THREADING_LAYER"] = "SEQUENTIAL"
os.environ["MKL_CBWR"] = "COMPATIBLE"
import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

MKL_PATH = "/opt/conda/lib/libmkl_rt.so"
OUT = os.path.join(ROOT, "tests", "golden")
ALPHA, BETA = 0.5, -0.5
LOCAL_SHAPES = [(67, 53, 41), (128, 96, 200), (33, 70, 301), (1, 17, 5)]
# (r, c, nb, m, n, k): the 2x2 grid of C1, C3's 2x4, and 1x2, with ragged panels
SUMMA_CASES = [(2, 2, 16, 45, 37, 61), (1, 2, 8, 30, 41, 27), (2, 4, 16, 53, 66, 130), (2, 2, 128, 260, 200, 300)]


def mkl():
    lib = c.CDLL(MKL_PATH)
    buf = c.create_string_buffer(256)
    lib.mkl_get_version_string(buf, 256)
    return lib, buf.value.decode().strip()


def _i(x):
    return c.byref(c.c_int(int(x)))


def gemm(lib, dt, ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc):
    """One dgemm_/sgemm_ call (Fortran interface, column-major, in place on C)."""
    s = c.c_double if dt == np.float64 else c.c_float
    f = lib.dgemm_ if dt == np.float64 else lib.sgemm_
    p = lambda a: a.ctypes.data_as(c.c_void_p)
    f(c.c_char_p(ta.encode()), c.c_char_p(tb.encode()), _i(m), _i(n), _i(k), c.byref(s(alpha)), p(A), _i(lda),
      p(B), _i(ldb), c.byref(s(beta)), p(C), _i(ldc))


def local_cases(lib):
    out = {}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        for (m, n, k) in LOCAL_SHAPES:
            for ta in "NT":
                for tb in "NT":
                    seed = 100 + 7 * len(out)
                    A = np.asfortranarray(oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, seed, 0.0, 0.1, dt))
                    B = np.asfortranarray(oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, seed + 1, 0.0, 0.1, dt))
                    C = np.asfortranarray(oracle.hash_matrix(m, n, seed + 2, 0.0, 0.1, dt))
                    gemm(lib, dt, ta, tb, m, n, k, ALPHA, A, A.shape[0], B, B.shape[0], BETA, C, m)
                    key = f"{tag}_{ta}{tb}_{m}x{n}x{k}"
                    out[key] = C
                    out[key + "_seed"] = np.array([seed, seed + 1, seed + 2])
    return out


def summa_nnc(lib, dt, r, c_, nb, A, B, C):
    """The reference's SUMMA_NNC on an r x c grid (NN.hpp:341-385), rank by
    rank, every local update one MKL call; returns the assembled global C."""
    m, k = A.shape
    n = B.shape[1]
    MC, MR = 0, 2  # oracle's distribution ids: local_block(G, U, V, r, c, vc)
    G = np.array(C, dtype=dt, order="F")
    for vc in range(r * c_):
        mc, mr = vc % r, vc // r
        rows = np.arange(mc, m, r)          # [MC,*] / [MC,MR] local rows (alignment 0)
        cols = np.arange(mr, n, c_)         # [*,MR] / [MR,*] local columns
        Cl = np.asfortranarray(G[np.ix_(rows, cols)] * dt(BETA))  # Scale(beta, C): one rounding per entry
        for k0 in range(0, k, nb):
            kb = min(nb, k - k0)
            A1 = np.asfortranarray(A[np.ix_(rows, np.arange(k0, k0 + kb))])        # A1[MC,*]
            B1T = np.asfortranarray(B[np.ix_(np.arange(k0, k0 + kb), cols)].T)     # B1Trans[MR,*]
            if len(rows) and len(cols):
                gemm(lib, dt, "N", "T", len(rows), len(cols), kb, ALPHA, A1, max(1, len(rows)), B1T,
                     max(1, len(cols)), 1.0, Cl, max(1, len(rows)))
        G[np.ix_(rows, cols)] = Cl
    return G


def summa_cases(lib):
    out = {}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        for i, (r, c_, nb, m, n, k) in enumerate(SUMMA_CASES):
            seed = 500 + 10 * i
            A = oracle.hash_matrix(m, k, seed, 0.0, 0.1, dt)
            B = oracle.hash_matrix(k, n, seed + 1, 0.0, 0.1, dt)
            C = oracle.hash_matrix(m, n, seed + 2, 0.0, 0.1, dt)
            key = f"{tag}_{r}x{c_}_nb{nb}_{m}x{n}x{k}"
            out[key] = summa_nnc(lib, dt, r, c_, nb, A, B, C)
            out[key + "_seed"] = np.array([seed, seed + 1, seed + 2])
    return out


ORIENT_CASES = [(2, 2, 16, 45, 37, 61), (2, 4, 16, 53, 66, 130)]
DOT_CASES = [(2, 2, 20, 24, 130), (2, 4, 19, 30, 257)]
C1_SAMPLE = (37, 41)  # row and column strides of the stored sample of C1's result


def summa_c(lib, dt, oa, ob, r, c_, nb, A, B, C):
    """SUMMA_C for any orientation pair, rank by rank, as the reference's
    SUMMA_{NN,NT,TN,TT}C_impl issue their local updates (one MKL call per
    Blocksize() panel, flags as LocalGemm passes them)."""
    opA = A if oa == "N" else A.T
    opB = B if ob == "N" else B.T
    m, k = opA.shape
    n = opB.shape[1]
    G = np.array(C, dtype=dt, order="F")
    for vc in range(r * c_):
        mc, mr = vc % r, vc // r
        rows, cols = np.arange(mc, m, r), np.arange(mr, n, c_)
        Cl = np.asfortranarray(G[np.ix_(rows, cols)] * dt(BETA))
        for k0 in range(0, k, nb):
            kb = min(nb, k - k0)
            ks = np.arange(k0, k0 + kb)
            if not (len(rows) and len(cols)):
                continue
            # A1 as the reference holds it: [MC,*] (N, mloc x kb) or [*,MC] (T, kb x mloc)
            A1 = np.asfortranarray(opA[np.ix_(rows, ks)] if oa == "N" else opA[np.ix_(rows, ks)].T)
            # B1 as the reference holds it: B1Trans[MR,*] (NN, TN: nloc x kb) or [*,MR] (NT, TT: kb x nloc)
            bt = "T" if ob == "N" else "N"
            B1 = np.asfortranarray(opB[np.ix_(ks, cols)].T if bt == "T" else opB[np.ix_(ks, cols)])
            if oa == "N" and ob == "N":
                fa, fb = "N", "T"
            elif oa == "N":
                fa, fb = "N", "N"
            elif ob == "N":
                fa, fb = "T", "T"
            else:
                fa, fb = "T", "N"
            gemm(lib, dt, fa, fb, len(rows), len(cols), kb, ALPHA, A1, A1.shape[0], B1, B1.shape[0], 1.0, Cl,
                 len(rows))
        G[np.ix_(rows, cols)] = Cl
    return G


def summa_dot(lib, dt, oa, r, c_, A, B, C, block=2000):
    """SUMMA_Dot (TN.hpp:371-416 / NN.hpp:461-511): op(A) and B with k over the VC
    ranks (vc = kk mod p), per block of C every rank's local product
    (dgemm_ beta = 0), summed over the ranks in rank order, added to C11."""
    opA = A if oa == "N" else A.T
    m, k = opA.shape
    n = B.shape[1]
    p = r * c_
    G = np.array(C, dtype=dt, order="F") * dt(BETA)
    for i0 in range(0, m, block):
        i1 = min(m, i0 + block)
        for j0 in range(0, n, block):
            j1 = min(n, j0 + block)
            total = None
            for vc in range(p):
                ks = np.arange(vc, k, p)
                P = np.zeros((i1 - i0, j1 - j0), dtype=dt, order="F")
                if len(ks):
                    # the rank's [VC,*] / [*,VC] local slices as the reference stores them
                    A1 = np.asfortranarray(A[np.ix_(ks, np.arange(i0, i1))] if oa == "T"
                                           else A[np.ix_(np.arange(i0, i1), ks)])
                    B1 = np.asfortranarray(B[np.ix_(ks, np.arange(j0, j1))])
                    gemm(lib, dt, oa, "N", i1 - i0, j1 - j0, len(ks), ALPHA, A1, A1.shape[0], B1, B1.shape[0], 0.0,
                         P, i1 - i0)
                total = P if total is None else total + P
            G[i0:i1, j0:j1] += total
    return G


def orient_cases(lib):
    out = {}
    for dt, tag in ((np.float64, "f64"), (np.float32, "f32")):
        for i, (r, c_, nb, m, n, k) in enumerate(ORIENT_CASES):
            for oa, ob in (("N", "T"), ("T", "N"), ("T", "T")):
                seed = 700 + 10 * len(out)
                A = oracle.hash_matrix(m if oa == "N" else k, k if oa == "N" else m, seed, 0.0, 0.1, dt)
                B = oracle.hash_matrix(k if ob == "N" else n, n if ob == "N" else k, seed + 1, 0.0, 0.1, dt)
                C = oracle.hash_matrix(m, n, seed + 2, 0.0, 0.1, dt)
                key = f"{tag}_{r}x{c_}_nb{nb}_{m}x{n}x{k}_{oa}{ob}_C"
                out[key] = summa_c(lib, dt, oa, ob, r, c_, nb, A, B, C)
                out[key + "_seed"] = np.array([seed, seed + 1, seed + 2])
        for (r, c_, m, n, k) in DOT_CASES:
            for oa in ("T", "N"):
                seed = 700 + 10 * len(out)
                A = oracle.hash_matrix(m if oa == "N" else k, k if oa == "N" else m, seed, 0.0, 0.1, dt)
                B = oracle.hash_matrix(k, n, seed + 1, 0.0, 0.1, dt)
                C = oracle.hash_matrix(m, n, seed + 2, 0.0, 0.1, dt)
                key = f"{tag}_{r}x{c_}_nb16_{m}x{n}x{k}_{oa}N_DOT"
                out[key] = summa_dot(lib, dt, oa, r, c_, A, B, C)
                out[key + "_seed"] = np.array([seed, seed + 1, seed + 2])
    # C1 (BASELINE.json configs[0]) at its own size, sampled
    n1, seed = 4096, 900
    A = oracle.hash_matrix(n1, n1, seed, 0.0, 0.1)
    B = oracle.hash_matrix(n1, n1, seed + 1, 0.0, 0.1)
    C = oracle.hash_matrix(n1, n1, seed + 2, 0.0, 0.1)
    G = summa_nnc(lib, np.float64, 2, 2, 128, A, B, C)
    key = f"f64_2x2_nb128_{n1}x{n1}x{n1}_NN_C_sample"
    out[key] = np.ascontiguousarray(G[::C1_SAMPLE[0], ::C1_SAMPLE[1]])
    out[key + "_seed"] = np.array([seed, seed + 1, seed + 2])
    out[key + "_stride"] = np.array(C1_SAMPLE)
    return out


def main():
    lib, version = mkl()
    os.makedirs(OUT, exist_ok=True)
    meta = np.array([version, "MKL_THREADING_LAYER=SEQUENTIAL MKL_CBWR=COMPATIBLE", f"alpha={ALPHA} beta={BETA}"])
    np.savez_compressed(os.path.join(OUT, "mkl_local.npz"), _mkl=meta, **local_cases(lib))
    np.savez_compressed(os.path.join(OUT, "mkl_summa.npz"), _mkl=meta, **summa_cases(lib))
    np.savez_compressed(os.path.join(OUT, "mkl_summa_orient.npz"), _mkl=meta, **orient_cases(lib))
    print(version)


if __name__ == "__main__":
    main()
