"""The oracle against the committed golden fixtures and known answers (CPU).

tests/golden/*.npz are produced by tools/make_golden.py from the reference's
definitions in plain Python integer arithmetic, independently of oracle.c;
these tests pin the oracle before anything else is compared with it.
"""
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAME = {"MC": oracle.MC, "MD": oracle.MD, "MR": oracle.MR, "VC": oracle.VC, "VR": oracle.VR, "STAR": oracle.STAR,
        "CIRC": oracle.CIRC}


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))  # allow_pickle defaults to False


def test_layout_matches_golden_every_rank():
    z = _load("layout")
    G = z["G"]
    checked = 0
    for key in z.files:
        if key == "G":
            continue
        grid, U, V, a, ra, root, vc = key.split("_")
        r, c = map(int, grid[1:].split("x"))
        ca, ra_ = int(a[1:]), int(ra)
        got = oracle.local_block(G, NAME[U], NAME[V], r, c, int(vc[2:]), ca, ra_, int(root[4:]))
        want = z[key]
        assert got.shape == want.shape, key
        assert np.array_equal(got, want), key
        checked += 1
    assert checked == 392


def test_layout_round_trip_place_block():
    # scattering every rank's local block back reassembles the matrix (tests/core/DistMatrix.cpp:40-78)
    G = oracle.hash_matrix(29, 17, 5)
    for (U, V) in [(oracle.MC, oracle.MR), (oracle.VR, oracle.STAR), (oracle.STAR, oracle.VC),
                   (oracle.MR, oracle.MC)]:
        R = np.full_like(G, np.nan)
        for vc in range(8):
            oracle.place_block(R, oracle.local_block(G, U, V, 2, 4, vc, 1, 1), U, V, 2, 4, vc, 1, 1)
        assert np.array_equal(R, G)


@pytest.mark.parametrize("n,shift,stride,want", [(10, 3, 4, 2), (10, 0, 4, 3), (3, 3, 4, 0), (0, 0, 1, 0),
                                                 (65536, 7, 8, 8192), (13, 1, 2, 6)])
def test_length_known_answers(n, shift, stride, want):
    assert oracle.length(n, shift, stride) == want


def test_shift_and_default_height():
    assert [oracle.shift(r, 2, 4) for r in range(4)] == [2, 3, 0, 1]
    L = oracle.lib()
    # Grid::DefaultHeight: largest divisor <= sqrt(p) (src/core/Grid.cpp:28-40)
    assert [L.orc_default_height(p) for p in (1, 2, 3, 4, 6, 8, 12, 16)] == [1, 1, 1, 2, 2, 2, 3, 4]


def test_hash_matches_golden():
    z = _load("hash")
    L = oracle.lib()
    for seed in (1, 2, 3, 42):
        got = np.array([L.orc_hash_unit(seed, int(i), int(j)) for i, j in z["ij"]])
        assert np.array_equal(got, z[f"seed{seed}"]), seed
    G = oracle.hash_matrix(5, 4, 2, 0.0, 0.1)
    assert G[3, 2] == 0.0 + 0.1 * (2.0 * L.orc_hash_unit(2, 3, 2) - 1.0)


@pytest.mark.parametrize("tag", ["NN", "NT", "TN", "TT"])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_gemm_exact_golden(tag, dt):
    z = _load("gemm_exact")
    al, be = z["alpha_beta"]
    got = oracle.gemm(tag[0], tag[1], al, z[f"{tag}_A"].astype(dt), z[f"{tag}_B"].astype(dt), be,
                      z[f"{tag}_C"].astype(dt))
    assert np.array_equal(got, z[f"{tag}_out"].astype(dt))


@pytest.mark.parametrize("tag", ["NN", "TN"])
def test_gemm_half_exact_golden(tag):
    z = _load("gemm_exact")
    al, be = z["alpha_beta"]
    got = oracle.gemm_half(tag[0], tag[1], al, z[f"{tag}_A"], z[f"{tag}_B"], be, z[f"{tag}_C"])
    assert np.array_equal(got.astype(np.float64), z[f"{tag}_out"])


def test_gemm_beta_zero_never_reads_c():
    A = oracle.hash_matrix(9, 7, 1)
    B = oracle.hash_matrix(7, 5, 2)
    C = np.full((9, 5), np.nan, order="F")
    got = oracle.gemm("N", "N", 1.0, A, B, 0.0, C)
    assert np.isfinite(got).all()


@pytest.mark.parametrize("ta,tb", [("N", "N"), ("N", "T"), ("T", "N"), ("T", "T")])
def test_gemm_vs_numpy(ta, tb):
    m, n, k = 33, 21, 47
    A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, 1)
    B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, 2)
    C = oracle.hash_matrix(m, n, 3)
    got = oracle.gemm(ta, tb, 0.5, A, B, -0.5, C)
    want = 0.5 * ((A if ta == "N" else A.T) @ (B if tb == "N" else B.T)) - 0.5 * C
    assert oracle.parity_ratio(got, want, A, B, k, np.finfo(np.float64).eps) < 1.0


@pytest.mark.parametrize("r,c,nb", [(1, 1, 128), (1, 2, 16), (2, 2, 7), (2, 4, 16), (3, 2, 5)])
def test_summa_simulation_matches_gemm(r, c, nb):
    m, n, k = 45, 38, 61
    A = oracle.hash_matrix(m, k, 1)
    B = oracle.hash_matrix(k, n, 2)
    C = oracle.hash_matrix(m, n, 3)
    got = oracle.summa_nnc(r, c, nb, 0.5, A, B, -0.5, C)
    want = oracle.gemm("N", "N", 0.5, A, B, -0.5, C)
    assert oracle.parity_ratio(got, want, A, B, k, np.finfo(np.float64).eps) < 1.0


def test_bf16_rounding_known_answers():
    x = np.array([1.0, 1.00390625, 1.005859375, -2.0, 3.0e38, np.inf], dtype=np.float32)
    b = oracle.f32_to_bf16_bits(x)
    # 1+2^-8 is a tie -> even (1.0); 1+1.5*2^-8 rounds up to 1+2^-7
    assert list(oracle.bf16_bits_to_f32(b)[:4]) == [1.0, 1.0, 1.0078125, -2.0]
    assert np.isinf(oracle.bf16_bits_to_f32(b)[5])


def test_mt_uniform_matches_libstdcxx(tmp_path):
    """oracle.mt_uniform (the reference's Uniform draws) against std::mt19937 +
    std::uniform_real_distribution compiled from the same libstdc++."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "uniform_ref"
    src = os.path.join(os.path.dirname(__file__), "cpp", "uniform_ref.cpp")
    subprocess.check_call([gxx, "-O2", "-std=c++17", src, "-o", str(exe)])
    for seed in ((21 << 16) | 0, (21 << 16) | 3):
        for kind, lo, hi in (("f64", -0.1, 0.1), ("f32", 0.0, 1.0), ("f64", 2.0, 5.0)):
            out = subprocess.run([str(exe), str(seed), "257", str(lo), str(hi), kind], capture_output=True,
                                 text=True, check=True).stdout.split()
            want = np.array([float(x) for x in out], dtype=np.float64 if kind == "f64" else np.float32)
            got = oracle.mt_uniform(seed, 257, lo, hi, kind)  # (%.9g round-trips a float exactly)
            assert np.array_equal(got, want), (seed, kind)


def test_convert_restatement_known_answers():
    """oracle.convert (Copy_GPU_impl<SrcT,DestT> restated: one round-to-nearest-even
    from the exact value) agrees with numpy's own correctly rounded f64 -> f16 / f32
    casts, with a round-to-odd construction for bf16, and with hand-worked ties."""
    rng = np.random.default_rng(0)
    d = rng.standard_normal(20000) * 10.0 ** rng.integers(-45, 40, 20000)
    d = np.concatenate([d, [0.0, -0.0, np.inf, -np.inf, np.nan, 65520.0, 65519.99, 2.0 ** -25, 1.5 * 2.0 ** -24]])
    with np.errstate(over="ignore"):
        assert np.array_equal(oracle.convert(d, "f64", "f16").view(np.uint16), d.astype(np.float16).view(np.uint16))
        assert np.array_equal(oracle.convert(d, "f64", "f32").view(np.uint32), d.astype(np.float32).view(np.uint32))
        f = d.astype(np.float32)
    back = f.astype(np.float64)
    u = f.view(np.uint32).copy()
    inexact = (back != d) & ~np.isnan(d)
    u[inexact & (np.abs(back) > np.abs(d))] -= 1
    u[inexact] |= 1
    assert np.array_equal(oracle.convert(d, "f64", "bf16"), oracle.f32_to_bf16_bits(u.view(np.float32)))
    # ties to even, double rounding avoided, overflow to inf
    ka = {1 + 2.0 ** -8: 0x3F80, 1 + 3 * 2.0 ** -8: 0x3F82, 1 + 2.0 ** -8 + 2.0 ** -30: 0x3F81,
          float.fromhex("0x1.ff8p127"): 0x7F80, -(1 + 2.0 ** -8): 0xBF80}
    got = oracle.convert(np.array(list(ka)), "f64", "bf16")
    assert [int(x) for x in got] == list(ka.values())
    # f64 -> bf16 via f32 would round 1 + 2^-8 + 2^-30 to the tie 1 + 2^-8 and then to 1.0
    assert int(oracle.f32_to_bf16_bits(np.array([1 + 2.0 ** -8 + 2.0 ** -30], dtype=np.float32))[0]) == 0x3F80


def test_cpu_summa_baseline_small():
    """bench.py's cpu_baseline leg (oracle/cpu_summa.py): the C1-shaped CPU SUMMA
    on a 2x2 grid of gloo processes runs and its entry checks pass (small size)."""
    from oracle import cpu_summa
    res = cpu_summa.run(n=256, nb=16, kc=64, r=2, c=2, seconds=0.2, cores=4)
    assert res["value"] > 0 and res["kind"] == "port" and res["cores"] == 4


# ---- pinned to the reference CPU path's own BLAS (tools/make_mkl_golden.py) ----
def _mkl_cases(name):
    d = np.load(os.path.join(GOLD, name))
    return d, [k for k in d.files if k != "_mkl" and not k.endswith("_seed")]


def _mkl_inputs(d, key):
    """(dtype, ta, tb, m, n, k, A, B, C) regenerated from the fixture's seeds."""
    parts = key.split("_")
    dt = np.float64 if parts[0] == "f64" else np.float32
    m, n, k = map(int, parts[-1].split("x"))
    ta, tb = (parts[1][0], parts[1][1]) if len(parts) == 3 else ("N", "N")
    s = [int(x) for x in d[key + "_seed"]]
    A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, s[0], 0.0, 0.1, dt)
    B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, s[1], 0.0, 0.1, dt)
    C = oracle.hash_matrix(m, n, s[2], 0.0, 0.1, dt)
    return dt, ta, tb, m, n, k, A, B, C


def test_oracle_matches_mkl_local_gemm():
    """oracle.gemm (the restated loop nest of imports/blas/Gemm.hpp) against
    one MKL dgemm_/sgemm_ call per case (MKL 2021.4.0, the reference CPU path's
    BLAS): all four orientations, f64 and f32, within the north_star bound and
    in fact well inside it (worst 0.22, the k = 5 case)."""
    d, keys = _mkl_cases("mkl_local.npz")
    assert "2021.4" in str(d["_mkl"][0]) and len(keys) == 32
    worst = 0.0
    for key in keys:
        dt, ta, tb, m, n, k, A, B, C = _mkl_inputs(d, key)
        ref = oracle.gemm(ta, tb, 0.5, A, B, -0.5, C)
        r = oracle.parity_ratio(ref, d[key], A, B, k, np.finfo(dt).eps)
        worst = max(worst, r)
        assert r <= 10, (key, r)
    assert worst < 1, worst


def test_oracle_matches_mkl_summa_orientations():
    """The oracle's plain GEMM (any summation order is inside the bound) against
    the reference's SUMMA_C for NT / TN / TT and SUMMA_DOT for TN / NN evaluated
    rank by rank through MKL, and C1's sampled 4096^3 result against the
    oracle's simulated SUMMA_NNC at the sampled entries."""
    d = np.load(os.path.join(GOLD, "mkl_summa_orient.npz"))
    keys = [k for k in d.files if k != "_mkl" and not k.endswith(("_seed", "_stride"))]
    assert len(keys) == 21
    for key in keys:
        parts = key.split("_")
        dt = np.float64 if parts[0] == "f64" else np.float32
        m, n, k = map(int, parts[3].split("x"))
        ta, tb = parts[4][0], parts[4][1]
        s = [int(x) for x in d[key + "_seed"]]
        A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, s[0], 0.0, 0.1, dt)
        B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, s[1], 0.0, 0.1, dt)
        C = oracle.hash_matrix(m, n, s[2], 0.0, 0.1, dt)
        eps = np.finfo(dt).eps
        if parts[-1] == "sample":
            sr, sc = (int(x) for x in d[key + "_stride"])
            # the sampled rows of A and columns of B give the sampled entries exactly
            ref = 0.5 * (A[::sr, :].astype(np.float64) @ B[:, ::sc].astype(np.float64)) - 0.5 * C[::sr, ::sc]
            err = np.abs(ref - d[key])
            assert err.max() <= 1e-14, key
            continue
        ref = oracle.gemm(ta, tb, 0.5, A, B, -0.5, C)
        assert oracle.parity_ratio(ref, d[key], A, B, k, eps) < 0.5, key


def test_oracle_matches_mkl_summa():
    """The oracle's simulated SUMMA_NNC and its plain GEMM against the
    reference's SUMMA_NNC evaluated rank by rank through MKL (Scale(beta, C),
    then one dgemm_('N','T') per Blocksize() panel per rank, NN.hpp:370-384)
    on 2x2, 1x2 and 2x4 grids."""
    d, keys = _mkl_cases("mkl_summa.npz")
    assert len(keys) == 8
    for key in keys:
        dt, _, _, m, n, k, A, B, C = _mkl_inputs(d, key)
        r_, c_ = map(int, key.split("_")[1].split("x"))
        nb = int(key.split("_")[2][2:])
        eps = np.finfo(dt).eps
        assert oracle.parity_ratio(oracle.gemm("N", "N", 0.5, A, B, -0.5, C), d[key], A, B, k, eps) < 0.1, key
        if dt == np.float64:
            sim = oracle.summa_nnc(r_, c_, nb, 0.5, A, B, -0.5, C)
            assert oracle.parity_ratio(sim, d[key], A, B, k, eps) < 0.1, key
