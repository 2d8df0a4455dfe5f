"""The C-ABI boundary on CPU: the library loads, exports every symbol the
headers declare, maps errors to the reference's exception types, fails loudly
without a device, and the drop-in C++ header compiles and runs (Device::CPU
matrices, 1x1 grid).  No GPU compute here."""
import os
import re
import shutil
import subprocess

import numpy as np
import oracle
import pytest

from elemental_amd import _lib as L
from elemental_amd import el

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "elemental_amd.h")


def test_every_declared_symbol_is_exported():
    names = L.declared_symbols(HEADER)
    assert len(names) >= 70
    lib = L.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and nm agrees that they are real dynamic exports with C linkage
    if shutil.which("nm"):
        out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
        exported = set(re.findall(r"\sT\s(elx_\w+)$", out, re.M))
        assert set(names) <= exported, sorted(set(names) - exported)


def test_python_signatures_cover_header():
    assert set(L.declared_symbols(HEADER)) == set(L._SIGS), set(L.declared_symbols(HEADER)) ^ set(L._SIGS)


def test_enum_ordinals_match_reference():
    text = open(HEADER).read()
    vals = dict((k, int(v)) for k, v in re.findall(r"#define (ELX_\w+)\s+(\d+)", text))
    # El::Dist (include/El/core/types.hpp), El::Orientation, El::GemmAlgorithm (level3.hpp:22-35)
    assert [vals[f"ELX_{d}"] for d in ("MC", "MD", "MR", "VC", "VR", "STAR", "CIRC")] == list(range(7))
    assert [vals[f"ELX_{o}"] for o in ("NORMAL", "TRANSPOSE", "ADJOINT")] == [0, 1, 2]
    algs = ["DEFAULT", "SUMMA_A_MS", "SUMMA_A", "SUMMA_B_MS", "SUMMA_B", "SUMMA_C_MS", "SUMMA_C", "SUMMA_DOT",
            "CANNON"]
    assert [vals[f"ELX_GEMM_{a}"] for a in algs] == list(range(9))
    assert (el.MC, el.MR, el.STAR, el.CIRC) == (0, 2, 5, 6)


def test_error_mapping_and_messages():
    g = el.Grid()
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=4, width=3)
    B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=4, width=3)
    C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=4, width=3)
    with pytest.raises(L.LogicError, match="onformal|dimension|match"):
        el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, B, 0.0, C)
    with pytest.raises(L.LogicError, match="invalid distribution"):
        L.call("elx_dm_create", L.ctypes.byref(L.ctypes.c_void_p()), g.h, el.F64, el.MD, el.MR, el.CPU, 0)
    with pytest.raises(L.LogicError, match="Invalid root"):  # one diagonal on a 1x1 grid
        L.call("elx_dm_create", L.ctypes.byref(L.ctypes.c_void_p()), g.h, el.F64, el.MD, el.STAR, el.CPU, 1)
    with pytest.raises(L.LogicError, match="Unsupported Gemm option"):  # Cannon is NN only (NT.hpp:526)
        el.Gemm(el.NORMAL, el.TRANSPOSE, 1.0, A, el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=3, width=3),
                0.0, C, alg=el.GEMM_CANNON)


def test_gpu_matrix_without_device_fails_loudly():
    if el.device_count() > 0:
        pytest.skip("a device is visible")
    g = el.Grid()
    with pytest.raises(L.ElxError):
        el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=8, width=8)
    with pytest.raises(L.ElxError):
        L.call("elx_gemm_f64", 0, 0, 1, 1, 1, 1.0, None, 1, None, 1, 0.0, None, 1, None)


def test_pool_bins_and_cap_setting_without_device():
    """The caching allocator's bin rule (powers of two to 1 MiB, then eight bins
    per octave: runtime.hpp's contract) and its cap setting
    (H_CUB_MAX_CACHED_SIZE, cub.cpp:37-43) need no device."""
    lib = L.lib()
    assert [lib.elx_pool_bin_bytes(b) for b in (0, 1, 512, 513, 5000, 1 << 20)] == [512, 512, 512, 1024, 8192, 1 << 20]
    assert lib.elx_pool_bin_bytes((1 << 20) + 1) == (1 << 20) + (128 << 10)
    prev = 0
    for b in [(1 << 20) + 1, (3 << 20) + 7, 100 << 20, (1 << 30) + 1, 5 << 30, 32 << 30, (1 << 35) + 3]:
        bb = lib.elx_pool_bin_bytes(b)
        assert b <= bb <= b * 1.125 and bb % (128 << 10) == 0 and bb > prev
        assert lib.elx_pool_bin_cacheable(b) == 1
        prev = bb
    # requests whose rounding would overflow size_t get no bin (0): Alloc reports
    # out-of-memory instead of handing out a zero-byte block (e.g. El.hpp's
    # SendRecv scratch for a negative int count cast to size_t)
    smax = (1 << 64) - 1
    for b in (smax, smax - 5, (1 << 64) - (1 << 58)):
        assert lib.elx_pool_bin_bytes(b) == 0, b
    assert lib.elx_pool_bin_bytes(1 << 62) == 1 << 62
    assert lib.elx_pool_bin_bytes((1 << 63) + 1) == (1 << 63) + (1 << 59)
    old = L.ctypes.c_size_t()
    L.call("elx_pool_max_cached", L.ctypes.byref(old))
    try:
        L.call("elx_pool_set_max_cached", 123 << 20)
        v = L.ctypes.c_size_t()
        L.call("elx_pool_max_cached", L.ctypes.byref(v))
        assert v.value == 123 << 20
    finally:
        L.call("elx_pool_set_max_cached", old.value)
    r = L.ctypes.c_size_t(7)
    L.call("elx_pool_backing_reserved", L.ctypes.byref(r))
    assert r.value == 0  # no device touched: no backing pool yet


def _cub_bin(b, growth, min_bin, max_bin):
    """hipCUB CachingDeviceAllocator::DeviceAllocate's bin choice (the
    reference's pool, configured by cub.cpp:21-35): above growth^max_bin the
    request is its own (uncached) block; else the smallest growth^k >= bytes,
    at least growth^min_bin.  Blocks here are whole 512-B granules."""
    gran = lambda x: max(512, (x + 511) // 512 * 512)  # noqa: E731
    if max_bin is not None and b > growth ** max_bin:
        return gran(b), 0
    p = growth ** min_bin
    while p < b:
        p *= growth
    return gran(p), 1


@pytest.mark.parametrize("env", [
    {"H_CUB_BIN_GROWTH": "2"},
    {"H_CUB_BIN_GROWTH": "8"},
    {"H_CUB_BIN_GROWTH": "3", "H_CUB_MIN_BIN": "7"},
    {"H_CUB_MIN_BIN": "12"},
    {"H_CUB_MAX_BIN": "20"},
    {"H_CUB_BIN_GROWTH": "4", "H_CUB_MIN_BIN": "3", "H_CUB_MAX_BIN": "12"},
])
def test_pool_cub_bin_knobs(env):
    """H_CUB_BIN_GROWTH / H_CUB_MIN_BIN / H_CUB_MAX_BIN (cub.cpp:21-35) switch
    the bins to CUB's geometric ones; sizes above the max bin are own-size,
    uncached blocks.  Read once per process, so each setting runs in its own."""
    import json
    import os
    import subprocess
    import sys
    sizes = [0, 1, 100, 511, 512, 513, 4096, 5000, 65537, 1 << 20, (1 << 20) + 1, 3 << 20, 123456789, 5 << 30,
             (1 << 64) - 1]
    code = ("import json,sys; sys.path.insert(0, %r); from elemental_amd import _lib as L; lib = L.lib(); "
            "print(json.dumps([[lib.elx_pool_bin_bytes(b), lib.elx_pool_bin_cacheable(b)] for b in %r]))"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), sizes))
    e = {k: v for k, v in os.environ.items() if not k.startswith("H_CUB_")}
    e.update(env)
    out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout.strip().splitlines()[-1])
    g = int(env.get("H_CUB_BIN_GROWTH", 2))
    mn = int(env.get("H_CUB_MIN_BIN", 1))
    mx = int(env["H_CUB_MAX_BIN"]) if "H_CUB_MAX_BIN" in env else None
    want = [list(_cub_bin(b, g, mn, mx)) for b in sizes]
    # SIZE_MAX: no growth^k holds it, and an own-size block would overflow the
    # 512-B rounding: no bin (0), whichever way it is classified
    want[-1][0] = 0
    assert got == want, list(zip(sizes, got, want))


def test_cpu_matrices_local_gemm_and_redistribution():
    g = el.Grid()
    import oracle
    Ah, Bh, Ch = oracle.hash_matrix(17, 9, 1), oracle.hash_matrix(9, 6, 2), oracle.hash_matrix(17, 6, 3)
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=17, width=9)
    B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=9, width=6)
    C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=17, width=6)
    A.set_local(Ah), B.set_local(Bh), C.set_local(Ch)
    el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
    want = oracle.gemm("N", "N", 0.5, Ah, Bh, -0.5, Ch)
    assert oracle.parity_ratio(C.get_local(), want, Ah, Bh, 9, np.finfo(float).eps) <= 10
    S = el.DistMatrix(g, el.F64, el.STAR, el.VC, el.CPU)
    S.assign(A)
    assert np.array_equal(S.get_local(), Ah)


@pytest.mark.parametrize("dtype", [el.F64, el.F32])
def test_frobenius_norm_scaled(dtype):
    """El::FrobeniusNorm with the reference's scaled sum of squares
    (Frobenius.cpp:37-44): entries whose squares overflow (1e200 in f64, 1e30 in
    f32) or underflow give the right norm; NaN propagates; zero is zero."""
    g = el.Grid()
    big = 1e200 if dtype == el.F64 else 1e30
    npt = np.float64 if dtype == el.F64 else np.float32
    for scale in (1.0, big, 1.0 / big):
        a = (oracle.hash_matrix(13, 7, 5) * scale).astype(npt)
        A = el.DistMatrix(g, dtype, el.MC, el.MR, el.CPU, height=13, width=7)
        A.set_local(a)
        want = scale * np.linalg.norm(oracle.hash_matrix(13, 7, 5))
        got = el.FrobeniusNorm(A)
        assert np.isfinite(got) and abs(got - want) <= 1e-5 * want, (scale, got, want)
    Z = el.DistMatrix(g, dtype, el.MC, el.MR, el.CPU, height=4, width=4)
    el.Zero(Z)
    assert el.FrobeniusNorm(Z) == 0.0
    Z.Set(1, 2, float("nan"))
    assert np.isnan(el.FrobeniusNorm(Z))


def test_cpp_dropin_header_compiles_and_runs(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "test_el_api"
    libdir = os.path.dirname(L.LIB_PATH)
    subprocess.check_call([gxx, "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_el_api.cpp"), "-o", str(exe), "-L", libdir,
                           "-lelemental_amd", f"-Wl,-rpath,{libdir}"])
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    assert "OK" in res.stdout


def test_lds_dma_tile_rule(tmp_path):
    """The fp64 / fp32 LDS-DMA kernels' 128 x 128 vs 64 x 64 tile choice and the
    split-k plan (kernels.hpp prefer_t64, dma_plan) on the shapes the round-4
    measurements set them by: host-only code, compiled against the HIP headers."""
    gxx = shutil.which("g++")
    if gxx is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("no g++ / HIP headers")
    exe = tmp_path / "test_tile_rule"
    subprocess.check_call([gxx, "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I", os.path.join(ROOT, "elemental_amd", "csrc", "kernels"),
                           os.path.join(ROOT, "tests", "cpp", "test_tile_rule.cpp"), "-o", str(exe)])
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stdout + res.stderr


def test_c_header_is_plain_c():
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    # the boundary header must compile as C99 (no C++ types leak into signatures)
    subprocess.check_call([gcc, "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", HEADER])


def test_attach_caller_storage():
    """ElementalMatrix::Attach: the library computes straight into caller memory."""
    import oracle
    g = el.Grid()
    m, n, k = 11, 7, 5
    Ah = oracle.hash_matrix(m, k, 1)
    Bh = oracle.hash_matrix(k, n, 2)
    Cpad = np.asfortranarray(np.full((m + 3, n), 7.0))   # ldim = m + 3, padding rows untouched
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU).attach(m, k, 0, 0, Ah.ctypes.data, m)
    B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU).attach(k, n, 0, 0, Bh.ctypes.data, k)
    C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU).attach(m, n, 0, 0, Cpad.ctypes.data, m + 3)
    assert C.info()["ldim"] == m + 3 and C.info()["viewing"]
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, B, 0.0, C)
    want = oracle.gemm("N", "N", 1.0, Ah, Bh, 0.0, np.zeros((m, n), order="F"))
    assert oracle.parity_ratio(Cpad[:m], want, Ah, Bh, k, np.finfo(float).eps) <= 10
    assert (Cpad[m:] == 7.0).all()
    with pytest.raises(L.LogicError):
        C.Resize(3, 3)
    with pytest.raises(L.LogicError):
        el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU).attach(m, n, 0, 0, Cpad.ctypes.data, m - 1)


@pytest.mark.parametrize("dt,kind", [(el.F64, "f64"), (el.F32, "f32"), (el.F16, "f16"), (el.BF16, "bf16")])
def test_uniform_reproduces_reference_draws(dt, kind):
    """El::InitializeRandom + El::Uniform on a 1x1 grid: the reference's mt19937
    draws in column-major order (oracle.mt_uniform), bit for bit."""
    import oracle
    g = el.Grid()
    el.InitializeRandom(True, 0)
    A = el.DistMatrix(g, dt, el.MC, el.MR, el.CPU)
    el.Uniform(A, 13, 7, 0.5, 0.5)
    want = oracle.mt_uniform((21 << 16) | 0, 13 * 7, 0.0, 1.0, kind).reshape((13, 7), order="F")
    got = A.get_local()
    assert np.array_equal(got.view(np.uint16) if kind in ("f16", "bf16") else got,
                          want.view(np.uint16) if kind == "f16" else want)
    # the generator advances: a second call continues the same stream
    B = el.DistMatrix(g, dt, el.MC, el.MR, el.CPU)
    el.Uniform(B, 3, 2, 0.5, 0.5)
    nxt = oracle.mt_uniform((21 << 16) | 0, 13 * 7 + 6, 0.0, 1.0, kind)[13 * 7:].reshape((3, 2), order="F")
    got = B.get_local()
    assert np.array_equal(got.view(np.uint16) if kind in ("f16", "bf16") else got,
                          nxt.view(np.uint16) if kind == "f16" else nxt)


def test_functor_header_compiles_for_gfx950(tmp_path):
    """include/El/EntrywiseMap.hip.hpp through El.hpp under hipcc (the caller's
    compiler): a device lambda map/combine instantiates and codegens for gfx950."""
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    subprocess.check_call([hipcc, "-std=c++17", "-O1", "--offload-arch=gfx950", "-c", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_entrywise_functor.hip"), "-o",
                           str(tmp_path / "t.o")])


def test_gemm_suite_driver_cpu(tmp_path):
    """tests/cpp/gemm_suite.cpp (built by build()): the reference suite's
    experiment-file format (Gemm_Suite.cpp:274-276,494-540) on Device::CPU
    matrices, warm-up associativity residuals enforced (--check), the results
    file in the suite's format (:617-662)."""
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "gemm_suite")
    if not os.path.exists(exe):
        pytest.skip("gemm_suite not built (run __graft_entry__.build())")
    exp = tmp_path / "exp.txt"
    exp.write_text("# comment\nCPU:Double:N:N:SUMMA_C:37:29:41:8\nCPU:Double:T:N:SUMMA_A:20:25:33:4\n"
                   "CPU:Float:N:T:SUMMA_B:18:40:22:8\nCPU:Double:T:T:SUMMA_DOT:12:13:300:16\n"
                   "CPU:Double:N:N:CANNON:24:24:24:8\nnot an experiment\n")
    res = tmp_path / "res.txt"
    r = subprocess.run([exe, "--f", str(exp), "--o", str(res), "--warmup", "2", "--runs", "3", "--check"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("|| E ||_F / || Y ||_F") == 10
    lines = res.read_text().splitlines()
    assert [ln.split(":")[:9] for ln in lines][0] == ["CPU", "double", "Normal", "Normal", "SUMMA_C", "37", "29",
                                                      "41", "8"]
    assert len(lines) == 5 and all(len(ln.split(":")) == 12 for ln in lines)
    assert lines[2].startswith("CPU:float:Normal:Transpose:SUMMA_B:")


def test_mpi_collectives_reject_negative_counts():
    """Every El::mpi / raw collective entry checks count >= 0 before it sizes a
    buffer or hands the count to RCCL (a negative int64 would become a huge
    size_t there)."""
    c = el.Comm.self_comm()
    buf = np.zeros(8)
    p = buf.ctypes.data
    CPU = L.CPU
    calls = [
        ("elx_mpi_allgather", (c.h, L.F64, CPU, p, p, -1, None)),
        ("elx_mpi_reduce_scatter", (c.h, L.F64, CPU, 0, p, p, -2, None)),
        ("elx_mpi_allreduce", (c.h, L.F64, CPU, 0, p, p, -1, None)),
        ("elx_mpi_alltoall", (c.h, L.F64, CPU, p, p, -3, None)),
        ("elx_mpi_bcast", (c.h, L.F64, CPU, p, -1, 0, None)),
        ("elx_mpi_sendrecv", (c.h, L.F64, CPU, p, -1, 0, p, 1, 0, None)),
        ("elx_mpi_sendrecv", (c.h, L.F64, CPU, p, 1, 0, p, -1, 0, None)),
        ("elx_comm_allgather", (c.h, L.F64, p, p, -1, None)),
        ("elx_comm_allreduce", (c.h, L.F64, p, p, -1, None)),
        ("elx_comm_bcast", (c.h, L.F64, p, -1, 0, None)),
    ]
    for name, args in calls:
        with pytest.raises(L.LogicError, match="negative count"):
            L.call(name, *args)
    assert np.all(buf == 0)
