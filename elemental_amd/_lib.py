"""ctypes binding of libelemental_amd.so (the C-ABI in include/elemental_amd.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C elemental_amd/csrc``).  There is no fallback: if the library is
missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t,
                    c_ubyte, c_uint16, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libelemental_amd.so")

# status codes / enums (mirrors include/elemental_amd.h)
OK, ERR_LOGIC, ERR_HIP, ERR_COMM, ERR_RUNTIME, ERR_UNSUPPORTED, ERR_NO_DEVICE, ERR_SINGULAR = range(8)
NORMAL, TRANSPOSE, ADJOINT = 0, 1, 2
MC, MD, MR, VC, VR, STAR, CIRC = range(7)
(GEMM_DEFAULT, GEMM_SUMMA_A_MS, GEMM_SUMMA_A, GEMM_SUMMA_B_MS, GEMM_SUMMA_B, GEMM_SUMMA_C_MS,
 GEMM_SUMMA_C, GEMM_SUMMA_DOT, GEMM_CANNON) = range(9)
ROW_MAJOR, COLUMN_MAJOR = 0, 1
LOWER, UPPER = 0, 1  # El::UpperOrLower (include/El/core/types.hpp:511-515)
LEFT, RIGHT = 0, 1  # El::LeftOrRight (types.hpp:418-422)
NON_UNIT, UNIT = 0, 1  # El::UnitOrNonUnit (types.hpp:489-493)
CPU, GPU = 0, 1
F32, F64, F16, BF16 = 0, 1, 2, 3
I32, I64, U8 = 4, 5, 6  # communication buffers only (elx_mpi_*, elx_comm_*)
OP_SUM, OP_PROD, OP_MAX, OP_MIN = 0, 1, 2, 3
(MAP_IDENTITY, MAP_NEGATE, MAP_ABS, MAP_SQUARE, MAP_SQRT, MAP_EXP, MAP_LOG, MAP_RELU, MAP_SIGMOID,
 MAP_RECIP, MAP_TANH) = range(11)
(COMBINE_ADD, COMBINE_SUB, COMBINE_MUL, COMBINE_DIV, COMBINE_MAX, COMBINE_MIN, COMBINE_RELU_GRAD) = range(7)
FILE_AUTO, FILE_BINARY, FILE_BINARY_FLAT = 0, 3, 4
COLL_ALLGATHER, COLL_REDUCE_SCATTER, COLL_ALLTOALL, COLL_SENDRECV, COLL_BCAST, COLL_ALLREDUCE, \
    COLL_BARRIER = range(7)

HOST_COLL_FN = CFUNCTYPE(c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_int)
HOST_SPLIT_FN = CFUNCTYPE(c_int, c_void_p, c_int, c_int, c_int, POINTER(c_int), POINTER(c_int), POINTER(c_int))

_vp, _i, _i64, _d = c_void_p, c_int, c_int64, c_double
_SIGS = {
    "elx_last_error": (c_char_p, []),
    "elx_version": (_i, []),
    "elx_device_count": (_i, [POINTER(c_int)]),
    "elx_set_device": (_i, [_i]),
    "elx_get_device": (_i, [POINTER(c_int)]),
    "elx_device_synchronize": (_i, []),
    "elx_default_stream": (_i, [POINTER(c_void_p)]),
    "elx_comm_stream": (_i, [POINTER(c_void_p)]),
    "elx_reserved_cus": (_i, [POINTER(c_int)]),
    "elx_stream_create": (_i, [POINTER(c_void_p)]),
    "elx_stream_destroy": (_i, [_vp]),
    "elx_stream_synchronize": (_i, [_vp]),
    "elx_default_event": (_i, [POINTER(c_void_p)]),
    "elx_event_create": (_i, [POINTER(c_void_p)]),
    "elx_event_destroy": (_i, [_vp]),
    "elx_event_record": (_i, [_vp, _vp]),
    "elx_stream_wait_event": (_i, [_vp, _vp]),
    "elx_event_synchronize": (_i, [_vp]),
    "elx_pool_alloc": (_i, [POINTER(c_void_p), c_size_t, _vp]),
    "elx_pool_free": (_i, [_vp, _vp]),
    "elx_pool_trim": (_i, [c_size_t]),
    "elx_pool_stats": (_i, [POINTER(c_size_t), POINTER(c_size_t)]),
    "elx_pool_set_max_cached": (_i, [c_size_t]),
    "elx_pool_max_cached": (_i, [POINTER(c_size_t)]),
    "elx_pool_bin_bytes": (c_size_t, [c_size_t]),
    "elx_pool_bin_cacheable": (_i, [c_size_t]),
    "elx_pool_backing_reserved": (_i, [POINTER(c_size_t)]),
    "elx_memcpy_h2d": (_i, [_vp, _vp, c_size_t, _vp]),
    "elx_memcpy_d2h": (_i, [_vp, _vp, c_size_t, _vp]),
    "elx_memcpy_d2d": (_i, [_vp, _vp, c_size_t, _vp]),
    "elx_gemm_f64": (_i, [_i, _i, _i64, _i64, _i64, _d, _vp, _i64, _vp, _i64, _d, _vp, _i64, _vp]),
    "elx_gemm_f32": (_i, [_i, _i, _i64, _i64, _i64, c_float, _vp, _i64, _vp, _i64, c_float, _vp, _i64, _vp]),
    "elx_gemm_f16": (_i, [_i, _i, _i64, _i64, _i64, c_float, _vp, _i64, _vp, _i64, c_float, _vp, _i64, _vp]),
    "elx_gemm_bf16": (_i, [_i, _i, _i64, _i64, _i64, c_float, _vp, _i64, _vp, _i64, c_float, _vp, _i64, _vp]),
    "elx_matrix_gemm": (_i, [_i, _i, _i, _i, _i64, _i64, _i64, _d, _vp, _i64, _vp, _i64, _d, _vp, _i64, _vp]),
    "elx_matrix_fill": (_i, [_i, _i, _i64, _i64, _d, _vp, _i64, _vp]),
    "elx_matrix_scale": (_i, [_i, _i, _i64, _i64, _d, _vp, _i64, _vp]),
    "elx_matrix_axpy": (_i, [_i, _i, _i64, _i64, _d, _vp, _i64, _vp, _i64, _vp]),
    "elx_matrix_copy": (_i, [_i, _i, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_axpy2d": (_i, [_i, _i64, _i64, _d, _vp, _i64, _i64, _vp, _i64, _i64, _vp]),
    "elx_copy2d": (_i, [_i, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp]),
    "elx_pack_strided": (_i, [_i, _i, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_unpack_strided": (_i, [_i, _i, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_pack_partial_strided": (_i, [_i, _i, _i, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp,
                                      _i64, _vp]),
    "elx_unpack_partial_strided": (_i, [_i, _i, _i, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64,
                                        _vp, _i64, _vp]),
    "elx_unpack_axpy_strided": (_i, [_i, _i, _i64, _i64, _d, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_copy2d_convert": (_i, [_i, _i, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp]),
    "elx_transpose": (_i, [_i, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_scale2d": (_i, [_i, _i64, _i64, _d, _vp, _i64, _vp]),
    "elx_fill2d": (_i, [_i, _i64, _i64, _d, _vp, _i64, _vp]),
    "elx_hadamard2d": (_i, [_i, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_entrywise_map": (_i, [_i, _i, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_combine": (_i, [_i, _i, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "elx_fill_hash": (_i, [_i, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64, c_uint64, _d, _d, _vp]),
    "elx_comm_unique_id": (_i, [POINTER(c_ubyte)]),
    "elx_comm_init_rccl": (_i, [POINTER(c_void_p), _i, _i, POINTER(c_ubyte)]),
    "elx_comm_init_host": (_i, [POINTER(c_void_p), _i, _i, HOST_COLL_FN, HOST_SPLIT_FN, _vp]),
    "elx_comm_wrap_rccl": (_i, [POINTER(c_void_p), _vp]),
    "elx_comm_rank": (_i, [_vp, POINTER(c_int)]),
    "elx_comm_size": (_i, [_vp, POINTER(c_int)]),
    "elx_comm_destroy": (_i, [_vp]),
    "elx_comm_world": (_i, [POINTER(c_void_p)]),
    "elx_comm_set_world": (_i, [_vp]),
    "elx_rendezvous_bcast": (_i, [_vp, c_size_t, _i, _i, c_char_p, _i, _d]),
    "elx_watchdog_stage": (_i, [c_char_p, _d]),
    "elx_watchdog_epitaph": (_i, [c_char_p, _i]),
    "elx_comm_allgather": (_i, [_vp, _i, _vp, _vp, _i64, _vp]),
    "elx_comm_reduce_scatter": (_i, [_vp, _i, _vp, _vp, _i64, _vp]),
    "elx_comm_barrier": (_i, [_vp]),
    "elx_comm_split": (_i, [_vp, _i, _i, POINTER(c_void_p)]),
    "elx_comm_allreduce": (_i, [_vp, _i, _vp, _vp, _i64, _vp]),
    "elx_comm_bcast": (_i, [_vp, _i, _vp, _i64, _i, _vp]),
    "elx_comm_alltoall": (_i, [_vp, _i, _vp, _vp, _i64, _vp]),
    "elx_comm_sendrecv": (_i, [_vp, _i, _vp, _i, _vp, _i, _i64, _vp]),
    "elx_mpi_allgather": (_i, [_vp, _i, _i, _vp, _vp, c_int64, _vp]),
    "elx_mpi_reduce_scatter": (_i, [_vp, _i, _i, _i, _vp, _vp, c_int64, _vp]),
    "elx_mpi_allreduce": (_i, [_vp, _i, _i, _i, _vp, _vp, c_int64, _vp]),
    "elx_mpi_alltoall": (_i, [_vp, _i, _i, _vp, _vp, c_int64, _vp]),
    "elx_mpi_bcast": (_i, [_vp, _i, _i, _vp, c_int64, _i, _vp]),
    "elx_mpi_sendrecv": (_i, [_vp, _i, _i, _vp, c_int64, _i, _vp, c_int64, _i, _vp]),
    "elx_comm_stats": (_i, [POINTER(c_int64), POINTER(c_double), POINTER(c_int64)]),
    "elx_comm_stats_reset": (_i, []),
    "elx_grid_default_height": (_i, [_i]),
    "elx_grid_create": (_i, [POINTER(c_void_p), _vp, _i, _i]),
    "elx_grid_info": (_i, [_vp, POINTER(c_int)]),
    "elx_grid_destroy": (_i, [_vp]),
    "elx_dm_create": (_i, [POINTER(c_void_p), _vp, _i, _i, _i, _i, _i]),
    "elx_dm_destroy": (_i, [_vp]),
    "elx_dm_align": (_i, [_vp, _i, _i, _i]),
    "elx_dm_align_with": (_i, [_vp, _vp, _i]),
    "elx_dm_resize": (_i, [_vp, _i64, _i64]),
    "elx_dm_info": (_i, [_vp, POINTER(c_int64)]),
    "elx_dm_buffer": (_i, [_vp, POINTER(c_void_p)]),
    "elx_dm_set_local": (_i, [_vp, _vp, _i64]),
    "elx_dm_get_local": (_i, [_vp, _vp, _i64]),
    "elx_dm_frobenius_norm": (_i, [_vp, POINTER(c_double)]),
    "elx_dm_view": (_i, [POINTER(c_void_p), _vp, _i64, _i64, _i64, _i64]),
    "elx_dm_attach": (_i, [_vp, _i64, _i64, _i, _i, _vp, _i64, _i]),
    "elx_dm_copy": (_i, [_vp, _vp]),
    "elx_dm_transpose": (_i, [_vp, _vp]),
    "elx_dm_fill_hash": (_i, [_vp, c_uint64, _d, _d]),
    "elx_initialize_random": (_i, [_i, _i]),
    "elx_dm_uniform": (_i, [_vp, _i64, _i64, _d, _d]),
    "elx_dm_make_uniform": (_i, [_vp, _d, _d]),
    "elx_dm_synchronize": (_i, [_vp]),
    "elx_dm_set_stream": (_i, [_vp, _vp]),
    "elx_dm_stream": (_i, [_vp, POINTER(c_void_p)]),
    "elx_dm_write": (_i, [_vp, c_char_p, _i, _i]),
    "elx_dm_read": (_i, [_vp, c_char_p, _i, _i]),
    "elx_dm_get": (_i, [_vp, _i64, _i64, POINTER(c_double)]),
    "elx_dm_set": (_i, [_vp, _i64, _i64, _d]),
    "elx_dm_update": (_i, [_vp, _i64, _i64, _d]),
    "elx_dm_fill": (_i, [_vp, _d]),
    "elx_dm_axpy": (_i, [_d, _vp, _vp]),
    "elx_dm_scale": (_i, [_d, _vp]),
    "elx_dm_zero": (_i, [_vp]),
    "elx_dm_hadamard": (_i, [_vp, _vp, _vp]),
    "elx_dm_entrywise_map": (_i, [_i, _vp, _vp]),
    "elx_dm_combine": (_i, [_i, _vp, _vp]),
    "elx_dm_axpy_contract": (_i, [_d, _vp, _vp]),
    "elx_gemm": (_i, [_i, _i, _d, _vp, _vp, _d, _vp, _i]),
    "elx_local_gemm": (_i, [_i, _i, _d, _vp, _vp, _d, _vp]),
    "elx_syrk": (_i, [_i, _i, _d, _vp, _d, _vp, _i]),
    "elx_trrk": (_i, [_i, _i, _i, _d, _vp, _vp, _d, _vp]),
    "elx_syr2k": (_i, [_i, _i, _d, _vp, _vp, _d, _vp, _i]),
    "elx_trsm": (_i, [_i, _i, _i, _i, _d, _vp, _vp, _i]),
    "elx_symm": (_i, [_i, _i, _d, _vp, _vp, _d, _vp, _i]),
    "elx_dm_scale_trapezoid": (_i, [_d, _i, _vp, _i64]),
    "elx_set_blocksize": (_i, [_i64]),
    "elx_blocksize": (_i64, []),
    "elx_push_blocksize": (_i, [_i64]),
    "elx_pop_blocksize": (_i, []),
    "elx_empty_blocksize_stack": (_i, []),
    "elx_initialize": (_i, []),
    "elx_finalize": (_i, []),
    "elx_set_compute_panel": (_i, [_i64]),
    "elx_last_gemm_algorithm": (_i, []),
    "elx_set_stream_pool_size": (_i, [_i]),
    "elx_stream_pool_size": (_i, []),
    "elx_set_profiling": (_i, [_i]),
    "elx_profile_stats": (_i, [POINTER(c_double), POINTER(c_int64), POINTER(c_double), POINTER(c_double),
                               POINTER(c_int64)]),
    "elx_profile_transfers": (_i, [POINTER(c_double), POINTER(c_int64), POINTER(c_int64)]),
    "elx_profile_pipeline": (_i, [POINTER(c_double), POINTER(c_int64)]),
}


class ElxError(RuntimeError):
    """Raised for a nonzero ELX_ERR_* status; `code` holds the status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[elx error {code}] {msg}")
        self.code = code


class LogicError(ElxError):
    pass


class UnsupportedError(LogicError):
    pass


class NoDeviceError(ElxError):
    pass


class SingularMatrixError(ElxError):
    """El::SingularMatrixException (include/El/core/environment/decl.hpp:209-214)."""


_EXC = {ERR_LOGIC: LogicError, ERR_UNSUPPORTED: UnsupportedError, ERR_NO_DEVICE: NoDeviceError,
        ERR_SINGULAR: SingularMatrixError}

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "(there is no fallback implementation)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != OK:
        msg = lib().elx_last_error().decode(errors="replace")
        raise _EXC.get(rc, ElxError)(rc, msg)


def call(name: str, *args):
    """Call an int-returning entry point and raise on failure."""
    check(getattr(lib(), name)(*args))


def declared_symbols(header: str | None = None) -> list[str]:
    """Names of every function declared in include/elemental_amd.h."""
    import re
    header = header or os.path.join(os.path.dirname(_HERE), "include", "elemental_amd.h")
    text = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\s*\*|int64_t|size_t|int)\s+(elx_\w+)\s*\(", text, re.M)))
