"""Pack / unpack C-ABI (elx_pack_* / elx_unpack_*) on host buffers against a
numpy restatement of the reference's portion loops
(include/El/blas_like/level1/Copy/util.hpp: StridedPack/Unpack :667-718,
ColStrided* :359-417, RowStrided* :148-184, PartialColStrided* :460-552,
PartialRowStrided* :186-230; Axpy/util.hpp:23-50 for the axpy unpack).
Bit-exact: these are copies (and one axpy with an exact alpha)."""
import ctypes

import numpy as np
import pytest

from elemental_amd import _lib as L
from elemental_amd import el

CPU = 0


def shift(k, align, stride):  # Shift_ (indexing/impl.hpp:244-245)
    return (k - align) % stride


def length(n, s, stride):  # Length_ (indexing/impl.hpp:33-36)
    return (n - s - 1) // stride + 1 if n > s else 0


def p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def padded(h, w, ld, seed):
    rng = np.random.default_rng(seed)
    buf = np.asfortranarray(rng.standard_normal((ld, max(w, 1))))
    return buf


@pytest.mark.parametrize("h,w,ca,cs,ra,rs", [(13, 7, 0, 1, 0, 3), (13, 7, 2, 4, 0, 1), (11, 9, 1, 2, 2, 4),
                                             (3, 2, 1, 4, 0, 3), (0, 5, 0, 2, 0, 2), (8, 8, 0, 2, 1, 2)])
def test_strided_pack_unpack(h, w, ca, cs, ra, rs):
    ld = h + 3
    A = padded(h, w, ld, 1)
    ps = max(1, -(-h // cs) * -(-w // rs))
    got = np.full(cs * rs * ps, np.nan)
    L.call("elx_pack_strided", CPU, el.F64, h, w, ca, cs, ra, rs, p(A), ld, p(got), ps, None)
    want = np.full(cs * rs * ps, np.nan)
    for l in range(rs):
        rsh = shift(l, ra, rs)
        for k in range(cs):
            csh = shift(k, ca, cs)
            sub = A[csh:h:cs, rsh:w:rs]
            assert sub.shape == (length(h, csh, cs), length(w, rsh, rs))
            q = (k + l * cs) * ps
            want[q:q + sub.size] = sub.ravel(order="F")
    assert np.array_equal(got, want, equal_nan=True)
    # unpack is the inverse on the lattice rows/columns; padding rows untouched
    B = np.asfortranarray(np.full_like(A, -7.0))
    L.call("elx_unpack_strided", CPU, el.F64, h, w, ca, cs, ra, rs, p(got), ps, p(B), ld, None)
    assert np.array_equal(B[:h, :w], A[:h, :w])
    assert np.all(B[h:, :] == -7.0)
    # fused reduce-scatter epilogue: B += alpha * portions
    L.call("elx_unpack_axpy_strided", CPU, el.F64, h, w, -2.0, ca, cs, ra, rs, p(got), ps, p(B), ld, None)
    assert np.array_equal(B[:h, :w], -A[:h, :w])


@pytest.mark.parametrize("cols", [1, 0])
@pytest.mark.parametrize("n,align,su,sp,rank_part", [(19, 0, 2, 2, 1), (23, 3, 4, 2, 0), (9, 1, 2, 4, 3),
                                                     (5, 2, 4, 2, 1)])
def test_partial_strided_pack_unpack(cols, n, align, su, sp, rank_part):
    """PartialCol/RowStridedPack: the local matrix holds the partial lattice
    rank_part (stride sp); portion k = the rows (columns) of full-stride rank
    rank_part + k*sp (stride su*sp)."""
    stride = su * sp
    other = 6
    shift0 = shift(rank_part, align, sp)
    nloc = length(n, shift0, sp)
    if cols:
        h, w, lh, lw = n, other, nloc, other
    else:
        h, w, lh, lw = other, n, other, nloc
    ld = lh + 2
    A = padded(lh, lw, ld, 2)
    ps = max(1, -(-n // stride) * other)
    got = np.full(su * ps, np.nan)
    L.call("elx_pack_partial_strided", CPU, el.F64, cols, h, w, align, stride, su, sp, rank_part, shift0, p(A), ld,
           p(got), ps, None)
    want = np.full(su * ps, np.nan)
    for k in range(su):
        sh = shift(rank_part + k * sp, align, stride)
        off = (sh - shift0) // sp
        ln = length(n, sh, stride)
        sub = A[off::su, :lw][:ln] if cols else A[:lh, off::su][:, :ln]
        assert sub.shape == ((ln, lw) if cols else (lh, ln))
        want[k * ps:k * ps + sub.size] = sub.ravel(order="F")
    assert np.array_equal(got, want, equal_nan=True)
    B = np.asfortranarray(np.full_like(A, -7.0))
    L.call("elx_unpack_partial_strided", CPU, el.F64, cols, h, w, align, stride, su, sp, rank_part, shift0, p(got),
           ps, p(B), ld, None)
    assert np.array_equal(B[:lh, :lw], A[:lh, :lw])


def test_pack_rejects_short_portions():
    A = padded(8, 4, 8, 3)
    out = np.zeros(64)
    with pytest.raises(L.LogicError, match="portion"):
        L.call("elx_pack_strided", CPU, el.F64, 8, 4, 0, 2, 0, 1, p(A), 8, p(out), 15, None)
    with pytest.raises(L.LogicError, match="stride"):
        L.call("elx_pack_partial_strided", CPU, el.F64, 1, 8, 4, 0, 4, 3, 2, 0, 0, p(A), 8, p(out), 16, None)
