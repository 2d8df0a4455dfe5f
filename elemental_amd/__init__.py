"""elemental_amd: MI355X-native El::Gemm path (SUMMA over DistMatrix, gfx950 MFMA kernels, RCCL).

The product is libelemental_amd.so (C-ABI: include/elemental_amd.h); this
package only binds it (``_lib``), mirrors the El:: objects (``el``) and
provides the gloo host-collective bridge used by CPU multi-rank runs
(``torch_bridge``).
"""
__version__ = "0.1.0"
