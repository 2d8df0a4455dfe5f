"""Derived PMC metrics shared by tools/summarize_profiles.py and tools/pmc_compare.py.

Round 4 repair of the "MFMA busy" figure: rounds 1-3 divided
SQ_VALU_MFMA_BUSY_CYCLES by GRBM_GUI_ACTIVE, but that counter read an exact
power of two in every profile (2^41 for every fp64 launch, 2^36 for every C5
launch, 2^33 for two different kernels), so the quotient only scaled the
inverse kernel time.  The MFMA utilisation is now derived from the MOPS
counters, which tools/mfma_calib.hip / tools/pmc_calib.sh calibrate against
kernels of known MFMA count (SQ_INSTS_VALU_MFMA_MOPS_* = FLOPs / 512):

  mfma_util = MOPS * 512 / (FLOP per cycle per CU * 256 CUs * cycles)

with cycles = GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
and FLOP per cycle per CU = dense peak / (256 CUs x 2.4 GHz): f64 128, f32 256,
bf16 / f16 4096 (v_mfma_f64_16x16x4_f64 = 2048 FLOP in 64 cycles per SIMD,
v_mfma_f32_16x16x32_bf16 = 16384 FLOP in 16, MI355X_MICROARCH.md).  That is
the fraction of the MFMA pipes' cycles spent on useful MFMAs at the clock the
kernel actually ran at; `effective_clock_ghz` carries the clock part of the
gap to the 2.4 GHz peak.
"""
FLOP_PER_CYCLE_CU = {"f64": 128.0, "f32": 256.0, "bf16": 4096.0, "f16": 4096.0}
MOPS_COUNTER = {"f64": "SQ_INSTS_VALU_MFMA_MOPS_F64", "f32": "SQ_INSTS_VALU_MFMA_MOPS_F32",
                "bf16": "SQ_INSTS_VALU_MFMA_MOPS_BF16", "f16": "SQ_INSTS_VALU_MFMA_MOPS_F16"}
NCU = 256


def pegged(v: float) -> bool:
    """An exact power of two of at least 2^30: the saturated / stuck reading
    rounds 1-3 took for MFMA busy cycles."""
    iv = int(v)
    return v == iv and iv >= (1 << 30) and (iv & (iv - 1)) == 0


def derive(c: dict, avg_s: float | None, dtype: str, flops: float | None = None) -> dict:
    """Metrics from per-launch counter means `c` (summed over XCDs / SEs)."""
    out = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if cyc > 0 and avg_s:
        out["effective_clock_ghz"] = cyc / avg_s / 1e9
    mops = c.get(MOPS_COUNTER.get(dtype, ""))
    if mops is not None:
        out["mfma_flops_counted"] = mops * 512.0
        if flops:
            out["mops_vs_algorithmic_flops"] = mops * 512.0 / flops
        if cyc > 0:
            out["mfma_util"] = mops * 512.0 / (FLOP_PER_CYCLE_CU[dtype] * NCU * cyc)
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if busy is not None:
        out["mfma_busy_cycles_raw"] = busy
        out["mfma_busy_cycles_pegged"] = pegged(busy)
    if "FETCH_SIZE" in c:
        out["fabric_read_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024.0  # gfx950: FETCH_SIZE counts half of wide reads
    if "WRITE_SIZE" in c:
        out["fabric_write_bytes"] = c["WRITE_SIZE"] * 1024.0
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    return out
