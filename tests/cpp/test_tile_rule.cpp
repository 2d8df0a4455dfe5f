// Host-side check of the LDS-DMA kernels' tile choice (kernels.hpp prefer_t64)
// and split-k plan (dma_plan) on the shapes the round-4 measurements set them
// by (profiles/r04_t64_rule_ab.log, r04_small_t64_ab.log, r04_t64_waves8_ab.log).
// Built and run by tests/test_capi_cpu.py (no GPU needed).
#include <cstdio>
#include "kernels.hpp"

using elx::kern::i64;

static int bad = 0;

static void expect(bool got, bool want, const char* what, i64 m, i64 n) {
    if (got != want) {
        std::printf("FAIL %s m=%lld n=%lld: got %d want %d\n", what, (long long)m, (long long)n, got, want);
        ++bad;
    }
}

int main() {
    using elx::kern::prefer_t64;
    struct Case { i64 m, n; bool f32, f64; };
    const Case cases[] = {
        {2048, 2048, false, true},   // 256 128-tiles: fp64 takes 64 x 64 (eight waves beat one workgroup per CU)
        {1536, 2048, true, true},    // 192: fewer than the CUs
        {2560, 2560, true, true},    // 400: balance 0.78 vs 0.89
        {3072, 3072, true, true},    // 576: balance 0.56 vs 1.0
        {3584, 3584, true, true},    // 784
        {2048, 4096, false, false},  // 512: a multiple of 256
        {4096, 4096, false, false},  // 1024
        {1024, 1024, true, true},    // 64
        {16384, 16384, false, false},
        {32768, 32768, false, false},
        {8192, 524288 / 64, false, false},
    };
    for (const Case& c : cases) {
        expect(prefer_t64(1, c.m, c.n), c.f32, "fp32 rule", c.m, c.n);
        expect(prefer_t64(1, c.m, c.n, 256), c.f64, "fp64 rule", c.m, c.n);
        expect(prefer_t64(0, c.m, c.n, 256), false, "mode 0", c.m, c.n);
        expect(prefer_t64(2, c.m, c.n), true, "mode 2", c.m, c.n);
    }
    // dma_plan: whole k once the tiles fill two slots per CU; split-k below
    const elx::kern::DmaPlan big = elx::kern::dma_plan(true, 1024, 4096, 16);
    if (!big.use || big.nz != 1 || big.kmain != 4096) { std::printf("FAIL plan 1024 tiles\n"); ++bad; }
    const elx::kern::DmaPlan few = elx::kern::dma_plan(true, 64, 2048, 16);  // 1024^2 in 128-tiles
    if (!few.use || few.nz != 4 || few.kchunk * few.nz < few.kmain) { std::printf("FAIL plan 64 tiles: nz %d\n", few.nz); ++bad; }
    const elx::kern::DmaPlan t64 = elx::kern::dma_plan(true, 256, 2048, 16);  // 1024^2 in 64-tiles
    if (!t64.use || t64.nz != 1) { std::printf("FAIL plan 256 tiles: nz %d\n", t64.nz); ++bad; }
    // the 16-bit four-wave kernel's tile (h16_plan): 256 / 192 / 128 by the
    // round-6 map (profiles/r06d_h16_tile_map.log, r06c_h16_tile192_sweep.log);
    // 4608^3 (324 256-tiles) takes 256 with the split-k tail, TN the 224-tiles
    // (profiles/r06v_h16_tailsk_ab.log)
    struct H { i64 m, n, k; int wm; bool tn; };
    const H hc[] = {
        {3072, 3072, 3072, 6, false},   {6144, 6144, 6144, 8, false},   {3072, 3072, 12288, 6, false},
        {2560, 2560, 8192, 4, false},   {2560, 2560, 2560, 4, false},   {3584, 3584, 3584, 8, false},
        {4096, 4096, 4096, 8, false},   {4608, 4608, 4608, 8, false},   {5120, 5120, 5120, 8, false},
        {7168, 7168, 7168, 8, false},   {12288, 12288, 12288, 8, false}, {32768, 32768, 32768, 8, false},
        {16384, 8192, 8192, 8, false},  {2048, 2048, 2048, 4, false},   {1536, 2048, 2048, 2, false},
        {1024, 1024, 8192, 4, false},   {4096, 2048, 4096, 4, false},   {8192, 4096, 2048, 8, false},
        {6144, 4096, 4096, 8, false},   {3072, 8192, 4096, 8, false},   // 1.5 rounds: 256 stays
        // 64-tiles: 64..255 128-tiles and no split-k
        {1024, 1024, 1024, 2, false},   {1536, 1536, 1536, 2, false},   {1024, 2048, 1024, 2, false},
        {512, 1024, 1024, 4, false},    {1024, 1024, 1024, 2, true},
        // TN may take the 224- and 160-tiles
        {3584, 3584, 3584, 7, true},    {2560, 2560, 2560, 5, true},    {3072, 3072, 3072, 6, true},
        {4096, 4096, 4096, 8, true},    {16384, 16384, 16384, 8, true}, {2048, 2048, 2048, 4, true},
        {4608, 4608, 4608, 7, true},
    };
    for (const H& c : hc) {
        const elx::kern::H16Plan pl = elx::kern::h16_plan(c.m, c.n, c.k, c.tn);
        if (pl.wm != c.wm) {
            std::printf("FAIL h16_plan %lld x %lld x %lld%s: wm %d want %d\n", (long long)c.m, (long long)c.n,
                        (long long)c.k, c.tn ? " TN" : "", pl.wm, c.wm);
            ++bad;
        }
    }
    const elx::kern::H16Plan sk = elx::kern::h16_plan(1024, 1024, 8192);  // 64 128-tiles: split k
    if (sk.nz < 2 || sk.kchunk * sk.nz < 8192) { std::printf("FAIL h16 split 1024^2 x 8192: nz %lld\n", (long long)sk.nz); ++bad; }
    std::printf("%s (%d failures)\n", bad ? "FAILED" : "ok", bad);
    return bad ? 1 : 0;
}
