/* CPU SUMMA for bench.py's cpu_baseline leg — TEST INFRASTRUCTURE ONLY.
 *
 * BASELINE.json configs[0] (C1), El::Gemm NN fp64 m=n=k=N on an r x c grid,
 * run the way the reference's CPU path runs it (SUMMA_NNC,
 * src/blas_like/level3/Gemm/NN.hpp:341-385) on one node: one process per grid
 * rank (column-major grid, src/core/Grid.cpp:147-148), element-cyclic [MC,MR]
 * local blocks (src/core/indexing/impl.hpp:33-36,244-245), C := beta C first
 * (Gemm.cpp:282), then per Blocksize() panel k0:k0+nb
 *
 *   A1[MC,*] <- A(:, k0:k0+nb)   all-gather over the grid row    (RowAllGather)
 *   B1[*,MR] <- B(k0:k0+nb, :)   all-gather over the grid column (NN.hpp:370-372's
 *                                  [MR,*] gather, untransposed)
 *   C_loc   += alpha A1 B1       one dgemm_ of MKL (the reference's BLAS) per panel
 *
 * The all-gathers use shared memory, as MPI's on-node transport does: each rank
 * packs its portion of the panel into its slot of a shared segment (sender copy),
 * all ranks meet at a process-shared barrier, each copies its peers' portions
 * into its panel (receiver copy).  Two slot sets alternate, so one barrier per
 * panel suffices: a slot is rewritten two panels later, after every reader has
 * passed the barrier that follows its reads.  Times in dgemm_ and in the
 * exchange (pack + barrier + unpack) are reported separately, as the reference's
 * BasicGemm does (tests/blas_like/BasicGemm.cpp:11-82).
 *
 *   cpu_summa N NB R C THREADS SECONDS MKL_PATH
 * prints one JSON object; inputs are the oracle's hash (Uniform(-0.1, 0.1)),
 * alpha = 0.5, beta = -0.5; 8 entries per rank are checked against direct dot
 * products of the global inputs before the timing is reported.
 *
 * Placement (round 4): rank q pins itself to its own THREADS cpus of the
 * process's allowed set (cpus q*THREADS .. q*THREADS+THREADS-1 of it) before
 * MKL's OpenMP runtime starts, and its threads spin between the per-panel
 * calls (OMP_WAIT_POLICY=ACTIVE: the cpus are the rank's alone), as an MPI
 * launcher's --bind-to core placement runs the reference.  CPU_SUMMA_PIN=0
 * keeps the unpinned, passive-wait placement of rounds 2-3.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <cpuid.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "oracle.h"

typedef void (*dgemm_fn)(const char*, const char*, const int*, const int*, const int*, const double*, const double*,
                         const int*, const double*, const int*, const double*, double*, const int*);
typedef void (*set_threads_fn)(const int*);

struct Shared {
    pthread_barrier_t bar;
    int steps;          /* decided by rank 0 after the calibration step */
    int failed;         /* any rank's entry check failed */
    double elapsed[64]; /* per rank: timed steps */
    double t_gemm[64], t_xchg[64];
};

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int64_t len(int64_t n, int64_t shift, int64_t stride) { return n > shift ? (n - shift - 1) / stride + 1 : 0; }

struct Rank {
    int rank, n, nb, r, c, mc, mr, world, threads;
    int64_t lh, lw;
    double *A, *B, *C0, *C, *A1, *B1;
    double* slots;
    size_t slot_elems;
    struct Shared* sh;
    dgemm_fn dgemm;
    double tg, tx;
};

/* slot (set s, rank q): A portion (lh_q x ceil(nb/c)) then B portion (ceil(nb/r) x lw_q), column-major */
static double* slot(const struct Rank* R, int set, int q) {
    return R->slots + ((size_t)set * R->world + q) * R->slot_elems;
}

static void one_step(struct Rank* R) {
    const int n = R->n, nb = R->nb, r = R->r, c = R->c, mc = R->mc, mr = R->mr;
    const int64_t lh = R->lh, lw = R->lw;
    const double alpha = 0.5, beta = -0.5, one = 1.0;
    const int ilh = (int)lh, ilw = (int)lw, inb = nb;
    for (int64_t q = 0; q < lh * lw; ++q) R->C[q] = beta * R->C0[q];
    int set = 0;
    for (int k0 = 0; k0 < n; k0 += nb, set ^= 1) {
        const int kb = n - k0 < nb ? n - k0 : nb;
        const double t0 = now();
        /* sender copy: my columns of A(:, k0:k0+kb) (j = mr + jl c) and rows of B(k0:k0+kb, :) (i = mc + il r) */
        double* s = slot(R, set, R->rank);
        const int64_t ja = (k0 - mr + c - 1) / c, jb = (k0 + kb - mr + c - 1) / c;
        const int64_t ia = (k0 - mc + r - 1) / r, ib = (k0 + kb - mc + r - 1) / r;
        /* the copies run on the rank's threads (the MKL GNU-threading pool's runtime),
           as a threaded MPI pack would; column by column, so no two threads share a
           destination cache line of any size that matters */
        double* sb = s + lh * ((nb + c - 1) / c);
        const int64_t nja = jb - ja, nib = ib - ia, lhB = len(n, mc, r);
#pragma omp parallel num_threads(R->threads)
        {
#pragma omp for schedule(static) nowait
            for (int64_t q = 0; q < nja; ++q) memcpy(s + q * lh, R->A + (ja + q) * lh, sizeof(double) * lh);
#pragma omp for schedule(static)
            for (int64_t jl = 0; jl < lw; ++jl) memcpy(sb + jl * nib, R->B + ia + jl * lhB, sizeof(double) * nib);
        }
        pthread_barrier_wait(&R->sh->bar);
        /* receiver copy: column q of A1 is global column k0 + q, held by grid column (k0 + q) mod c;
           row q of B1 is global row k0 + q, held by grid row (k0 + q) mod r */
#pragma omp parallel num_threads(R->threads)
        {
#pragma omp for schedule(static) nowait
            for (int q = 0; q < kb; ++q) {
                const int j = k0 + q, pc = j % c;
                const double* pa = slot(R, set, mc + r * pc);
                const int64_t pja = (k0 - pc + c - 1) / c;
                memcpy(R->A1 + (int64_t)q * lh, pa + (j / c - pja) * lh, sizeof(double) * lh);
            }
#pragma omp for schedule(static)
            for (int64_t jl = 0; jl < lw; ++jl)
                for (int pr = 0; pr < r; ++pr) {
                    const double* pb = slot(R, set, pr + r * mr) + len(n, pr, r) * ((nb + c - 1) / c);
                    const int64_t pia = (k0 - pr + r - 1) / r, cnt = (k0 + kb - pr + r - 1) / r - pia;
                    for (int64_t t = 0; t < cnt; ++t) R->B1[(pr + (pia + t) * r - k0) + jl * nb] = pb[t + jl * cnt];
                }
        }
        const double t1 = now();
        const int ikb = kb;
        R->dgemm("N", "N", &ilh, &ilw, &ikb, &alpha, R->A1, &ilh, R->B1, &inb, &one, R->C, &ilh);
        const double t2 = now();
        R->tx += t1 - t0;
        R->tg += t2 - t1;
    }
}

static int pin_ranks(void) {
    const char* e = getenv("CPU_SUMMA_PIN");
    return !(e && e[0] == '0');
}

static int run_rank(int rank, int n, int nb, int r, int c, int threads, double seconds, const char* mkl_path,
                    struct Shared* sh, double* slots, size_t slot_elems) {
    if (pin_ranks()) {  /* this rank's own cpus (see the header) */
        cpu_set_t all, mine;
        CPU_ZERO(&mine);
        if (sched_getaffinity(0, sizeof(all), &all) == 0) {
            int seen = 0, got = 0;
            for (int cpu = 0; cpu < CPU_SETSIZE && got < threads; ++cpu) {
                if (!CPU_ISSET(cpu, &all)) continue;
                if (seen++ >= rank * threads) { CPU_SET(cpu, &mine); ++got; }
            }
            if (got == threads) sched_setaffinity(0, sizeof(mine), &mine);
        }
    }
    struct Rank R = {0};
    R.rank = rank; R.n = n; R.nb = nb; R.r = r; R.c = c; R.world = r * c; R.threads = threads;
    R.mc = rank % r; R.mr = rank / r;
    R.lh = len(n, R.mc, r); R.lw = len(n, R.mr, c);
    R.slots = slots; R.slot_elems = slot_elems; R.sh = sh;
    const int64_t lh = R.lh, lw = R.lw;
    R.A = malloc(sizeof(double) * lh * lw);
    R.B = malloc(sizeof(double) * lh * lw);
    R.C0 = malloc(sizeof(double) * lh * lw);
    R.C = malloc(sizeof(double) * lh * lw);
    R.A1 = malloc(sizeof(double) * lh * nb);
    R.B1 = malloc(sizeof(double) * nb * lw);
    if (!R.A || !R.B || !R.C0 || !R.C || !R.A1 || !R.B1) return 2;
    /* [MC,MR] local blocks of the global hash matrices: X(i,j) with i = mc + il r, j = mr + jl c */
    for (int64_t jl = 0; jl < lw; ++jl)
        for (int64_t il = 0; il < lh; ++il) {
            const int64_t i = R.mc + il * r, j = R.mr + jl * c;
            R.A[il + jl * lh] = -0.1 + 0.2 * orc_hash_unit(1, i, j);
            R.B[il + jl * lh] = -0.1 + 0.2 * orc_hash_unit(2, i, j);
            R.C0[il + jl * lh] = -0.1 + 0.2 * orc_hash_unit(3, i, j);
        }
    void* mkl = dlopen(mkl_path, RTLD_NOW | RTLD_LOCAL);
    if (!mkl) { fprintf(stderr, "cpu_summa: cannot load %s\n", mkl_path); return 3; }
    R.dgemm = (dgemm_fn)dlsym(mkl, "dgemm_");
    set_threads_fn set_threads = (set_threads_fn)dlsym(mkl, "mkl_set_num_threads");
    if (!R.dgemm || !set_threads) return 3;
    set_threads(&threads);

    one_step(&R); /* warm-up: thread pool, pages */
    /* a few entries against direct dot products of the global inputs */
    uint64_t z = 0x9e3779b97f4a7c15ull * (uint64_t)(rank + 1);
    for (int t = 0; t < 8 && lh && lw; ++t) {
        z = orc_splitmix64(z);
        const int64_t il = (int64_t)(z % (uint64_t)lh), jl = (int64_t)((z >> 32) % (uint64_t)lw);
        const int64_t i = R.mc + il * r, j = R.mr + jl * c;
        double want = 0;
        for (int64_t q = 0; q < n; ++q)
            want += (-0.1 + 0.2 * orc_hash_unit(1, i, q)) * (-0.1 + 0.2 * orc_hash_unit(2, q, j));
        want = 0.5 * want - 0.5 * (-0.1 + 0.2 * orc_hash_unit(3, i, j));
        if (fabs(R.C[il + jl * lh] - want) > 1e-12) {
            fprintf(stderr, "cpu_summa: rank %d entry (%ld,%ld) %.17g vs %.17g\n", rank, (long)i, (long)j,
                    R.C[il + jl * lh], want);
            sh->failed = 1;
        }
    }
    pthread_barrier_wait(&sh->bar);
    double t0 = now();
    one_step(&R);
    const double first = now() - t0;
    if (rank == 0) {
        const int s = (int)(seconds / (first > 1e-3 ? first : 1e-3));
        sh->steps = s < 2 ? 2 : s;
    }
    pthread_barrier_wait(&sh->bar);
    R.tg = R.tx = 0;
    t0 = now();
    for (int s = 0; s < sh->steps; ++s) one_step(&R);
    pthread_barrier_wait(&sh->bar);
    sh->elapsed[rank] = now() - t0;
    sh->t_gemm[rank] = R.tg;
    sh->t_xchg[rank] = R.tx;
    free(R.A); free(R.B); free(R.C0); free(R.C); free(R.A1); free(R.B1);
    return 0;
}

/* MKL 2021.4 runs its AVX-512 kernels only where it finds an Intel CPU (AVX2
 * code elsewhere).  The reference's C1 figure was measured on a Xeon (BASELINE.md
 * §2), i.e. through those kernels; the GPU box's host is an AMD EPYC 9575F (Zen 5,
 * full AVX-512).  MKL asks this function whether the CPU is Intel's: exported
 * from the executable (-rdynamic), it is what the dlopen'd MKL binds to, and it
 * says yes, so the baseline runs the reference's code path on this host too.
 * CPU_SUMMA_MKL_VENDOR=1 answers from the CPUID vendor string instead (MKL's own
 * dispatch). */
int mkl_serv_intel_cpu_true(void) {
    const char* v = getenv("CPU_SUMMA_MKL_VENDOR");
    if (!(v && v[0] == '1')) return 1;
    unsigned a, b, c, d;
    if (!__get_cpuid(0, &a, &b, &c, &d)) return 0;
    return b == 0x756e6547u && d == 0x49656e69u && c == 0x6c65746eu; /* "GenuineIntel" */
}

int main(int argc, char** argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s N NB R C THREADS SECONDS MKL_PATH\n", argv[0]);
        return 1;
    }
    const int n = atoi(argv[1]), nb = atoi(argv[2]), r = atoi(argv[3]), c = atoi(argv[4]), threads = atoi(argv[5]);
    const double seconds = atof(argv[6]);
    const char* mkl = argv[7];
    const int world = r * c;
    if (n <= 0 || nb <= 0 || r <= 0 || c <= 0 || world > 64 || threads <= 0) return 1;
    /* one slot per (set, rank): the largest A portion plus the largest B portion */
    const size_t slot_elems = (size_t)len(n, 0, r) * ((nb + c - 1) / c) + (size_t)((nb + r - 1) / r) * len(n, 0, c);
    const size_t bytes = sizeof(struct Shared) + 64 + sizeof(double) * slot_elems * 2 * world;
    char* seg = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (seg == MAP_FAILED) return 2;
    struct Shared* sh = (struct Shared*)seg;
    double* slots = (double*)(seg + ((sizeof(struct Shared) + 63) / 64) * 64);
    pthread_barrierattr_t ba;
    pthread_barrierattr_init(&ba);
    pthread_barrierattr_setpshared(&ba, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init(&sh->bar, &ba, (unsigned)world);
    setenv("MKL_THREADING_LAYER", "GNU", 1); /* the reference's runs require GNU or SEQUENTIAL */
    if (!getenv("OMP_WAIT_POLICY")) setenv("OMP_WAIT_POLICY", pin_ranks() ? "ACTIVE" : "PASSIVE", 1);
    if (!getenv("MKL_DYNAMIC")) setenv("MKL_DYNAMIC", "FALSE", 1);  /* exactly THREADS threads per call */
    pid_t pids[64];
    for (int q = 0; q < world; ++q) {
        pids[q] = fork();
        if (pids[q] < 0) return 2;
        if (pids[q] == 0) _exit(run_rank(q, n, nb, r, c, threads, seconds, mkl, sh, slots, slot_elems));
    }
    int bad = 0;
    for (int q = 0; q < world; ++q) {
        int st = 0;
        waitpid(pids[q], &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad = 1;
    }
    if (bad || sh->failed) {
        fprintf(stderr, "cpu_summa: a rank failed\n");
        return 4;
    }
    double el = 0, tg = 0, tx = 0;
    for (int q = 0; q < world; ++q) {
        if (sh->elapsed[q] > el) el = sh->elapsed[q];
        tg += sh->t_gemm[q] / world;
        tx += sh->t_xchg[q] / world;
    }
    const double tf = 2.0 * (double)n * n * n * sh->steps / el / 1e12;
    printf("{\"value\": %.4f, \"steps\": %d, \"elapsed_s\": %.3f, \"gemm_s\": %.3f, \"exchange_s\": %.3f}\n", tf,
           sh->steps, el, tg, tx);
    return 0;
}
