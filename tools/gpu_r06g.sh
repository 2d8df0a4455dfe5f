#!/bin/bash
# round-6 call g: the N > 1 bench line through bench.py's own rank launch,
# host-staged on one GPU (1x2, 2x2, 2x4), the pool release-path timings, and the
# rocprofv3 kernel-trace summary of the default N = 1 line
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r06_rehearsal
for n in 2 4 8; do
  ELX_BENCH_COMM=host timeout -k 10 400 python3 bench.py --gpus $n --size 8192 --steps 2 --warmup 1 \
    > gpurun_out/r06_rehearsal/r$n.json 2> gpurun_out/r06_rehearsal/r$n.err
  rc=$?; echo "gpus $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "release_path" > gpurun_out/r06g_release.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06g -o bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3-1gpu > $R/gpurun_out/prof_r06g_bench.log 2>&1 || exit $?
exit 0
