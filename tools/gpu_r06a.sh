set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pool" > gpurun_out/r06a_pool.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py -k "blas1 or summa or rccl" > gpurun_out/r06a_dist.log 2>&1 && \
ELX_BENCH_COMM=host timeout -k 10 600 python3 bench.py --gpus 2 --size 8192 --steps 2 > gpurun_out/r06a_launch2.json 2> gpurun_out/r06a_launch2.err
echo "rc=$?"
