#!/bin/bash
# round-6 call t: the k tail inside the 16-bit kernel: exact tests, the fuzz
# shapes, the main loop against HEAD's (no tail: must not move), and odd-k timing
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split or ktail" > gpurun_out/r06t_tests.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/h16_exact_check.py . 4032,4624,808 3720,2456,1000 1096,4528,912 1608,3672,944 4024,4096,1352 3376,1024,432 4440,1320,736 3064,1808,264 > gpurun_out/r06t_fuzz.log 2>&1 || exit $?
timeout -k 10 900 bash tools/variant_ab.sh head 3 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,0,0,32768,32768,32768 bf16,0,0,3072,3072,3072 bf16,0,0,4096,4096,4096 bf16,1,0,3584,3584,3584 > gpurun_out/r06t_loop_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_KTAIL 1,0 --beta 1 --reps 3 bf16,0,0,4032,4624,808 bf16,0,0,3720,2456,1000 bf16,0,0,16384,16384,16424 bf16,0,1,8192,8192,8200 > gpurun_out/r06t_ktail_ab.log 2>&1 || exit $?
exit 0
