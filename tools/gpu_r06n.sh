#!/bin/bash
# round-6 call n: fragment reads one per two MFMAs (variant rs2) against HEAD,
# alternating processes; the variant's exact-integer check first
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 tools/h16_exact_check.py tools/_build_probe/rs2 > gpurun_out/r06n_tests.log 2>&1 || exit $?
timeout -k 10 900 bash tools/variant_ab.sh rs2 3 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,1,0,16384,16384,16384 bf16,1,1,16384,16384,16384 bf16,0,0,32768,32768,32768 bf16,0,0,4096,4096,4096 > gpurun_out/r06n_rs2_ab.log 2>&1 || exit $?
exit 0
