#!/bin/bash
# round-6 call z4: kernel traces of two grids still behind hipBLASLt
# (3328 x 6656 x 4096: 256 + 82 256-tiles, split-k tail; 6144 x 4096^2: 1.5 rounds)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for s in 3328,6656,4096 6144,4096,4096; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06z4_${s//,/x} -o t -- python3 $R/tools/h16_env_ab.py ELX_H16_TILE 0 --reps 1 bf16,0,0,$s > $R/gpurun_out/prof_r06z4_${s//,/x}.log 2>&1 || exit $?
done
exit 0
