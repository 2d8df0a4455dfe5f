#!/bin/bash
# round-6 call o: exact-integer fuzz of the 16-bit plan (random shapes, every
# orientation, both types: tiles, tail split, k tails)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python3 tools/h16_exact_check.py . 4032,4624,808 3720,2456,1000 2872,1688,1408 1096,4528,912 1416,4064,256 3224,4096,320 3088,4192,192 1608,3672,944 4024,4096,1352 3376,1024,432 1472,2512,232 4440,1320,736 1944,2352,1408 3064,1808,264 3584,4368,1856 1104,1248,256 4096,4352,1024 3584,3584,512 2560,2560,704 7168,1024,1024 4608,2304,1088 > gpurun_out/r06o_fuzz.log 2>&1 || exit $?
exit 0
