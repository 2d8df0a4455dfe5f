#!/bin/bash
# Build a variant of the library for an in-box A/B (tools/variant_ab.sh):
#   tools/variant_build.sh <name> <file-in-csrc>=<replacement source> ...
# copies csrc, swaps in the given files, builds into tools/_build_probe/<name>/
# elemental_amd (the python package + its own .so; scratch, git-ignored).
set -e
N=$1; shift
R=/root/repo
rm -rf /tmp/hs_$N /tmp/hb_$N $R/tools/_build_probe/$N
mkdir -p /tmp/hs_$N/elemental_amd /tmp/hs_$N/include $R/tools/_build_probe/$N
cp -r $R/elemental_amd/csrc /tmp/hs_$N/elemental_amd/csrc
cp $R/include/elemental_amd.h /tmp/hs_$N/include/
for kv in "$@"; do cp "${kv#*=}" /tmp/hs_$N/elemental_amd/csrc/"${kv%%=*}"; done
cp -r $R/elemental_amd $R/tools/_build_probe/$N/
rm -rf $R/tools/_build_probe/$N/elemental_amd/csrc $R/tools/_build_probe/$N/elemental_amd/libelemental_amd.so
make -s -j8 -C /tmp/hs_$N/elemental_amd/csrc OUT=$R/tools/_build_probe/$N/elemental_amd/libelemental_amd.so BUILD=/tmp/hb_$N 2>&1 | grep -E "error" || true
ls -la $R/tools/_build_probe/$N/elemental_amd/libelemental_amd.so
