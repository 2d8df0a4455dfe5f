#!/bin/bash
# A/B of the in-tree library ("head") against a variant tree built by
# tools/variant_build.sh, alternating processes on one box (HENV / VENV: env
# assignments for each arm):
#   HENV="" VENV="" tools/variant_ab.sh <name> <reps> <gemm_bench specs...>
set -o pipefail
R=$GRAFT_REPO_ROOT
V=$1; REPS=$2; shift 2
S="$*"
cd $R/tools
run() {  # $1 = package root, $2 = env assignments for this arm
  env $2 timeout -k 10 300 python3 -c "
import sys; sys.argv=['gemm_bench.py']+'$S'.split()
sys.path.insert(0,'$1'); sys.path.insert(1,'$R/tools')
import elemental_amd._lib as L; print(L.LIB_PATH)
exec(open('$R/tools/gemm_bench.py').read().replace('sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))',''))
" 2>&1 | grep -v amdgpu.ids
}
for rep in $(seq 1 $REPS); do
  echo "== head rep $rep [$HENV]"; run $R "$HENV" || exit 1
  echo "== $V rep $rep [$VENV]"; run $R/tools/_build_probe/$V "$VENV" || exit 1
done
