#!/bin/bash
# Runs a sequence of GPU steps, each under its own time limit. A step that
# times out, aborts or segfaults (124/137/134/139) ends the session; an
# ordinary failure (e.g. a failing test) is recorded and the next step runs.
# usage: tools/gpu_session.sh "name|seconds|command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in 124|137|134|139) echo "fatal rc=$rc: stopping session"; exit $rc;; esac
done
exit 0
