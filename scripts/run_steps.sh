#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to gpurun_out/<dir>/<name>.log:
#   scripts/run_steps.sh <dir> "<name>|<seconds>|<command>" ...
# A failing step (ordinary non-zero exit) is reported and the next step runs; a step that ends by
# a time limit, abort or crash (exit 124, 134, 137, 139) stops the run: nothing more touches the GPU.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; shift; mkdir -p "$out"
rc_all=0
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "   exit $rc"; tail -4 "$out/$name.log"
  case $rc in 124|134|137|139) echo "stopping after $name (exit $rc)"; exit $rc ;; esac
  [ $rc -ne 0 ] && rc_all=$rc
done
exit $rc_all
