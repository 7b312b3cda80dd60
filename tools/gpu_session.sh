#!/bin/bash
# One gpurun session: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# usage: tools/gpu_session.sh <tag> "<step cmd>" ["<step cmd>" ...]
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a "$out/steps.log"
  start=$(date +%s)
  bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc ($(( $(date +%s) - start ))s)" | tee -a "$out/steps.log"
  tail -5 "$out/step$i.log"
  # 0 ok, 1 test failures / python error: keep going; anything else (abort, segv, timeout): stop
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
    echo "=== stopping after rc=$rc" | tee -a "$out/steps.log"
    exit $rc
  fi
done
