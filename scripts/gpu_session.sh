#!/bin/bash
# Run GPU steps in order; stop at the first step that crashes (fault/abort/timeout).
# Test failures (pytest rc 1) do not stop the session; crashes (rc >= 2 except pytest's 5) do.
# usage: scripts/gpu_session.sh "<name>:<timeout>:<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] $cmd" >&2
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc" >&2
  tail -4 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping after crash in $name (rc=$rc)" >&2
    exit $rc
  fi
done
exit 0
