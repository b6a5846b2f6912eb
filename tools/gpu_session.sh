#!/bin/bash
# Runs a list of GPU steps in order; each step has its own time limit; stops at the first fault / abort / timeout
# (exit 124/134/137/139 or signal) -- ordinary test failures (exit 1) do not stop later steps.
# usage: tools/gpu_session.sh "<seconds>|<name>|<command>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $(date +%T) timeout ${secs}s: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ -n "$GPU_SESSION_STRICT" ] && [ $rc -ne 0 ]; then echo "=== stopping (strict): step $name ended with $rc"; exit $rc; fi
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping: step $name ended with $rc"; exit $rc ;;
  esac
  # a GPU fault surfaces in Python as an ordinary exception (exit 1): stop on the fault words too
  if grep -q -i -E "illegal memory access|memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU fault|hipErrorLaunchFailure|unspecified launch failure" "gpurun_out/$name.log"; then
    echo "=== stopping: step $name logged a GPU fault"; exit 86
  fi
done
