#!/bin/bash
# Retry *acquiring* a GPU box (gpurun exit 3 = nothing ran, nothing charged).
# Any other exit code -- including failures of the command itself -- is final.
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep ${WAIT:-60}
done
exit 3
