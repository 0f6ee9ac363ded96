#!/bin/bash
# Run one gpurun call; retry only when no box was obtained (exit 3: nothing ran).
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 45
done
exit 3
