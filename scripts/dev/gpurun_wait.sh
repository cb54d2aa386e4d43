#!/bin/bash
# run one gpurun command, waiting for a free slot (retries only while gpurun reports no free
# slot / box: exit 3 or a transient status; any other outcome is final)
out=${GPURUN_LOG:-gpurun_out/last_gpurun.log}
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then exit $rc; fi
  sleep 120
done
exit 3
