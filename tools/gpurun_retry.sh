#!/bin/bash
# gpurun with waits while no GPU slot is free ("status=transient" / exit code 3: nothing ran,
# nothing charged).  Any other outcome, success or failure, is returned at once.
log=$(mktemp)
for i in $(seq 1 40); do
    /usr/local/graft/bin/gpurun "$@" 2>&1 | tee "$log"
    rc=${PIPESTATUS[0]}
    if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then rm -f "$log"; exit $rc; fi
    sleep 60
done
rm -f "$log"
exit 3
