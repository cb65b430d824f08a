# gpurun with a bounded wait for a free slot: retries only when gpurun reports that
# no box or slot was free (nothing ran, nothing charged), at most 8 times, 3 min apart.
#   bash tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "status=ok" $LOG; then sleep 180; continue; fi
  exit $rc
done
exit 3
