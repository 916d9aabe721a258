# Run GPU steps in order: each argument is one shell command (its own time
# limit inside).  An ordinary failure (rc 1-123) is reported and the next step
# still runs; a time limit, abort or crash (rc >= 124, 134, 139) ends the call.
set -u
for step in "$@"; do
  echo "== $step"
  bash -c "$step"
  rc=$?
  echo "== rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc: stopping"; exit $rc; fi
done
