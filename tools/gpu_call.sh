#!/bin/bash
# Run several GPU step scripts in order; stop at the first that dies by a signal / time limit / abort
# (rc >= 124), go on after an ordinary failure (rc 1-123: e.g. a failing test).
cd "$GRAFT_REPO_ROOT" || exit 1
final=0
for step in "$@"; do
  echo "=== $step"
  bash -c "$step"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  if [ $rc -ne 0 ]; then final=$rc; fi
done
exit $final
