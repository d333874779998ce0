#!/bin/bash
# Run selected GPU test files (default: all -m gpu), each step under its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LOG=${LOG:-gpurun_out/pytest_sel.log}
timeout -k 10 ${TMO:-600} python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread "$@" > $LOG 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $LOG
exit $rc
