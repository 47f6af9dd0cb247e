#!/bin/bash
# A pytest selection (PYTEST_K over TESTS), then scripts/r04_check.sh's legs / diagnostics
# without its full suite; each GPU step under its own limit, the first failure ends the call.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_sel.txt 2>&1 || { tail -30 $O/pytest_sel.txt; exit 1; }
tail -1 $O/pytest_sel.txt
SKIP_TESTS=1 bash scripts/r04_check.sh
