#!/bin/bash
# GPU tests of a subset (TESTS), then an A/B of env variants (VARIANTS, as
# scripts/ab_variants.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_sub.log; [ "$rc" -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then bash scripts/ab_variants.sh; exit $?; fi
exit 0
