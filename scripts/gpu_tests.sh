#!/bin/bash
# GPU parity suite (optionally a subset: TESTS="tests/x.py tests/y.py"), then smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 ${T_TEST:-1000} python -u -m pytest $T -v -m gpu -x --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ "$rc" -eq 0 ] || exit $rc
if [ -z "$NO_SMOKE" ]; then
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
exit $rc
fi
