# One GPU call: parity tests, bench, rocprofv3 trace + PMC passes.  Stops at the first
# crash/timeout (exit >1); a plain test failure (exit 1) still lets the bench run.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 480 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
if [ "${PROFILE:-1}" = "1" ]; then bash tools/gpu_profile.sh || exit $?; fi
exit 0
