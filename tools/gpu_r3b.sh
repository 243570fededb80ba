# GPU suite, then the round-3 profiles (tools/gpu_profile_r3.sh), then a bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=25 \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
if [ "${PROFILE:-1}" = "1" ]; then bash tools/gpu_profile_r3.sh || exit $?; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
exit 0
