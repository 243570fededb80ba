# Round 4: GPU suite (any failure ends the call: nothing after it may run on a red suite),
# then optional path benchmarks / bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
  --durations=15 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "${PATHS_ARGS:-}" ]; then
  timeout -k 10 400 python -u tools/bench_paths.py $PATHS_ARGS > gpurun_out/paths.json 2> gpurun_out/paths.err || exit $?
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
fi
exit 0
