set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
[ -n "${PATHS_ARGS:-}" ] && { timeout -k 10 400 python -u tools/bench_paths.py $PATHS_ARGS > gpurun_out/paths.json 2> gpurun_out/paths.err || exit $?; }
exit 0
