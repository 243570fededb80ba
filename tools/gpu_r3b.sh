# GPU suite, then the round-3 profiles (tools/gpu_profile_r3.sh) summarised into profiles/ on
# the box (copied to gpurun_out/profiles_new/ so they come back), then a bench line that reads
# those same summaries: its live kernel times and the committed rocprof averages are from one box.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=25 \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  bash tools/gpu_profile_r3.sh || exit $?
  python tools/summarize_profile.py --round r03 > gpurun_out/summarize.log 2>&1 || exit 4
  mkdir -p gpurun_out/profiles_new
  cp profiles/r03_*kernel_stats.csv profiles/pmc_*_r03.json gpurun_out/profiles_new/ || exit 5
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
exit 0
