# Round-2 GPU call: smoke, GPU parity tests, bench (N = 1), and a 2-rank launcher rehearsal
# (gloo, both ranks on the box's one GPU).  Stops at the first crash/timeout (exit > 1).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
  timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --allow-shared-gpu --steps 5 --warmup 2 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank.err || exit $?
fi
exit 0
