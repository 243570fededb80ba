set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc > gpurun_out/nproc.txt; lscpu | head -20 > gpurun_out/lscpu.txt
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"
exit $rc
