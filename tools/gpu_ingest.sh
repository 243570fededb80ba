# whitelist ingest + base_frequency: parity tests, the bench path, a kernel trace of the path
# (TESTS=0 skips the tests)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "encode_var or base_frequency or whitelist or golden" tests/test_fastq.py > gpurun_out/ingest_tests.log 2>&1 || exit 1
  tail -3 gpurun_out/ingest_tests.log
fi
timeout -k 10 240 python -u tools/run_path.py whitelist 20 > gpurun_out/wl.json 2> gpurun_out/wl.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/wlprof -o wl --output-format csv -- python3 tools/run_path.py whitelist 20 > gpurun_out/wlprof.log 2>&1
rc=$?; cat gpurun_out/wl.json; exit $rc
