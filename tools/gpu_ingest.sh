# whitelist ingest + base_frequency: parity tests, the bench path, a kernel trace of the path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "encode_var or base_frequency or whitelist or golden" tests/test_fastq.py > gpurun_out/ingest_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/run_path.py whitelist > gpurun_out/wl.json 2> gpurun_out/wl.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/wlprof -o wl -- python3 tools/run_path.py whitelist > gpurun_out/wlprof.log 2>&1
rc=$?; tail -3 gpurun_out/ingest_tests.log; cat gpurun_out/wl.json; exit $rc
