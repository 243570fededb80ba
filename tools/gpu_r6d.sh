# Round 6: the whole GPU suite on the current tree, then the host-array path again (pool fix).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6d
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python3 tools/run_paths.py host_arrays > $P/host_arrays.json 2> $P/host_arrays.err || exit 3
echo done
