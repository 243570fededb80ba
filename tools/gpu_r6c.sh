# Round 6: the streamed batch-array tests, the host-array bench path, and the tile squares A/B.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6c
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_devices.py::test_batch_arrays_streamed" "tests/test_gpu_parity.py::test_hamming_golden" \
  "tests/test_gpu_parity.py::test_decode_array_golden" "tests/test_gpu_parity.py::test_negative_ints_golden" > $P/pytest.log 2>&1
rc=$?
tail -3 $P/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python3 tools/run_paths.py host_arrays > $P/host_arrays.json 2> $P/host_arrays.err || exit 3
timeout -k 10 400 python3 tools/tile_ab.py base= sqabl=sctools_amd/libsctools_hip_sqabl.so --rounds 3 > $P/tile_sq_ab.jsonl 2>&1 || exit 3
echo done
