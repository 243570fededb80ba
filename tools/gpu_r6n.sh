# Round 6: the nearest tests incl. the whitelist-order cases
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6n
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_devices.py -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "nearest or corrector" > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -2 $P/pytest.log
echo done
