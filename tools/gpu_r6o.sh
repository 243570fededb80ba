# Round 6: nearest B-side winners through an 8-bit rank in the A bucket + the offset table instead of
# the permutation: the nearest tests, then config 4's path A/B against HEAD's library
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6o
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_devices.py -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "nearest or corrector" > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -2 $P/pytest.log
timeout -k 10 900 python3 tools/ab_libs.py --path config4 --variant base=sctools_amd/libsctools_hip_base.so --variant rank= --rounds 4 > $P/ab.jsonl 2> $P/ab.err || { tail $P/ab.err; exit 3; }
tail -1 $P/ab.jsonl
echo done
