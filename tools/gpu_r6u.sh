# Round 6: count buffers zeroed on the tail stream after their read-back (no zero kernel, one wait
# fewer on the main stream): the sharded / pipelined GPU tests, then the emulated rank share at
# W = 2, 4, 8 with the build beside the count (side) or in line (main), interleaved
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6u
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_devices.py -x -q -m gpu --timeout 200 \
  --timeout-method thread -k "sharded or pipelined or ranks or multirank or rccl or devices or 737k" > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -2 $P/pytest.log
for i in 1 2; do
  for w in 8 4 2; do
    for m in side main; do
      timeout -k 10 300 python3 tools/w8_share.py $w 40 $m > $P/w${w}_${m}_$i.json 2> $P/err || { tail $P/err; exit 3; }
      echo $w $m $(cat $P/w${w}_${m}_$i.json)
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 tools/w8_share.py 8 40 main > $P/trace.log 2>&1 || exit 3
echo done
