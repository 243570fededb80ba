# Round 6: pipelined step with the next build enqueued before this step's tail: the sharded /
# pipelined GPU tests, the emulated W = 8 share (plain and traced), the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6q
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_devices.py -x -q -m gpu --timeout 200 \
  --timeout-method thread -k "sharded or pipelined or ranks or multirank or rccl or devices or 737k" > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -2 $P/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/w8_share.py 8 40 > $P/w8_$i.json 2> $P/w8_$i.err || { tail $P/w8_$i.err; exit 3; }
  cat $P/w8_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 tools/w8_share.py 8 40 > $P/trace.log 2>&1 || exit 3
timeout -k 10 600 python3 bench.py --no-paths --no-cpu > $P/bench.log 2> $P/bench.err || { tail $P/bench.err; exit 3; }
python3 -c "
import json; d=json.loads(open('$P/bench.log').read().strip().splitlines()[-1]); print('bench ms_per_step', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['other_kernel']['ms'])"
echo done
