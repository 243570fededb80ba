#!/bin/bash
# the whole -m gpu suite on the current tree, then the scalar per-call latencies (two rounds) and
# the C-call floor probe
set -u
P=gpurun_out/r6r
mkdir -p $P
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python3 tools/scalar_latency.py > $P/latency.$r.json 2> $P/latency.$r.err || exit 3
  cat $P/latency.$r.json
done
timeout -k 10 120 tools/scalar_floor_probe > $P/floor.jsonl 2> $P/floor.err || exit 3
grep '"c_call"' $P/floor.jsonl
