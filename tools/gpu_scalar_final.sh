#!/bin/bash
# scalar drop-in calls on the final library: the server's GPU tests, the C call floor probe and the
# Python per-call latencies (tools/scalar_latency.py), two rounds
set -u
P=gpurun_out/r6o
mkdir -p $P
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scalar_server.py \
  > $P/pytest_scalar.log 2>&1 || { tail -30 $P/pytest_scalar.log; exit 3; }
tail -1 $P/pytest_scalar.log
timeout -k 10 120 tools/scalar_floor_probe > $P/floor.jsonl 2> $P/floor.err || exit 3
for r in 1 2; do
  timeout -k 10 120 python3 tools/scalar_latency.py > $P/latency.$r.json 2> $P/latency.$r.err || exit 3
  cat $P/latency.$r.json
done
