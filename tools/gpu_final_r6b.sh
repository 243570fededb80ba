#!/bin/bash
# round-6 closing run on the final tree: the whole -m gpu suite, smoke(), the default bench line
set -u
P=gpurun_out/r6final
mkdir -p $P
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?; tail -2 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $P/smoke.log 2>&1 || { tail -5 $P/smoke.log; exit 3; }
tail -1 $P/smoke.log
timeout -k 10 600 python3 bench.py > $P/bench.json 2> $P/bench.err || exit 3
python3 -c "import json; d=json.loads(open('$P/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['paths']['dropin_summary_737k'].get('ms'), d['paths']['scalar_calls'].get('us_per_call'))"
