# Round 6 late: the whole -m gpu suite on the current tree, smoke(), then the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6final
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $P/smoke.log 2>&1 || { tail $P/smoke.log; exit 3; }
tail -1 $P/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.log 2> $P/bench.err || { tail $P/bench.err; exit 3; }
python3 -c "
import json; d=json.loads(open('$P/bench.log').read().strip().splitlines()[-1])
print('ms_per_step', d['ms_per_step'], 'value', d['value'], 'frac', d['roofline']['frac'])
c=d['paths']['config4_nearest']; print('config4', c['ms'], c['shuffled_whitelist_ms'], c['shuffled_whitelist_answers_equal'], c['check'])"
echo done
