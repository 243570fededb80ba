# Round 6: nearest with the whitelist in alphabetical (key) order -- whitelist indices written by the
# query kernel, no index pass -- vs the same whitelist shuffled: the nearest GPU tests, config 4's
# bench path twice, a kernel trace and the TCC request pass of the path.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6k
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_devices.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "nearest or corrector" > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -3 $P/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/run_path.py config4 10 > $P/config4_$i.json 2> $P/config4_$i.err || { tail $P/config4_$i.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$P/config4_$i.json')); print('sorted', round(d['ms'],4), 'shuffled', round(d['shuffled_whitelist_ms'],4), d['shuffled_whitelist_answers_equal'], d['check'])"
done
N="python3 tools/run_path.py config4 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $N > $P/trace.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum -d $P/pmc1 -o run --output-format csv -- $N > $P/pmc1.log 2>&1 || echo "pmc1 failed"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc2 -o run --output-format csv -- $N > $P/pmc2.log 2>&1 || echo "pmc2 failed"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $P/pmc3 -o run --output-format csv -- $N > $P/pmc3.log 2>&1 || echo "pmc3 failed"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P/pmc4 -o run --output-format csv -- $N > $P/pmc4.log 2>&1 || echo "pmc4 failed"
echo done
