# Round 6, final tree (clock-settle steps in the bench): the rocprofv3 kernel trace + stats of the EXACT driver command
# (python3 bench.py --gpus 1 --steps 20 --warmup 5), the headline PMC passes (each its own run),
# and config 4's queries under the trace and the L2 passes.
# Summarise with: python tools/summarize_profile.py --round r06f --src gpurun_out/prof6f
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/prof6f
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/trace.log 2>&1 || exit 3
B="python3 bench.py --no-cpu --no-paths --pair-steps 0 --steps 5 --warmup 2 --settle-steps 0"
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $P/pmc$i -o run --output-format csv -- $B > $P/pmc$i.log 2>&1 || echo "pmc pass $i failed"
done
N="python3 tools/nearest_run.py --reps 3"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $P/ntrace -o run --output-format csv -- $N > $P/ntrace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $P/npmc$i -o run --output-format csv -- $N > $P/npmc$i.log 2>&1 || echo "nearest pmc pass $i failed"
done
grep -h '^{' $P/trace.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced run ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline'].get('kernel_ms'))"
echo done
