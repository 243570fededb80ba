# Round-5 rocprofv3 kernel traces and PMC passes (each pass its own run, within the per-block
# counter limits) of the side paths: the whitelist ingest / FASTQ / FASTQ -> nearest kernels
# (tools/run_paths.py) and config 4's nearest queries (tools/nearest_run.py), into the final
# round-5 profile directory; tools/summarize_profile.py --round r05 --src gpurun_out/prof5z.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/prof5z
mkdir -p $P
export TMPDIR=/tmp
I="python3 tools/run_paths.py whitelist fastq pipeline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $P/itrace -o run --output-format csv -- $I > $P/itrace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $P/ipmc$i -o run --output-format csv -- $I > $P/ipmc$i.log 2>&1 || echo "ingest pmc pass $i failed"
done
N="python3 tools/nearest_run.py --reps 3"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $P/ntrace -o run --output-format csv -- $N > $P/ntrace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $P/npmc$i -o run --output-format csv -- $N > $P/npmc$i.log 2>&1 || echo "nearest pmc pass $i failed"
done
exit 0
