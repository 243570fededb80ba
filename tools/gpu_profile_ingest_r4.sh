# The ingest / FASTQ part of tools/gpu_profile_r4.sh alone (kernel trace + PMC passes of
# tools/run_paths.py whitelist fastq pipeline) into gpurun_out/prof4/{itrace,ipmc*}.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/prof4
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
exit 0
