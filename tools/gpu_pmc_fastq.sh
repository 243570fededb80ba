# PMC of the FASTQ extraction kernels alone (tools/run_paths.py fastq): issue counters, then HBM
# bytes, each pass its own rocprofv3 run, into gpurun_out/pfq/.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/pfq
mkdir -p $P
export TMPDIR=/tmp
I="python3 tools/run_paths.py fastq"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $P/itrace -o run --output-format csv -- $I > $P/itrace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $P/ipmc$i -o run --output-format csv -- $I > $P/ipmc$i.log 2>&1 || echo "pmc pass $i failed"
done
exit 0
