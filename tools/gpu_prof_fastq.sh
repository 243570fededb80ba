# rocprofv3 kernel trace + PMC passes over the FASTQ extraction path (tools/bench_paths.py).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/proffq
B="python3 tools/bench_paths.py --reads 0 --stream-reads 0 --queries 0 --skip-allpairs5"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/proffq/trace -o run --output-format csv -- $B > gpurun_out/proffq/trace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/proffq/pmc$i -o run --output-format csv -- $B > gpurun_out/proffq/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; }
done
exit 0
