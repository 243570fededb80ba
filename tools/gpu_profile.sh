# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC passes
# (each pass its own run, within the per-block counter limits).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --pair-steps 2"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- $B > gpurun_out/prof/trace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE" \
           "SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/prof/pmc$i -o run --output-format csv -- $B > gpurun_out/prof/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; }
done
exit 0
