# PMC passes over the SPECTRAL seed kernels: the MFMA seed (default) and the walk seed.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python3 tools/spectral_time.py 2 2"
for v in mx walk; do
  mkdir -p gpurun_out/profs_$v
  sv=$v; [ $v = mx ] && sv=""
  export SCT_SPECTRAL_SEED=$sv
  i=0
  for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_WR SQ_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/profs_$v/pmc$i -o run --output-format csv -- $B > gpurun_out/profs_$v/pmc$i.log 2>&1 || { echo "pmc pass $v $i failed"; }
  done
done
exit 0
