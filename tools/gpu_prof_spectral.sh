# rocprofv3 kernel trace + HBM PMC passes over the SPECTRAL all-pairs kernels
# (tools/ab_allpairs.py, scheme 2) on config ${SP_CONFIG:-2}.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/profsp
B="python3 tools/ab_allpairs.py --config ${SP_CONFIG:-2} --rounds 3 --variants v=1,s=2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/profsp/trace -o run --output-format csv -- $B > gpurun_out/profsp/trace.log 2>&1 || exit 3
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" ${SP_PMC:-}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/profsp/pmc$i -o run --output-format csv -- $B > gpurun_out/profsp/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 4; }
done
