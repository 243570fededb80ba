# rocprofv3 kernel trace + PMC passes over the config-4 nearest-whitelist path only.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profn
export TMPDIR=/tmp
B="python3 tools/bench_paths.py --skip-allpairs5 --reads 1000000 --stream-reads 1000000"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/profn/trace -o run --output-format csv -- $B > gpurun_out/profn/trace.log 2>&1 || exit 3
i=0
for pmc in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TA_TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d gpurun_out/profn/pmc$i -o run --output-format csv -- $B > gpurun_out/profn/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; }
done
exit 0
