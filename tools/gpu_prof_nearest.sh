# rocprofv3 kernel trace + PMC passes over the config-4 nearest-whitelist query (100M
# ThreeBit queries, 737K whitelist, max_d 1): the shipped open-addressing pair-key tables
# ("after"), the CSR per-block buckets sized by distinct block values ("csr"), and with
# SCT_NEAREST_LOAD=1000000 the CSR buckets at the round-1 sizing of ~nw/2 ("before").
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python3 tools/bench_paths.py --reads 0 --stream-reads 0 --fastq-records 0 --skip-allpairs5 --queries 100000000"
for variant in after csr before; do
  D=gpurun_out/profn_$variant
  mkdir -p $D
  unset SCT_NEAREST_LOAD SCT_NEAREST_SCHEME
  if [ $variant = before ]; then export SCT_NEAREST_LOAD=1000000 SCT_NEAREST_SCHEME=csr; fi
  if [ $variant = csr ]; then export SCT_NEAREST_SCHEME=csr; fi
  timeout -k 10 240 $B > $D/bench.json 2> $D/bench.err || exit 3
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $B > $D/trace.log 2>&1 || exit 3
  i=0
  for pmc in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc -d $D/pmc$i -o run --output-format csv -- $B > $D/pmc$i.log 2>&1 || { echo "pmc pass $i failed ($variant)"; }
  done
done
exit 0
