# Round 5, first box: the whole GPU suite, then the config-5 all-pairs profile VERDICT r4 #2
# asks for (rocprofv3 kernel trace + PMC passes of seed16_sm_kernel / tile16_kernel, each pass
# its own run), then one default bench line.  Output under gpurun_out/prof5/;
# summarise with: python tools/summarize_profile.py --round r05 --src gpurun_out/prof5
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/prof5
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -5 $P/pytest_gpu.log
# 0 = green, 1 = a test failed (no fault): the profiles still run; anything else ends the call
[ $rc -le 1 ] || exit 3
C="python3 tools/run_paths.py config5_allpairs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/s5trace -o run --output-format csv -- $C > $P/s5trace.log 2>&1 || exit 3
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc -d $P/s5pmc$i -o run --output-format csv -- $C > $P/s5pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 3; }
done
timeout -k 10 400 python3 bench.py > $P/bench.log 2>&1 || exit 3
echo done
