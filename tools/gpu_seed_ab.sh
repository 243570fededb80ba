# SPECTRAL seed / layout variants: parity tests under each (SEEDS, env per entry "seed:ilv"),
# then seed / tile / count times.  AB list: entries "seed:ilv".
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in ${TESTS:-}; do
  sd=${e%%:*}; g=${e##*:}
  SCT_SPECTRAL_SEED=$sd SCT_SPECTRAL_ILV=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/seed_ab_${sd}_${g}_pytest.log 2>&1
  rc=$?; echo "$e pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
O=gpurun_out/seed_ab.jsonl
for rep in 1 2 3; do
  for e in ${AB:-walk:0}; do
    sd=${e%%:*}; g=${e##*:}
    r=$(SCT_SPECTRAL_SEED=$sd SCT_SPECTRAL_ILV=$g timeout -k 10 120 python3 tools/spectral_kernels.py 2 5) || exit $?
    t=$(SCT_SPECTRAL_SEED=$sd SCT_SPECTRAL_ILV=$g timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"seed\": \"$sd\", \"ilv\": \"$g\", \"k\": $r, \"count\": $t}" >> $O
  done
done
exit 0
