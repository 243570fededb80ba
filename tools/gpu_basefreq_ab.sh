# Round 5: base_frequency 32-bit form (base_frequency16_kernel, L <= 16) vs the 64-bit kernel
# (base library built by tools/build_base_lib.sh), rounds of 15 codes per lane 1 / 2 / 3 (SCT_BF_ROUNDS, read by the variant build of that A/B only), the
# whitelist path's base_frequency_ms (config 5's 3,686,400 16-bp codes), three interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/bf
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k base_frequency > $P/pytest.log 2>&1
rc=$?
tail -2 $P/pytest.log
[ $rc -eq 0 ] || exit 3
ext='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])["whitelist"]["base_frequency"]; print(json.dumps({"variant": sys.argv[1], "base_frequency_ms": d["ms"], "check": d["check"]["vs_oracle"]}))'
for r in 1 2 3; do
  SCTOOLS_HIP_LIB=sctools_amd/libsctools_hip_base.so timeout -k 10 120 python tools/run_paths.py whitelist 2>/dev/null | python -c "$ext" base >> $P/ab.jsonl || exit 3
  for R in 1 2 3; do
    SCT_BF_ROUNDS=$R timeout -k 10 120 python tools/run_paths.py whitelist 2>/dev/null | python -c "$ext" r$R >> $P/ab.jsonl || exit 3
  done
done
cat $P/ab.jsonl
