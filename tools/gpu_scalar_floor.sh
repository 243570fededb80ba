#!/bin/bash
# (historical: the variant libraries it compares were built from round-6 intermediate trees with
# tools/build_variant_lib.sh; their ablation macros are no longer in the sources -- results under
# profiles/scalar_floor_r06/)
# scalar server A/B: its GPU tests, the mailbox floors and the library's C call per server variant
# (tools/scalar_floor_probe.hip incl. the host-work sweep, tools/build_variant_lib.sh), and the
# Python drop-in calls (tools/scalar_latency.py)
set -u
P=gpurun_out/r6s
mkdir -p $P
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scalar_server.py \
  > $P/pytest_scalar.log 2>&1 || { tail -30 $P/pytest_scalar.log; exit 3; }
tail -1 $P/pytest_scalar.log
for r in 1 2; do
  for v in main nostagger oldsrv; do
    lib=$PWD/sctools_amd/libsctools_hip.so; [ $v != main ] && lib=$PWD/sctools_amd/libsctools_hip_$v.so
    SCTOOLS_HIP_LIB=$lib timeout -k 10 120 tools/scalar_floor_probe > $P/floor.$v.$r.jsonl 2> $P/floor.$v.$r.err || exit 3
    grep '"c_call"' $P/floor.$v.$r.jsonl | head -1 || exit 3
  done
done
for r in 1 2; do
  for v in main nostagger; do
    lib=""; [ $v != main ] && lib=$PWD/sctools_amd/libsctools_hip_$v.so
    SCTOOLS_HIP_LIB=$lib timeout -k 10 120 python3 tools/scalar_latency.py > $P/py.$v.$r.json 2> $P/py.$v.$r.err || exit 3
    echo "$v $r $(cat $P/py.$v.$r.json)"
  done
done
