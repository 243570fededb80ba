# Same-box A/B of the scalar-call latency (tools/scalar_latency.py) between the HEAD library
# (sctools_amd/libsctools_hip_base.so, tools/build_base_lib.sh) and the working tree's, two rounds.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6i
mkdir -p $P
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=$PWD/sctools_amd/libsctools_hip_base.so
    SCTOOLS_HIP_LIB=$lib timeout -k 10 120 python3 tools/scalar_latency.py > $P/$v.$r.json 2> $P/$v.$r.err || exit 3
    echo "$v $r $(cat $P/$v.$r.json)"
  done
done
