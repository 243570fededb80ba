# SPECTRAL count time vs chunk size with the seed grid sized per chunk (walks per workgroup
# = min(16, walks / 64)), and per-kernel times; then seed walks per workgroup at small chunks
# (ablation library, SCT_SEED_WALKS).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/chunk_sweep2.jsonl
for c in 4096 8192 16384 32768 65536 4096 8192 16384 32768 65536; do
  r=$(SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
  k=$(SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
  echo "{\"chunk\": $c, \"count\": $r, \"kernels\": $k}" >> $O
done
for c in 8192 16384; do
  for w in 1 2 4 8; do
    r=$(SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so SCT_SEED_WALKS=$w SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"chunk\": $c, \"walks\": $w, \"count\": $r}" >> $O
  done
done
exit 0
