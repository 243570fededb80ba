#!/bin/bash
# FASTQ range kernel at 8 waves per SIMD (timing-only variant, terminator list capped) vs the default,
# bench.py path_fastq in separate processes, interleaved
set -u
P=gpurun_out/r6z
mkdir -p $P
for r in 1 2 3; do
  for v in main fqocc; do
    lib=""; [ $v != main ] && lib=$PWD/sctools_amd/libsctools_hip_$v.so
    SCTOOLS_HIP_LIB=$lib timeout -k 10 120 python3 tools/run_paths.py fastq > $P/$v.$r.json 2> $P/$v.$r.err || exit 3
    python3 -c "import json; d=json.load(open('$P/$v.$r.json'))['fastq']; print('$v', $r, d['ms'], d['check'])"
  done
done
