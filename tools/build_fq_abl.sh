#!/bin/bash
# Timing-only ablation libraries of fastq_range_kernel (SCT_FQ_ABL = 1 no per-tile items, 2 name
# checks only, 3 no CB encode, 4 no terminator list, 5 per-line stores into an LDS sink): sctools_amd/libsctools_hip_fqabl<k>.so,
# loaded through SCTOOLS_HIP_LIB by tools/fastq_abl.py.  Wrong results by design.
set -eu
cd "$(dirname "$0")/../sctools_amd/csrc"
make -j8 >/dev/null
mkdir -p build_fqabl
OBJS=$(ls build/*.o | grep -v fastq.hip.o)
for k in ${KS:-1 2 3 4}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DSCT_FQ_ABL=$k \
    -c fastq.hip -o build_fqabl/fastq_$k.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $OBJS build_fqabl/fastq_$k.o -o ../libsctools_hip_fqabl$k.so
done
