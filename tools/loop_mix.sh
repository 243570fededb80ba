#!/bin/bash
# usage: tools/loop_mix.sh <file.s> <kernel-substring>: instruction mix of the hot loop
# (from the first ds_read_b128 to the next backward s_cbranch) of the named kernel.
f=$1; k=$2
L=$(grep -n "^_Z.*${k}.*:" $f | head -1 | cut -d: -f1)
awk -v L=$L 'NR>=L' $f | awk '/s_endpgm/{print; exit} {print}' > /tmp/_k.s
a=$(grep -n "ds_read_b128" /tmp/_k.s | head -1 | cut -d: -f1)
b=$(grep -n "s_cbranch_scc\|s_cbranch_vccnz\|s_cbranch_vccz" /tmp/_k.s | awk -F: -v a=$a '$1>a{print $1; exit}')
sed -n "${a},${b}p" /tmp/_k.s | grep -E "^\s+(v_|s_|ds_|global_)" | awk '{print $1}' | sort | uniq -c | sort -rn
echo "VALU total: $(sed -n "${a},${b}p" /tmp/_k.s | grep -cE '^\s+v_')  lines $a-$b"
