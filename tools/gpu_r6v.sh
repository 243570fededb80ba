# Round 6: A/B of the count buffers zeroed on the tail stream (new) against HEAD's module (old),
# emulated W = 8 and W = 4 rank shares, side build, interleaved on one box
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6v
mkdir -p $P
export TMPDIR=/tmp
for i in 1 2 3; do
  for w in 8 4; do
    for v in new old; do
      timeout -k 10 300 python3 tools/w8_share.py $w 60 side $v > $P/w${w}_${v}_$i.json 2> $P/err || { tail $P/err; exit 3; }
      echo $w $v $(cat $P/w${w}_${v}_$i.json)
    done
  done
done
echo done
