# Round 6: the pipelined step's new order (next build before this tail) vs the previous revision
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6r2
mkdir -p $P
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in new old; do
    timeout -k 10 300 python3 tools/w8_share.py 8 40 side $v > $P/w8_${v}_$i.json 2> $P/err || { tail $P/err; exit 3; }
    echo $v $(cat $P/w8_${v}_$i.json)
  done
done
echo done
