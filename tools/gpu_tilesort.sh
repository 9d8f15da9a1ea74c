#!/bin/bash
# node order inside a tile's bucket (GTF_TILE_SORT 0: node order, 1: exact slot count up)
# and the tile size (GTF_TILE)
set -o pipefail
O=gpurun_out/tilesort2
mkdir -p $O
for i in 1 2; do
  for v in "4096 0" "4096 1" "2048 1" "1024 1" "2048 0" "8192 1"; do
    set -- $v
    GTF_TILE=$1 GTF_TILE_SORT=$2 timeout -k 10 120 python tools/pass_loop.py 150 >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
