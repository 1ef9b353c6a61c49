set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r06j; mkdir -p $OUT
for rep in 1 2 3; do
  for v in cur prev; do
    if [ $v = cur ]; then CB=./tools/coalesce_bench; SK=./tools/seek_latency; else CB=./tools/abprev/coalesce_bench; SK=./tools/abprev/seek_latency; fi
    for sz in 65536 1048576; do
      echo "{\"v\": \"$v\", \"rep\": $rep, \"size\": $sz, \"out\": $(timeout -k 5 120 $CB 16 400 $sz | tail -1)}" >> $OUT/coalesce.jsonl || exit 1
    done
    echo "{\"v\": \"$v\", \"rep\": $rep, \"out\": $(timeout -k 5 120 $SK --mib 256 --reads 64000 --len 4096 --threads 16 | tail -1)}" >> $OUT/seek16.jsonl || exit 1
  done
done
cat $OUT/coalesce.jsonl | cut -c1-300
cat $OUT/seek16.jsonl | cut -c1-300
