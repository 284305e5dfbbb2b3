set -o pipefail
OUT=gpurun_out/coopb1; mkdir -p $OUT
for w in p2d_128 g3_standin; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 2000 --warmup 50 --no-traffic > $OUT/bench_$w.log 2>&1 || { echo "BENCH $w FAIL"; tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-1500
done
