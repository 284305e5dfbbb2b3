#!/bin/bash
# mode 3 against mode 6 (recomputed Ap) at 256^3, interleaved, the driver's
# bench command shape with a longer window; each run its own process
set -o pipefail
out=${1:-gpurun_out/ab6}
mkdir -p $out
for rep in 1 2; do
  for m in 3 6; do
    timeout -k 10 240 python -u bench.py --mode $m --steps 400 --warmup 20 --no-cpu --no-general \
      --no-traffic --profile-steps 100 > $out/mode${m}_rep${rep}.json 2> $out/mode${m}_rep${rep}.err || exit 1
  done
done
