#!/bin/bash
# The round's GPU record: the gpu test suite (as the driver runs it), smoke, the
# driver's bench command, rocprofv3 --kernel-trace --stats of that same
# command, FETCH_SIZE / WRITE_SIZE PMC passes (separate runs), the per-config
# lines. Stops at the first failing GPU step. Outputs in gpurun_out/$TAG.
#   tools/gpu_record.sh TAG [quick|full] [noconfigs]   (quick: skip pytest; noconfigs:
#   stop after the PMC passes)
set -o pipefail
TAG=${1:-rec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "quick" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
T0=$SECONDS; timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_driver.log; exit 1; }
echo "bench wall $((SECONDS-T0)) s"; tail -1 $OUT/bench_driver.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_prof.log; exit 1; }
tail -1 $OUT/bench_prof.log | cut -c1-200
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --no-cpu --no-general --steps 10 --warmup 2 --profile-steps 0 > $OUT/pmc_$C.log 2>&1 || { echo "PMC $C FAIL"; tail -20 $OUT/pmc_$C.log; exit 1; }
  echo "pmc $C ok"
done
[ "$3" = "noconfigs" ] && exit 0
timeout -k 10 600 python tools/configs_bench.py > $OUT/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -20 $OUT/configs.log; exit 1; }
cut -c1-240 $OUT/configs.log
timeout -k 10 400 bash tools/gpu_slab.sh $TAG/slab > $OUT/slab_all.log 2>&1 || { echo SLAB_FAIL; tail -20 $OUT/slab_all.log; exit 1; }
cat $OUT/slab_all.log
