export CFGS="|--steps 400 --warmup 10 --no-general --no-traffic;CGX_LIB=build_ab/apnt/libcgx.so|--steps 400 --warmup 10 --no-general --no-traffic;|--workload p3d_512 --steps 40 --warmup 4 --no-general --no-traffic;CGX_LIB=build_ab/apnt/libcgx.so|--workload p3d_512 --steps 40 --warmup 4 --no-general --no-traffic"
export ROUNDS=2
bash tools/gpu_ab_cfg.sh abapnt
