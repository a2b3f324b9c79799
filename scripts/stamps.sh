# diagnostic: per-phase cycle stamps of the slab kernels (stamped build, never the product)
mkdir -p gpurun_out
PCC_LIB=$PWD/point-cloud_amd/build/stamps/libpcconv.so timeout -k 10 300 python bench.py --points ${STAMP_POINTS:-1000000000} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/stamps.json 2> gpurun_out/stamps.err
