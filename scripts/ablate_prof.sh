# per-dispatch timings of the slab kernels under timing-only ablations (PCC_ABLATE)
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for a in 0 1 4; do
  PCC_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/ablp_$a -o run --output-format csv -- python $R/bench.py --points 200000000 --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/ablp_$a.log 2>&1 || exit 1
done
