mkdir -p gpurun_out
for a in 0 1 2 3 4; do
  PCC_ABLATE=$a timeout -k 10 200 python bench.py --points 200000000 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/abl_$a.json 2>gpurun_out/abl_$a.err || exit 1
done
