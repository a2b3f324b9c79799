# diagnostic: level-0 binning time of the tile-shape variants (make -C point-cloud_amd l0var)
set -o pipefail
mkdir -p gpurun_out
for v in base 1024_3 1024_4 512_6 base 1024_3; do
  if [ $v = base ]; then L=$PWD/point-cloud_amd/build/libpcconv.so; else L=$PWD/point-cloud_amd/build/l0_$v/libpcconv.so; fi
  PCC_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/l0_$v.json 2> gpurun_out/l0_$v.err || { echo "variant $v failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/l0_$v.json'));print('$v', round(d['ms_per_step'],2), round(d['stage_ms']['level0_ms'],2))"
done
