# SURVEY 8d mode (A) CPU baseline (LRU-100 + .bin write-back) beside the GPU line, configs 1-5:
# full runs for configs 1-2, 60 s prefixes for 3-5 (bench.py --cpu-mode-a)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/mode_a
B="python3 -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --cpu-mode-a"
timeout -k 10 200 $B --points 100000 --seed 1 > gpurun_out/mode_a/c1.json 2> gpurun_out/mode_a/c1.err || exit 1
echo c1
timeout -k 10 300 $B --points 10000000 --seed 2 > gpurun_out/mode_a/c2.json 2> gpurun_out/mode_a/c2.err || exit 2
echo c2
timeout -k 10 200 $B --points 100000000 --seed 3 --kind 2 > gpurun_out/mode_a/c3.json 2> gpurun_out/mode_a/c3.err || exit 3
echo c3
timeout -k 10 250 $B --points 1000000000 --seed 4 > gpurun_out/mode_a/c4.json 2> gpurun_out/mode_a/c4.err || exit 4
echo c4
timeout -k 10 300 $B --points 100000000 --seed 5 --merge-prior 1000000000 > gpurun_out/mode_a/c5.json 2> gpurun_out/mode_a/c5.err || exit 5
echo c5
