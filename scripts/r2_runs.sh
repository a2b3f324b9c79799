set -o pipefail
mkdir -p gpurun_out
( timeout -k 10 900 python bench.py --cpu-full --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/cpufull.json 2> gpurun_out/cpufull.err ) &
CPID=$!
timeout -k 10 300 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 20000000 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
echo c3 done
timeout -k 10 400 python bench.py --points 100000000 --seed 5 --merge-prior 1000000000 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 2
echo c5 done
while kill -0 $CPID 2>/dev/null; do echo waiting-cpu-full; sleep 30; done
wait $CPID; echo cpufull rc=$?
