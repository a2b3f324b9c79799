# round 5: rehearsal of bench.py's N > 1 path (main_sharded: barriers, max over ranks, the one JSON
# line) with 2 and 4 ranks on ONE GPU over gloo (RCCL refuses two ranks on one device); 200M points
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD} && mkdir -p gpurun_out
for n in 2 4; do
  PCC_BENCH_BACKEND=gloo GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --points 200000000 \
    > gpurun_out/r5_bench_n$n.json 2> gpurun_out/r5_bench_n$n.err || { echo "n=$n failed"; tail -20 gpurun_out/r5_bench_n$n.err; exit 2; }
  tail -1 gpurun_out/r5_bench_n$n.json | cut -c1-400
done
