# round-2 final measurements: config 4 default bench, config 3, config 5 merge, configs 1-2, sharded N=1, CLI e2e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/fin_default.json 2> gpurun_out/fin_default.err || { echo "default bench failed"; exit 1; }
echo default-ok
timeout -k 10 300 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 20000000 > gpurun_out/fin_c3.json 2> gpurun_out/fin_c3.err || { echo "c3 failed"; exit 2; }
echo c3-ok
timeout -k 10 400 python bench.py --points 100000000 --seed 5 --merge-prior 1000000000 > gpurun_out/fin_c5.json 2> gpurun_out/fin_c5.err || { echo "c5 failed"; exit 3; }
echo c5-ok
timeout -k 10 300 python scripts/config12_bench.py > gpurun_out/fin_c12.json 2> gpurun_out/fin_c12.err || { echo "c12 failed"; exit 4; }
echo c12-ok
PCC_BENCH_SHARDED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/fin_sharded1.json 2> gpurun_out/fin_sharded1.err || { echo "sharded failed"; exit 5; }
echo sharded-ok
timeout -k 10 300 python scripts/cli_e2e.py > gpurun_out/fin_cli.json 2> gpurun_out/fin_cli.err || { echo "cli failed"; exit 6; }
echo cli-ok
