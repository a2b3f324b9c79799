# round-1 final evidence: parity suite, bench lines (config 4 with CPU baseline, config-3 shape,
# config 5), the sharded path through torchrun + RCCL at N=1, kernel trace + PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/fin_c4.json 2> gpurun_out/fin_c4.err || { echo "bench c4 failed"; exit 2; }
timeout -k 10 300 python bench.py --points 100000000 --kind 1 --seed 3 --cpu-sample 10000000 > gpurun_out/fin_c3.json 2> gpurun_out/fin_c3.err || { echo "bench c3 failed"; exit 3; }
timeout -k 10 600 python -u bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 2000000 > gpurun_out/fin_c5.json 2> gpurun_out/fin_c5.err || { echo "bench c5 failed"; exit 4; }
PCC_BENCH_SHARDED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 3 --warmup 1 > gpurun_out/fin_sharded1.json 2> gpurun_out/fin_sharded1.err || { echo "sharded bench failed"; tail -20 gpurun_out/fin_sharded1.err; exit 5; }
bash scripts/pmc.sh || exit 6
echo final-ok
