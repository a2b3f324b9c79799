# round-3 final rehearsal on the committed tree: the GPU suite, smoke, the
# default bench (the driver's command), configs 3 / 5 / 1-2, the sharded path at
# N = 1 (torchrun, RCCL) and the CLI end to end
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/fin_pytest.log 2>&1 || { echo "gpu suite failed"; tail -20 gpurun_out/fin_pytest.log; exit 1; }
echo suite-ok
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/fin_smoke.log; exit 2; }
echo smoke-ok
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/fin_default.json 2> gpurun_out/fin_default.err || { echo "default bench failed"; exit 3; }
echo default-ok
timeout -k 10 300 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 20000000 > gpurun_out/fin_c3.json 2> gpurun_out/fin_c3.err || { echo "c3 failed"; exit 4; }
echo c3-ok
timeout -k 10 400 python bench.py --points 100000000 --seed 5 --merge-prior 1000000000 > gpurun_out/fin_c5.json 2> gpurun_out/fin_c5.err || { echo "c5 failed"; exit 5; }
echo c5-ok
timeout -k 10 300 python scripts/config12_bench.py > gpurun_out/fin_c12.json 2> gpurun_out/fin_c12.err || { echo "c12 failed"; exit 6; }
echo c12-ok
PCC_BENCH_SHARDED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/fin_sharded1.json 2> gpurun_out/fin_sharded1.err || { echo "sharded failed"; exit 7; }
echo sharded-ok
timeout -k 10 300 python scripts/cli_e2e.py > gpurun_out/fin_cli.json 2> gpurun_out/fin_cli.err || { echo "cli failed"; exit 8; }
echo cli-ok
