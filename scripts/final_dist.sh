# final check of the sharded path: GPU dist/split/merge/input tests, then the torchrun N=1 sharded bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dist or split or merge or inputs or gloo" > gpurun_out/t_fd.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_fd.log; exit 1; }
tail -1 gpurun_out/t_fd.log
PCC_BENCH_SHARDED=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/fin_sharded1.json 2> gpurun_out/fin_sharded1.err || { echo "sharded failed"; tail gpurun_out/fin_sharded1.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/fin_sharded1.json'));print(round(d['ms_per_step'],2), d.get('stage_ms'))"
