# config 5 from disk: merge parity tests, then the load of the 1B cloud's cell
# files and the merge build (scripts/merge_disk_bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-merge or split or dist}" > gpurun_out/t_md.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_md.log; exit 1; }
tail -1 gpurun_out/t_md.log
PCC_VERBOSE=1 timeout -k 10 400 python -u scripts/merge_disk_bench.py > gpurun_out/merge_disk.json 2> gpurun_out/merge_disk.err || { echo "merge disk bench failed"; tail -5 gpurun_out/merge_disk.err; exit 3; }
grep "open:" gpurun_out/merge_disk.err
cat gpurun_out/merge_disk.json
