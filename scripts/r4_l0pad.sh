# level-0 pass 1 into a padded arena (runs at multiples of 64 points, k_l0_tile6
# (round 4: the padded variant was reverted after this A/B)
# PAD) against the in-place layout (PCC_L0_NO_PAD=1): parity, the 1B bench in
# both forms, and the HBM counters of level 0 in both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/pad
timeout -k 10 1100 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py tests/test_split_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pad/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pad/tests.log; exit 1; }
tail -1 gpurun_out/pad/tests.log
for round in 1 2; do
for v in pad nopad; do
  env $( [ $v = nopad ] && echo PCC_L0_NO_PAD=1 ) timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/pad/$v.$round.json 2> gpurun_out/pad/$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/pad/$v.$round.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/pad/$v.$round.json'));print('$v', $round, round(d['ms_per_step'],2), {k:round(v,3) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
cd /tmp && export TMPDIR=/tmp
for v in pad nopad; do
  for c in FETCH_SIZE WRITE_SIZE; do
    env $( [ $v = nopad ] && echo PCC_L0_NO_PAD=1 ) timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/pad/pmc_${v}_$c -o p -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 > /dev/null 2>&1 || { echo "pmc $v $c failed"; exit 3; }
  done
done
cd $R && python3 - <<'PY'
import csv
for v in ("pad", "nopad"):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for r in csv.DictReader(open(f"gpurun_out/pad/pmc_{v}_{c}/p_counter_collection.csv")):
            if r["Counter_Name"] != c: continue
            k = r["Kernel_Name"].split("(")[0]
            if "k_l0_tile6" in k or "k_l0_down5g" in k:
                tot.setdefault(k, {}).setdefault(c, 0.0)
                tot[k][c] += float(r["Counter_Value"]) * 1024
    for k, d in tot.items():
        print(v, k, {c: round(x / 1e9, 2) for c, x in d.items()}, "GB; corrected", round((2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) / 1e9, 2))
PY
