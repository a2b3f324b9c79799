"""Diagnostic: run the randomised cases (tests/fuzz_cases.py) `reps` times in one
process on the GPU against the oracle; for a cell that differs print, for the
first differing kept list or grid, both sides as input indices (= keys of a
plain build).  Usage: fuzz_diag.py REPS [first last] [nf]"""
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import numpy as np  # noqa: E402

import canon  # noqa: E402
from fuzz_cases import mid_case  # noqa: E402
from gpu_util import run_gpu, run_oracle  # noqa: E402

if os.environ.get("FUZZ_TORCH"):   # initialise torch's HIP runtime first, as tests/conftest.py does
    import torch
    torch.cuda.init()
reps = int(sys.argv[1])
lo, hi = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (0, 48)
nonfinite = sys.argv[-1] == "nf"
oracle = {}
bad = 0
for rep in range(reps):
    for seed in range(lo, hi):
        files, cfg, batch, kind = mid_case(seed, nonfinite=nonfinite)
        if seed not in oracle:
            to = tempfile.mkdtemp(dir="/dev/shm")
            assert run_oracle(to, files, cfg=cfg, batch=batch)[0] == 0
            oracle[seed] = canon.read_dir_fast(to)[0]
            shutil.rmtree(to)
        co = oracle[seed]
        tg = tempfile.mkdtemp(dir="/dev/shm")
        st = run_gpu(tg, files, cfg=cfg, batch=batch)
        cg = canon.read_dir_fast(tg)[0]
        shutil.rmtree(tg)
        d = canon.diff_fast(co, cg)
        if not d:
            continue
        bad += 1
        print("rep", rep, "seed", seed, kind, cfg, batch, "levels", st["levels"], "fold", st.get("level0_fold"),
              "diffs", len(d), d[:2], flush=True)
        allp = np.concatenate(files)
        index = {}
        for i in range(len(allp)):
            index.setdefault(bytes(allp[i].tobytes()), i)
        for k in sorted(set(co) & set(cg)):
            if co[k] == cg[k]:
                continue
            if co[k][1] != cg[k][1]:
                ga = sorted(index.get(bytes(co[k][1][j:j + 16]), -1) for j in range(0, len(co[k][1]), 16))
                gb = sorted(index.get(bytes(cg[k][1][j:j + 16]), -1) for j in range(0, len(cg[k][1]), 16))
                print(" cell", k, "grid only oracle", sorted(set(ga) - set(gb))[:16], "only gpu",
                      sorted(set(gb) - set(ga))[:16], flush=True)
                for i in sorted(set(ga) ^ set(gb))[:8]:
                    print("   point", i, allp[i], flush=True)
            for (ia, la), (ib, lb) in zip(co[k][2], cg[k][2]):
                if la != lb:
                    ka = [index.get(bytes(la[j:j + 16]), -1) for j in range(0, len(la or b""), 16)]
                    kb = [index.get(bytes(lb[j:j + 16]), -1) for j in range(0, len(lb or b""), 16)]
                    print(" cell", k, "child", ia, "n", len(ka), "same set", sorted(ka) == sorted(kb))
                    print("  oracle", ka[:48])
                    print("  gpu   ", kb[:48], flush=True)
                    break
            break
print("mismatching runs:", bad)
