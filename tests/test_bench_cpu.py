"""bench.py's JSON line (the driver's contract): the keys, types and the two
extra objects, built by record() from synthetic stage numbers (no GPU)."""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(HERE, "..", "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _line(world):
    b = _bench()
    sys.argv = ["bench.py"]
    args = b.parse()
    k = {"dense_arrivals": 2_780_291_831, "small_arrivals": 209_765_606, "dense_launches": 3, "small_launches": 4,
         "level0_ms": 16.5, "dense_ms": 33.5, "small_ms": 3.4, "bucket_ms": 1.3, "next_ms": 0.4}
    return args, b.record(args, world, 55.5, 4, 4680, 898_651, 2_990_057_437, k, 33.5,
                          "single GPU" if world == 1 else f"level-0 cell sharding over {world} ranks")


def test_record_has_the_contract_keys():
    args, r = _line(1)
    for key, typ in [("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int),
                     ("warmup", int), ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str),
                     ("dtype", str), ("data", str), ("config", dict), ("roofline", dict)]:
        assert isinstance(r[key], typ), key
    assert "vs_baseline" in r and r["vs_baseline"] is None
    assert r["value"] == args.points / 0.0555
    assert r["scaling"] in ("weak", "strong") and r["higher_is_better"] is True
    assert "workload" in r["config"] and "model" not in r["config"]
    rf = r["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in rf, key
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s"
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    assert abs(rf["achieved"] - 32.0 * 2_780_291_831 / 0.0335 / 1e9) < 1e-6


def test_record_for_several_ranks():
    _, r = _line(8)
    assert r["n_gpus"] == 8
    assert r["value"] > 0
