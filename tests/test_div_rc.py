"""The slab kernels' exact-reciprocal quotient (engine.hip div_rc, Markstein's
one-step correction) equals IEEE f32 division on the operand/divisor ranges the
kernels keep to (tests/div_rc_check.c, 2e7 random cases incl. near-integer
quotients and the /3 of hex.rs:76-78).  A C restatement of the same f32/FMA
sequence; the GPU parity suite checks the kernels themselves."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def _exe(tmp_path):
    exe = str(tmp_path / "div_rc_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "div_rc_check.c"), "-lm"],
                   check=True)
    return exe


def test_div_rc_exhaustive_default_divisors(tmp_path):
    r = subprocess.run([_exe(tmp_path), "exhaustive"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "exhaustive mismatches=0" in r.stdout and r.stdout.count("numerator mantissas checked") == 5


def test_div_rc_matches_ieee_division(tmp_path):
    exe = _exe(tmp_path)
    for seed in (1, 2):
        r = subprocess.run([exe, "10000000", str(seed)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout
        assert "mismatches=0" in r.stdout
