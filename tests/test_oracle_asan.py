"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY
§5: sanitizers on the C restatement): oracle/asan_driver.c calls every entry
point on small inputs (rule games, auto-reset, a caller's legal and illegal
moves, masks, encoders, canonical keys, scoring, greedy moves, searches);
any report aborts the run.  The sanitized build must also compute what the
optimised oracle computes (the driver's checksum, built twice)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _build_and_run(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = ["gcc", "-std=c11", "-fopenmp", "-ffp-contract=off", *flags, "-I", ORACLE, "-o", exe,
           os.path.join(ORACLE, "asan_driver.c"), os.path.join(ORACLE, "hz_oracle.c"), "-lm"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "ERROR: AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    line = [s for s in p.stdout.splitlines() if s.startswith("asan driver ok")]
    assert line, p.stdout[-2000:]
    return line[0]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan(tmp_path):
    san = _build_and_run(tmp_path, ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                                    "-fno-sanitize-recover=all"], "asan_driver")
    opt = _build_and_run(tmp_path, ["-O2"], "opt_driver")
    assert san == opt
