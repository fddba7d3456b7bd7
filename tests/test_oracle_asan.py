"""The C oracle under AddressSanitizer + UBSan (SURVEY.md §5 "Race detection / sanitizers"):
`make -C oracle asan` builds oracle/asan_check.c with dsp_oracle.c into oracle/_asan/ and the
driver runs every oracle entry point on edge-case clips (empty, 1 sample, < 1 frame, 1 s, 1.5 s,
silence, DC, clipping; 5 frame sizes x 3 windows x VAD on/off; the 4-thread batch entry against
the per-clip one) and the KNN at D = 15 / 40, k = 3 / 5 / 21.  Clean = exit 0, no report."""
import os
import subprocess

from conftest import REPO


def test_oracle_clean_under_asan():
    ora = os.path.join(REPO, "oracle")
    subprocess.run(["make", "-s", "-C", ora, "asan"], check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ora, "_asan", "asan_check")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert "clip mismatches 0, knn violations 0" in r.stdout
