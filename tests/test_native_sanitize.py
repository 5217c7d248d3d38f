"""The native MCTS engine (csrc/az_mcts.cpp: pointer-linked trees, per-slot state machines,
OpenMP collect/feed) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 race /
sanitizer row): tests/native/mcts_sanitize.cpp drives every include/az_mcts.h entry point --
episode and search mode, Connect4 7x7 / 5x5 and TicTacToe 3x3 / 4x4, GNN on and off, 3 host
threads, failed batches and aborted episodes, the error paths -- and any memory or UB error
aborts it.  Host code only (GPU sanitizers are not available on the pool)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_engine_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "mcts_sanitize")
    src = [os.path.join(ROOT, "tests", "native", "mcts_sanitize.cpp"),
           os.path.join(ROOT, "alphazero-gnn_amd", "csrc", "az_mcts.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fopenmp",
           "-ffp-contract=off", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"] + \
        src + ["-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="3")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "mcts_sanitize: ok" in r.stdout, \
        (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
